"""Explicit, opt-in access to the reference's own modules for the parts of its API this tier
does not rebuild (other tasks' loaders, evaluation helpers outside the EA path).

Nothing is loaded unless the environment variable GNNEA_UPSTREAM names the reference checkout
(the directory holding its ``utils/`` and ``SinkhornOT/``); no search of sys.path happens.  A
drop-in module calls ``merge(globals(), relpath, keep)`` once at import: the reference module
at ``$GNNEA_UPSTREAM/relpath`` is executed and its names that this module does not define are
added, and (for ``export``) this module's rebuilt functions are installed into it.
"""
import importlib.util
import os


def load(relpath, modname):
    """The reference module at $GNNEA_UPSTREAM/relpath, or None when GNNEA_UPSTREAM is unset."""
    root = os.environ.get("GNNEA_UPSTREAM")
    if not root:
        return None
    path = os.path.join(os.path.abspath(root), relpath)
    if not os.path.isfile(path):
        raise FileNotFoundError("GNNEA_UPSTREAM=%s has no %s" % (root, relpath))
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def merge(namespace, relpath, modname, export=()):
    """Add the reference module's missing names to ``namespace``; install ``export`` (names of
    rebuilt functions) into the reference module.  Returns the module or None."""
    mod = load(relpath, modname)
    if mod is None:
        return None
    for k, v in vars(mod).items():
        if not k.startswith("__"):
            namespace.setdefault(k, v)
    for k in export:
        setattr(mod, k, namespace[k])
    return mod

# Drop-in package: modules present here shadow the reference's same-named modules; any other
# module of the package (e.g. the reference's own loaders) is still found further down sys.path.
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)

"""Symbolise the PCs of a glog-style crash trace ("@ 0x... (unknown)") against a /proc/<pid>/maps
snapshot of the same process (bench.py writes one when GNNEA_EXIT_MAPS names a file).

    python tools/symbolize_crash.py LOG MAPS

Prints, per frame: address, mapped file, address relative to the file's load base, and llvm-symbolizer's function / source
when the file is present on this machine (the image is the same here and on the GPU box).
"""
import os
import re
import subprocess
import sys

SYMBOLIZER = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def load_maps(path):
    regions = []
    for line in open(path):
        parts = line.split()
        if len(parts) < 6 or not parts[5].startswith("/"):
            continue
        lo, hi = (int(x, 16) for x in parts[0].split("-"))
        regions.append((lo, hi, int(parts[2], 16), parts[5], parts[1]))
    return regions


def frames(log):
    out = []
    for line in open(log, errors="replace"):
        m = re.search(r"@\s+(0x[0-9a-f]+)", line)
        if m and ("PC:" in line or line.strip().startswith("@")):
            out.append(int(m.group(1), 16))
    return out


def locate(addr, regions):
    """(file, address relative to the file's load base, permissions): the base is the start of
    the file's offset-0 mapping, so the result is the ELF virtual address symbolizers expect."""
    for lo, hi, off, path, perm in regions:
        if lo <= addr < hi:
            base = min((r[0] for r in regions if r[3] == path and r[2] == 0), default=lo - off)
            return path, addr - base, perm
    return None, None, None


def main():
    log, maps = sys.argv[1], sys.argv[2]
    regions = load_maps(maps)
    for a in frames(log):
        path, off, perm = locate(a, regions)
        if path is None:
            print("0x%x  (not in a file mapping)" % a)
            continue
        sym = ""
        if os.path.exists(path) and os.path.exists(SYMBOLIZER):
            r = subprocess.run([SYMBOLIZER, "--obj=" + path, "--demangle", "--functions=linkage",
                                hex(off)], capture_output=True, text=True)
            sym = " | ".join(s for s in r.stdout.strip().splitlines() if s)
        print("0x%x  %s +0x%x [%s]  %s" % (a, path, off, perm, sym))


if __name__ == "__main__":
    main()

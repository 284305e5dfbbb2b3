#!/usr/bin/env python3
"""A/B harness: run a script against another build of libcgx.

  python tools/ab_lib.py /tmp/x/libcgx.so tools/slab_bench.py [args...]

Builds for an A/B come from `make -C conjugategradient_amd/csrc OUT=/tmp/x/libcgx.so
OBJDIR=/tmp/x EXTRA=-D...`. The product loader (conjugategradient_amd/_native.py)
always loads the in-tree library; this harness points it at the given file
before the script imports anything, and leaves unbound the entry points an
older build lacks. Child processes the script starts (torch.distributed.run
ranks) inherit the choice through $CGX_AB_LIB, read only here and by
tools/ab_site/sitecustomize.py.
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def use(path: str) -> None:
    sys.path.insert(0, ROOT)
    import conjugategradient_amd._native as N

    N.LIB_PATH = os.path.abspath(path)
    N._AB_BUILD = True


def main() -> None:
    if len(sys.argv) < 3:
        raise SystemExit(__doc__)
    lib, script = sys.argv[1], sys.argv[2]
    use(lib)
    os.environ["CGX_AB_LIB"] = os.path.abspath(lib)
    site = os.path.join(ROOT, "tools", "ab_site")
    os.environ["PYTHONPATH"] = site + os.pathsep + os.environ.get("PYTHONPATH", "")
    sys.argv = [script] + sys.argv[3:]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()

"""Child processes of tools/ab_lib.py (e.g. torch.distributed.run ranks) load
the A/B build named by $CGX_AB_LIB; only that harness puts this directory on
PYTHONPATH."""
import os

if os.environ.get("CGX_AB_LIB"):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import conjugategradient_amd._native as _N

    _N.LIB_PATH = os.environ["CGX_AB_LIB"]
    _N._AB_BUILD = True

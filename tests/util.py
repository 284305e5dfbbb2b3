"""Deterministic test inputs (numpy only; no reference code)."""
from __future__ import annotations

import numpy as np


# the G3_circuit stand-in generator lives with the bench workloads (one
# definition for tests, bench.py and tools/)
from conjugategradient_amd.workloads import coo_to_csr, irregular_spd  # noqa: E402,F401


def rel(a, b) -> float:
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(b))

"""Fingerprint of an input array stored in golden fixtures (the first 8 bytes
of its SHA-256 as an int64), shared by tools/c3_tie_fixture.py and the tests."""
import hashlib

import numpy as np


def fingerprint(arr) -> int:
    return int.from_bytes(hashlib.sha256(np.ascontiguousarray(arr).tobytes()).digest()[:8],
                          "little", signed=True)

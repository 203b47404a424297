"""CPU: the oracle is pinned by the reference's own unit tests (restated in
oracle/ref_tests.cc) and agrees with the committed golden fixtures."""
import os
import subprocess

import numpy as np

from conftest import ROOT, ensure_built


def test_oracle_passes_restated_reference_tests():
    ensure_built()
    exe = os.path.join(ROOT, "oracle", "_build", "ref_tests")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "failures: 0" in out.stdout


def test_oracle_levels_are_window_maxima(oracle):
    """Property (PrecomputationGridTest.CorrectValues): level d cell (x, y) is the
    max of the quantized level 0 over [x-(w-1), x] x [y-(w-1), y] (wide index)."""
    rng = np.random.RandomState(1)
    cells = rng.randint(0, 32768, size=(37, 29)).astype(np.uint16)
    om = oracle.fast2d((0.05, 1.0, 1.0), cells, 1.0, 0.5, 5)
    l0 = om.level(0).astype(int)
    for d in range(1, 5):
        w = 1 << d
        lv = om.level(d)
        ny, nx = l0.shape
        pad = np.zeros((ny + 2 * (w - 1), nx + 2 * (w - 1)), int)
        pad[w - 1:w - 1 + ny, w - 1:w - 1 + nx] = l0
        exp = np.zeros_like(lv, dtype=int)
        for y in range(lv.shape[0]):
            for x in range(lv.shape[1]):
                exp[y, x] = pad[y:y + w, x:x + w].max()
        np.testing.assert_array_equal(lv, exp)

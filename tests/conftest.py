"""Test configuration: the `gpu` marker, and loaders for the product package
(cartographer-1_amd/, importable only by path because of its name) and the
oracle (oracle/, test infrastructure)."""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_package():
    name = "cartographer_amd"
    if name in sys.modules:
        return sys.modules[name]
    pkg_dir = os.path.join(ROOT, "cartographer-1_amd")
    spec = importlib.util.spec_from_file_location(
        name, os.path.join(pkg_dir, "__init__.py"), submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def ensure_built():
    """Builds the product library, the synthetic-world library and the oracle
    if any is missing (cheap no-op when up to date)."""
    lib = os.path.join(ROOT, "cartographer-1_amd", "libcsm_amd.so")
    if not os.path.exists(lib) or not os.path.exists(
            os.path.join(ROOT, "cartographer-1_amd", "libcsm_synth.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "cartographer-1_amd", "csrc"),
                               "-j8"])
    if not os.path.exists(os.path.join(ROOT, "oracle", "_build", "liboracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-j8"])


@pytest.fixture(scope="session")
def csm():
    ensure_built()
    return load_package()


@pytest.fixture(scope="session")
def oracle():
    ensure_built()
    import oracle_lib
    return oracle_lib.Oracle()


def assert_search_ok(csm, status):
    """Every pair of a batch search was searched to the end: matched or no
    match. A negative status (an error, e.g. CSM_ERANGE) is never read as
    "no match" by a parity test."""
    import numpy as np
    st = np.asarray(status)
    bad = np.nonzero((st != csm.CSM_OK) & (st != csm.CSM_NO_MATCH))[0]
    assert len(bad) == 0, f"pairs {bad[:10].tolist()} returned error statuses {st[bad[:10]].tolist()}"

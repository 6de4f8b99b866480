import importlib.util
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


def load_cbg():
    """Import the product package (directory name has hyphens)."""
    name = "combblas_spmm_test_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(REPO, "combblas-spmm-test_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def cbg():
    return load_cbg()


@pytest.fixture(autouse=True)
def _release_device_cache(request):
    """after every GPU test: return libcbg's cached device memory to the driver, so
    that the multi-process tests that follow (several processes on the one GPU)
    find the HBM free (the scale-24 tile test alone caches hundreds of GB)"""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    mod = sys.modules.get("combblas_spmm_test_amd")
    if mod is not None and getattr(mod, "_lib", None) is not None:
        mod._lib.cbg_pool_trim()

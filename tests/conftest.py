import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtbe.so on the device)")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle.build import build_oracle
    return build_oracle()


@pytest.fixture(scope="session")
def engine_lib():
    """The HIP engine library, built in-tree if stale (hipcc cross-compiles without a GPU)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_tbe_build", os.path.join(ROOT, "distributedratelimiting.redis_amd", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.build_engine()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    torch.cuda.set_device(0)
    return torch.device("cuda:0")

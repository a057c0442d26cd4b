"""Test configuration.  `-m gpu` tests need an MI355X and call libpacmann.so
through its C ABI; everything else runs on CPU (oracle KATs, host logic,
ABI symbol checks, gloo multi-rank tests)."""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def ctx():
    import pacmann_amd as pm
    return pm.default_context()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    # hint-fold threads of the oracle's preprocessing (identical state for any
    # count); the GPU box gives a GPU 16 host cores
    O.set_prep_threads(min(16, os.cpu_count() or 1))
    return O


@pytest.fixture(scope="session")
def ctx_unfused():
    """A context that runs every batch-PIR step as the three separate kernels
    (PM_NO_FUSE=1, read at context creation) instead of the fused k_step."""
    import pacmann_amd as pm
    old = os.environ.get("PM_NO_FUSE")
    os.environ["PM_NO_FUSE"] = "1"
    try:
        return pm.Context(0)
    finally:
        if old is None:
            del os.environ["PM_NO_FUSE"]
        else:
            os.environ["PM_NO_FUSE"] = old


@pytest.fixture(params=["fused", "unfused"])
def step_ctx(request):
    """Both step paths: k_step (default) and the three-kernel fallback."""
    return request.getfixturevalue("ctx" if request.param == "fused" else "ctx_unfused")

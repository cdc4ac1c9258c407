import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Every GPU test (and every process a test spawns) runs the committed decode-kernel table
# (ops/tuned/decode_kernels_gfx950.json) instead of re-timing kernels at start-up: the kernel mix
# is then the same on every box, not the winner of a timing race on this one.
os.environ.setdefault("MPAMD_GEMM_AUTOTUNE", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP kernels")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU on this host")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _restore_gemm_modes():
    """Tests that force a decode-GEMM kernel (``ops.set_gemm_sk``) or policy put back whatever was
    set before them, so no test's outcome depends on which module ran first."""
    try:
        from src import ops
    except Exception:  # pragma: no cover - package import failure is reported by the tests
        yield
        return
    sk, policy = ops._GEMM_SK, ops.gemm_policy()
    yield
    ops.set_gemm_sk(sk)
    ops.set_gemm_policy(policy)

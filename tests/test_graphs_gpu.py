"""make_inference_graphed_callable (petals/llama/cuda_graphs.py:5-76) on a HIP graph."""
import pytest
import torch

from src import ops
from src.runtime.graphs import make_inference_graphed_callable

pytestmark = pytest.mark.gpu


def test_graphed_callable_replays_with_new_inputs():
    ops.require_native()
    w = torch.randn(128, 256, device="cuda", dtype=torch.bfloat16)

    def fn(x, pair):
        y = ops.rmsnorm(x, pair[0], 1e-5)
        return {"out": torch.relu(y @ w.t()), "sum": y.float().sum(-1) + pair[1]}

    x = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16)
    nw = torch.ones(256, device="cuda", dtype=torch.bfloat16)
    bias = torch.zeros(64, device="cuda")
    g = make_inference_graphed_callable(fn, (x, (nw, bias)))
    for seed in range(3):
        torch.manual_seed(seed)
        x2 = torch.randn(64, 256, device="cuda", dtype=torch.bfloat16)
        b2 = torch.randn(64, device="cuda")
        got = g(x2, (nw, b2))
        ref = fn(x2, (nw, b2))
        torch.testing.assert_close(got["out"], ref["out"])
        torch.testing.assert_close(got["sum"], ref["sum"])
    with pytest.raises(ValueError):
        g(x2)

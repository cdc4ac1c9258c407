"""``runtime.graphs.make_inference_graphed_callable`` (upstream petals/llama/cuda_graphs.py:5-76):
CPU pass-through, and on the GPU a graphed RMSNorm (the HIP kernel, as petals/llama/block.py:210-213
graphs the input norm) equal to the eager call for new inputs, with and without the copy."""
import pytest
import torch

from src import ops
from src.runtime.graphs import make_inference_graphed_callable


def _norm(x, w):
    return ops.rmsnorm(x, w, 1e-5)


def test_cpu_returns_the_callable():
    x, w = torch.randn(4, 64), torch.ones(64)
    assert make_inference_graphed_callable(_norm, (x, w)) is _norm


@pytest.mark.gpu
def test_graphed_rmsnorm_matches_eager():
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(8, 512, device="cuda", generator=g).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(512, device="cuda", generator=g)).to(torch.bfloat16)
    fn = make_inference_graphed_callable(_norm, (x, w))
    assert fn is not _norm
    for i in range(3):
        xi = torch.randn(8, 512, device="cuda", generator=g).to(torch.bfloat16)
        assert torch.equal(fn(xi, w), _norm(xi, w)), i
    # an argument that already is the static input: no copy, same result
    xs = fn.static_inputs[0]
    xs.copy_(torch.randn(8, 512, device="cuda", generator=g).to(torch.bfloat16))
    assert torch.equal(fn(xs, w), _norm(xs.clone(), w))
    with pytest.raises(ValueError):
        fn(torch.zeros(4, 512, device="cuda", dtype=torch.bfloat16), w)

"""Sampler semantics (reference src/rpc_handler.py:327-403) on the CPU path."""
import torch

from src import ops
from src.ops import reference as ref
from src.runtime.sampler import BatchSampler, SamplingParams, session_seed


def test_greedy_and_penalty():
    lg = torch.zeros(10)
    lg[3], lg[4] = 5.0, 4.9
    assert ref.sample_row(lg, 0.0, 0.9, 0) == 3
    # token 3 repeated 3x: rp**3 then last-3 strong penalty rp**3 -> token 4 wins under top_k=1
    assert ref.sample_row(lg, 1.0, 1.0, 1, 1.5, [3, 3, 3]) == 4
    # negative logits are multiplied by the penalty
    lg2 = torch.full((5,), -1.0)
    lg2[0] = -0.5
    assert ref.sample_row(lg2, 1.0, 1.0, 1, 2.0, [0]) != 0


def test_top_p_keeps_first_and_cum_le_p():
    lg = torch.log(torch.tensor([0.5, 0.3, 0.15, 0.05]))
    g = torch.Generator().manual_seed(0)
    seen = {ref.sample_row(lg, 1.0, 0.6, 0, 1.0, [], generator=g) for _ in range(200)}
    assert seen == {0}  # cum: 0.5 <= 0.6 kept, 0.8 > 0.6 dropped
    seen = {ref.sample_row(lg, 1.0, 0.85, 0, 1.0, [], generator=g) for _ in range(400)}
    assert seen == {0, 1}
    seen = {ref.sample_row(lg, 1.0, 0.1, 0, 1.0, [], generator=g) for _ in range(50)}
    assert seen == {0}  # first token always kept


def test_batch_sampler_cpu():
    s = BatchSampler("cpu")
    lg = torch.randn(3, 50)
    out = s(lg, [SamplingParams(0.0, 0.9, 0, 1.0)] * 3, [[], [], []], [1, 2, 3])
    assert torch.equal(out, torch.argmax(lg, -1))
    out = s(lg, [SamplingParams(1.0, 0.9, 5, 1.5)] * 3, [[1], [2, 2], []], [session_seed("a", 1)] * 3)
    assert out.shape == (3,) and int(out.max()) < 50

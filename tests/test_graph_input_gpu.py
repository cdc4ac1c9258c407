"""Stage-hop receive target (``StageExecutor.graph_input``): a hop received straight into the
static input of the decode graph the step replays - two receive graphs per batch bucket, used in
alternation - gives exactly the logits / hidden states of the ordinary path (receive slab + copy
into the graph input).  Reference hop: /root/reference/src/rpc_transport.py:738-766."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _stage(cfg, seed=4):
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    w = random_stage_weights(cfg, 2, 4, has_embed=False, has_head=False, device="cuda", seed=seed)
    return StageExecutor(cfg, w, "cuda", kv_cache_bytes=128 << 20, max_sessions=16, max_seq_len=256,
                         graph_max_batch=16)


def test_receive_into_graph_input_equals_copy_path():
    from src.models.config import resolve_model

    cfg = resolve_model("small-llama")
    a, b = _stage(cfg), _stage(cfg)
    owner = object()
    g = torch.Generator(device="cuda").manual_seed(0)
    n, H = 6, cfg.hidden_size
    seqs = [(f"s{i}", 9) for i in range(n)]
    x0 = (0.5 * torch.randn(n * 9, H, device="cuda", generator=g)).to(torch.bfloat16)
    ya, yb = a.forward(seqs, x0, reset=[True] * n), b.forward(seqs, x0, reset=[True] * n)
    assert torch.equal(ya, yb)
    slots = []
    for step in range(4):
        x = (0.5 * torch.randn(n, H, device="cuda", generator=g)).to(torch.bfloat16)
        ya = a.forward([(s, 1) for s, _ in seqs], x)
        buf, free = b.graph_input(n, 9 + step + 1, owner=owner)
        assert buf.shape == (b._bucket(n), H) and buf.is_contiguous()
        if free is not None:
            torch.cuda.current_stream().wait_event(free)
        buf[:n].copy_(x)  # what the RCCL receive writes
        pin = b._recv_pin[1]
        yb = b.forward([(s, 1) for s, _ in seqs], buf[:n], hook_owner=owner)
        slots.append(pin[-1])
        torch.cuda.synchronize()
        assert b.last_graphed and torch.equal(ya, yb), step
    assert slots == [1, 2, 1, 2]  # the two receive graphs alternate
    assert {k[-1] for k in b._graphs} >= {1, 2}
    # another caller (no owner) never replays a receive graph
    x = (0.5 * torch.randn(n, H, device="cuda", generator=g)).to(torch.bfloat16)
    b.graph_input(n, 14, owner=owner)
    yn = b.forward([(s, 1) for s, _ in seqs], x)  # no hook_owner: the slot-0 graph, pin untouched
    assert b._recv_pin is not None and torch.isfinite(yn.float()).all()

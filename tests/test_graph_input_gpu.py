"""Stage-hop receive target (``StageExecutor.graph_input``): a hop received straight into the
static input of the decode graph the step replays - two receive graphs per (owner, batch bucket),
used in alternation - gives exactly the logits / hidden states of the ordinary path (receive slab +
copy into the graph input).  Reference hop: /root/reference/src/rpc_transport.py:738-766; replay
into a static input surface: /root/reference/petals/llama/cuda_graphs.py:5-76.

The scenarios run in a child process (``python tests/test_graph_input_gpu.py <case>``): a device
fault there becomes this test's failure with the child's whole stderr, not the end of the suite.
Every step synchronises and compares, so a failure names its step."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stage(cfg, seed=4):
    from src.models.weights import random_stage_weights
    from src.runtime.executor import StageExecutor

    w = random_stage_weights(cfg, 2, 4, has_embed=False, has_head=False, device="cuda", seed=seed)
    return StageExecutor(cfg, w, "cuda", kv_cache_bytes=128 << 20, max_sessions=32, max_seq_len=256,
                         graph_max_batch=16)


def case_alternation():
    import torch

    from src.models.config import resolve_model

    cfg = resolve_model("small-llama")
    a, b = _stage(cfg), _stage(cfg)
    owner = object()
    g = torch.Generator(device="cuda").manual_seed(0)
    n, H = 6, cfg.hidden_size
    seqs = [(f"s{i}", 9) for i in range(n)]
    x0 = (0.5 * torch.randn(n * 9, H, device="cuda", generator=g)).to(torch.bfloat16)
    ya, yb = a.forward(seqs, x0, reset=[True] * n), b.forward(seqs, x0, reset=[True] * n)
    torch.cuda.synchronize()
    assert torch.equal(ya, yb), "prefill"
    slots = []
    for step in range(4):
        x = (0.5 * torch.randn(n, H, device="cuda", generator=g)).to(torch.bfloat16)
        ya = a.forward([(s, 1) for s, _ in seqs], x)
        buf, free = b.graph_input(n, 9 + step + 1, owner=owner)
        assert buf.shape == (b._bucket(n), H) and buf.is_contiguous()
        if free is not None:
            torch.cuda.current_stream().wait_event(free)
        buf[:n].copy_(x)  # what the channel's receive writes
        key = b._recv_pin[b._tag_of(owner)][0]
        yb = b.forward([(s, 1) for s, _ in seqs], buf[:n], hook_owner=owner)
        torch.cuda.synchronize()
        slots.append(key[-1])
        assert b.last_graphed and torch.equal(ya, yb), f"step {step}"
    assert slots == [1, 2, 1, 2], slots  # the two receive graphs alternate
    assert {k[-1] for k in b._graphs} >= {1, 2}
    # another caller (no owner) replays the shared slot-0 graph and leaves the owner's pin alone
    x = (0.5 * torch.randn(n, H, device="cuda", generator=g)).to(torch.bfloat16)
    b.graph_input(n, 14, owner=owner)
    ya = a.forward([(s, 1) for s, _ in seqs], x)
    yn = b.forward([(s, 1) for s, _ in seqs], x)
    torch.cuda.synchronize()
    assert torch.equal(ya, yn), "slot-0 graph"
    assert b._tag_of(owner) in b._recv_pin
    b.release_owner(owner)
    assert not b._recv_pin and not any(k[5] for k in b._graphs)


def case_two_owners():
    """two engines sharing one executor.  A's and B's receives interleave (A, B, B, A
    ...); each owner's replay reads its OWN payload, and a step whose shape no longer matches its
    receive graph copies from that buffer and marks it read."""
    import torch

    from src.models.config import resolve_model

    cfg = resolve_model("small-llama")
    ref, ex = _stage(cfg), _stage(cfg)
    oa, ob = object(), object()
    g = torch.Generator(device="cuda").manual_seed(1)
    n, H = 5, cfg.hidden_size
    sa = [(f"a{i}", 7) for i in range(n)]
    sb = [(f"b{i}", 7) for i in range(n)]
    for s in (sa, sb):
        x0 = (0.5 * torch.randn(n * 7, H, device="cuda", generator=g)).to(torch.bfloat16)
        assert torch.equal(ref.forward(s, x0, reset=[True] * n), ex.forward(s, x0, reset=[True] * n))
    ctx = {id(oa): 8, id(ob): 8}
    for step in range(6):
        # both owners' payloads land first (A then B, or B then A), then the two steps run in the
        # other order: the interleaving in which a shared slot counter handed B A's buffer
        first = "ab" if step % 2 == 0 else "ba"
        landed = {}
        for who in first:
            owner, seqs = (oa, sa) if who == "a" else (ob, sb)
            x = (0.5 * torch.randn(n, H, device="cuda", generator=g)).to(torch.bfloat16)
            buf, free = ex.graph_input(n, ctx[id(owner)], owner=owner)
            if free is not None:
                torch.cuda.current_stream().wait_event(free)
            buf[:n].copy_(x)
            landed[who] = (x, buf)
        for who in reversed(first):
            owner, seqs = (oa, sa) if who == "a" else (ob, sb)
            x, buf = landed[who]
            want = ref.forward([(s, 1) for s, _ in seqs], x)
            got = ex.forward([(s, 1) for s, _ in seqs], buf[:n], hook_owner=owner)
            torch.cuda.synchronize()
            assert torch.equal(want, got), f"step {step} owner {who}"
            ctx[id(owner)] += 1
    tags = {ex._tag_of(oa), ex._tag_of(ob)}
    assert len(tags) == 2 and {k[5] for k in ex._graphs} >= tags  # separate receive graphs per owner
    # pin mismatch: the owner's receive lands for 5 rows, the step then runs 3 of them (another
    # bucket): the replay copies from the pinned buffer, which is then marked read by that replay
    x = (0.5 * torch.randn(n, H, device="cuda", generator=g)).to(torch.bfloat16)
    buf, free = ex.graph_input(n, ctx[id(oa)], owner=oa)
    if free is not None:
        torch.cuda.current_stream().wait_event(free)
    buf[:n].copy_(x)
    pkey, pg = ex._recv_pin[ex._tag_of(oa)]
    want = ref.forward([(s, 1) for s, _ in sa[:3]], x[:3])
    got = ex.forward([(s, 1) for s, _ in sa[:3]], buf[:3], hook_owner=oa)
    torch.cuda.synchronize()
    assert torch.equal(want, got), "pin mismatch"
    assert ex._bucket(3) != ex._bucket(n) and pg.done_ev is ex._graphs[ex._graph_key(3, ctx[id(oa)], False)].done_ev


@pytest.mark.parametrize("case", ["alternation", "two_owners"])
def test_receive_into_graph_input(case):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-X", "faulthandler", os.path.abspath(__file__), case], cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "CASE OK" in r.stdout, \
        f"child rc={r.returncode}\n--- stdout ---\n{r.stdout[-4000:]}\n--- stderr ---\n{r.stderr[-12000:]}"


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    import torch

    with torch.no_grad():
        globals()["case_" + sys.argv[1]]()
    print("CASE OK", flush=True)

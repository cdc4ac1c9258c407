"""Stateless forward/backward through a swarm with deep prompts (upstream rpc_forward/rpc_backward,
petals/server/handler.py:352-488, block_functions.py:32-141) vs local autograd on the same weights."""
import pytest
import torch

from src.dht_utils import get_stage_key
from src.models.config import resolve_model
from src.models.weights import random_stage_weights
from src.rpc_transport import RpcTransport
from src.runtime.autograd_stage import AutogradStage

from .swarm_utils import ServerThread, server_argv, wait_for


def test_autograd_stage_matches_reference_forward():
    from src.models.reference_model import llama_forward

    cfg = resolve_model("tiny-llama")
    w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cpu",
                             dtype=torch.float32, seed=2)
    ids = torch.randint(0, cfg.vocab_size, (9,), generator=torch.Generator().manual_seed(1))
    ag = AutogradStage(cfg, w, "cpu", torch.float32)
    out = ag.forward(w.embed[ids].unsqueeze(0))
    torch.testing.assert_close(out[0], llama_forward([w], ids, return_hidden=True), atol=1e-5, rtol=1e-5)


def test_prompt_gradient_is_input_gradient_slice():
    """Upstream semantics: grad(prompt_i) == grad wrt hidden[:, :P] at block i's input."""
    cfg = resolve_model("tiny-llama")
    w = random_stage_weights(cfg, 0, 2, has_embed=False, has_head=False, device="cpu", dtype=torch.float32)
    ag = AutogradStage(cfg, w, "cpu", torch.float32)
    g = torch.Generator().manual_seed(0)
    h = torch.randn(2, 6, cfg.hidden_size, generator=g)
    p = 0.1 * torch.randn(2, 1, 3, cfg.hidden_size, generator=g)
    go = torch.randn(2, 6, cfg.hidden_size, generator=g)
    gh, gp = ag.backward(h, go, p)
    # with a zero prompt on block 0, grad(prompt_0) is the batch-summed input grad of its first 3 tokens
    p0 = p.clone()
    p0[0] = 0
    gh0, gp0 = ag.backward(h + torch.cat([p[0].expand(2, 3, -1), torch.zeros(2, 3, cfg.hidden_size)], 1), go, p0)
    torch.testing.assert_close(gp0[0, 0], gh0[:, :3].sum(0), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(gp[1], gp0[1], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-gpt2"])
def test_inference_with_deep_prompts_matches_stateless_forward(model):
    """Deep prompts in the KV-cached inference path (upstream iterate_rpc_inference) == stateless forward."""
    from src.runtime.executor import StageExecutor

    cfg = resolve_model(model)
    L, H = cfg.num_hidden_layers, cfg.hidden_size
    w = random_stage_weights(cfg, 1, L, has_embed=False, has_head=False, device="cpu", dtype=torch.float32)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=4, max_seq_len=128)
    ag = AutogradStage(cfg, w, "cpu", torch.float32)
    g = torch.Generator().manual_seed(3)
    h = torch.randn(9, H, generator=g)
    p = 0.5 * torch.randn(L - 1, 3, H, generator=g)
    out = ex.forward([("a", 6), ("b", 3)], torch.cat([h[:6], h[6:]]), prompts=[p, None])
    torch.testing.assert_close(out[:6], ag.forward(h[None, :6], p[:, None])[0], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(out[6:], ag.forward(h[None, 6:9])[0], atol=1e-5, rtol=1e-5)
    # next step without prompts attends to the prompted prefix
    nxt = torch.randn(1, H, generator=g)
    step = ex.forward([("a", 1)], nxt)
    full = ag.forward(torch.cat([h[:6], nxt])[None], p[:, None])[0, -1]
    torch.testing.assert_close(step[0], full, atol=1e-5, rtol=1e-5)


@pytest.mark.timeout(120)
def test_rpc_inference_accepts_prompts():
    from src.comm.rpc import RpcClient, get_loop
    from src.comm.wire import Message

    model = "tiny-llama"
    cfg = resolve_model(model)
    s1 = ServerThread(server_argv(model, "1,2", 1)).wait()
    try:
        addr, cl, loop = s1.srv.maddrs[0], RpcClient(), get_loop()
        h = torch.randn(1, 4, cfg.hidden_size)
        p = torch.randn(1, 1, 2, cfg.hidden_size)  # [n_blocks=1, B, P, H]

        def call(md, ts):
            return loop.run(cl.call(addr, "StageConnectionHandler.rpc_inference", Message(md, ts), 10.0))

        with_p = call({"session_id": "p", "has_prompts": True}, [h, p]).tensors[0]
        without = call({"session_id": "q"}, [h]).tensors[0]
        assert not torch.allclose(with_p[:, :2], without[:, :2])
        w = random_stage_weights(cfg, 1, 2, has_embed=False, has_head=False, device="cpu", dtype=torch.float32)
        ref = AutogradStage(cfg, w, "cpu", torch.float32).forward(h, p)
        torch.testing.assert_close(with_p, ref, atol=1e-5, rtol=1e-5)
        loop.run(cl.close())
    finally:
        s1.close()


@pytest.mark.gpu
def test_gpu_executor_deep_prompts():
    from src.runtime.executor import StageExecutor

    cfg = resolve_model("small-llama")
    L, H = cfg.num_hidden_layers, cfg.hidden_size
    w = random_stage_weights(cfg, 1, L, has_embed=False, has_head=False, device="cuda", seed=5)
    ex = StageExecutor(cfg, w, "cuda", kv_cache_bytes=64 << 20, max_sessions=4, max_seq_len=256)
    g = torch.Generator().manual_seed(0)
    h = torch.randn(12, H, generator=g).to("cuda", torch.bfloat16)
    p = (0.5 * torch.randn(L - 1, 4, H, generator=g)).to("cuda", torch.bfloat16)
    out = ex.forward([("a", 12)], h, prompts=[p]).float()
    ref = AutogradStage(cfg, w, "cuda").forward(h[None], p[:, None])[0].float()
    assert float((out - ref).norm() / ref.norm()) < 0.02
    plain = ex.forward([("b", 12)], h).float()
    assert float((plain[:4] - out[:4]).norm() / out[:4].norm()) > 0.05  # the prompt changed the output


@pytest.mark.gpu
@pytest.mark.parametrize("n_tok", [12, 100])
def test_gpu_executor_deep_prompts_nonunit_norms(n_tok):
    """The fused-norm path packs qkv / gate_up with the RMSNorm weights folded in: the
    row-major branch (deep prompts, 65..128-row steps) must not apply them twice."""
    from src.runtime.executor import StageExecutor

    cfg = resolve_model("small-llama")
    L, H = cfg.num_hidden_layers, cfg.hidden_size
    w = random_stage_weights(cfg, 1, L, has_embed=False, has_head=False, device="cuda", seed=6)
    for i, lay in enumerate(w.layers):
        gen = torch.Generator(device="cuda").manual_seed(50 + i)
        lay.input_norm = (torch.rand(H, device="cuda", generator=gen) + 0.5).to(torch.bfloat16)
        lay.post_norm = (torch.rand(H, device="cuda", generator=gen) + 0.5).to(torch.bfloat16)
    ex = StageExecutor(cfg, w, "cuda", kv_cache_bytes=64 << 20, max_sessions=4, max_seq_len=256)
    assert all(lay.folded for lay in w.layers)
    g = torch.Generator().manual_seed(1)
    h = torch.randn(n_tok, H, generator=g).to("cuda", torch.bfloat16)
    p = (0.5 * torch.randn(L - 1, 4, H, generator=g)).to("cuda", torch.bfloat16)
    ag = AutogradStage(cfg, w, "cuda")
    out = ex.forward([("a", n_tok)], h, prompts=[p]).float()
    ref = ag.forward(h[None], p[:, None])[0].float()
    assert float((out - ref).norm() / ref.norm()) < 0.02
    plain = ex.forward([("b", n_tok)], h).float()
    ref_plain = ag.forward(h[None])[0].float()
    assert float((plain - ref_plain).norm() / ref_plain.norm()) < 0.02


@pytest.mark.gpu
def test_autograd_stage_bf16_on_gpu_matches_fp32():
    import dataclasses

    cfg = resolve_model("small-llama")
    wg = random_stage_weights(cfg, 0, 2, has_embed=False, has_head=False, device="cuda", dtype=torch.bfloat16, seed=4)

    def f32(obj):  # the same weights, fp32 on the CPU
        return dataclasses.replace(obj, **{f.name: getattr(obj, f.name).float().cpu() for f in dataclasses.fields(obj)
                                           if isinstance(getattr(obj, f.name), torch.Tensor)})

    w32 = dataclasses.replace(wg, layers=[f32(lay) for lay in wg.layers])
    g = torch.Generator().manual_seed(0)
    h = torch.randn(2, 40, cfg.hidden_size, generator=g)
    p = 0.1 * torch.randn(2, 2, 4, cfg.hidden_size, generator=g)
    go = torch.randn(2, 40, cfg.hidden_size, generator=g)
    with torch.no_grad():
        fo = AutogradStage(cfg, wg, "cuda").forward(h.cuda(), p.cuda()).float().cpu()
        ro = AutogradStage(cfg, w32, "cpu", torch.float32).forward(h, p)
    ferr = float((fo - ro).norm() / ro.norm())
    assert ferr < 0.02, ferr
    gh, gp = AutogradStage(cfg, wg, "cuda").backward(h.cuda(), go.cuda(), p.cuda())
    rh, rp = AutogradStage(cfg, w32, "cpu", torch.float32).backward(h, go, p)
    assert gh.dtype == torch.bfloat16 and gh.is_cuda
    for a, b in ((gh, rh), (gp, rp)):
        err = (a.float().cpu() - b).norm() / b.norm()
        assert err < 0.03, float(err)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("model", ["tiny-gpt2", "tiny-llama"])
def test_remote_blocks_gradients_match_local(model):
    cfg = resolve_model(model)
    L, H = cfg.num_hidden_layers, cfg.hidden_size
    s1 = ServerThread(server_argv(model, "1,2", 1)).wait()
    s2 = ServerThread(server_argv(model, "1,2", 2, peers=s1.addr)).wait()
    try:
        assert wait_for(lambda: s1.dht.get(get_stage_key(2)) is not None)
        tx = RpcTransport("cpu", 0, [s1.addr], timeout=10.0, stage_keys=[get_stage_key(1), get_stage_key(2)],
                          model_name=model, total_blocks=L, start_block=1)
        g = torch.Generator().manual_seed(0)
        h = torch.randn(2, 5, H, generator=g).requires_grad_()
        prompts = (0.1 * torch.randn(L - 1, 1, 2, H, generator=g)).requires_grad_()
        wl = torch.randn(2, 5, H, generator=g)
        out = tx.remote_blocks(h, prompts)
        (out * wl).sum().backward()

        w = random_stage_weights(cfg, 1, L, has_embed=False, has_head=True, device="cpu", dtype=torch.float32)
        ag = AutogradStage(cfg, w, "cpu", torch.float32)
        h2, p2 = h.detach().clone().requires_grad_(), prompts.detach().clone().requires_grad_()
        out2 = ag.forward(h2, p2)
        (out2 * wl).sum().backward()
        torch.testing.assert_close(out, out2, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(h.grad, h2.grad, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(prompts.grad, p2.grad, atol=1e-5, rtol=1e-5)
        assert s1.srv.handler.stats.get("backward") == 1 and s2.srv.handler.stats.get("backward") == 1
        # no prompts: plain input gradient
        h3 = h.detach().clone().requires_grad_()
        tx.remote_blocks(h3).sum().backward()
        assert h3.grad is not None and torch.isfinite(h3.grad).all()
        tx.shutdown()
    finally:
        s1.close()
        s2.close()

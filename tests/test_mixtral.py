"""Mixtral sparse-MoE blocks (model_type "mixtral", accepted by reference src/llama_partition.py:81-83).

CPU: the executor's two MoE schedules (dense all-experts combine for T <= 64, expert-grouped
prefill for T > 64) vs the fp32 oracle; stage splits; the stateless autograd stage; HF
``MixtralForCausalLM`` checkpoint parity through the safetensors loader.
GPU (@gpu): packed decode GEMMs + hipGraph decode vs the fp32 oracle.
"""
import dataclasses

import pytest
import torch

from src.models.config import ModelConfig, resolve_model
from src.models.reference_model import reference_forward
from src.models.weights import build_stage_weights, random_stage_weights
from src.ops import moe
from src.runtime.autograd_stage import AutogradStage
from src.runtime.executor import StageExecutor


def _w(cfg, start, end, embed, head, device="cpu", dtype=torch.float32, seed=11):
    return random_stage_weights(cfg, start, end, has_embed=embed, has_head=head, device=device, dtype=dtype,
                                seed=seed)


def test_route_matches_hf_semantics():
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(9, 8, generator=g)
    w, idx = moe.route(logits, 2)
    p = torch.softmax(logits, -1)
    top = p.topk(2, -1)
    torch.testing.assert_close(idx, top.indices)
    torch.testing.assert_close(w, top.values / top.values.sum(-1, keepdim=True))
    d = moe.dense_weights(w, idx, 8)
    torch.testing.assert_close(d.sum(-1), torch.ones(9))
    assert int((d > 0).sum()) == 18


def test_mixtral_config_from_hf_dict():
    cfg = ModelConfig.from_hf_dict({"model_type": "mixtral", "vocab_size": 100, "hidden_size": 256,
                                    "intermediate_size": 512, "num_hidden_layers": 2, "num_attention_heads": 4,
                                    "num_key_value_heads": 2, "num_local_experts": 8, "num_experts_per_tok": 2,
                                    "sliding_window": None})
    assert cfg.is_moe and cfg.num_local_experts == 8 and cfg.num_experts_per_tok == 2
    dense = dataclasses.replace(cfg, num_local_experts=0)
    assert cfg.layer_param_bytes() > 4 * dense.layer_param_bytes()
    mistral = ModelConfig.from_hf_dict({"model_type": "mistral", "vocab_size": 100, "hidden_size": 256,
                                        "intermediate_size": 512, "num_hidden_layers": 2, "num_attention_heads": 4,
                                        "num_key_value_heads": 2, "sliding_window": 128})
    assert not mistral.is_moe and mistral.sliding_window == 128


def test_sparse_and_dense_schedules_match_oracle():
    cfg = resolve_model("tiny-mixtral")
    w = _w(cfg, 0, cfg.num_hidden_layers, True, True)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=16 << 20, max_sessions=4, max_seq_len=256)
    g = torch.Generator().manual_seed(1)
    a = torch.randint(0, cfg.vocab_size, (90,), generator=g)   # > 64 rows: expert-grouped prefill
    b = torch.randint(0, cfg.vocab_size, (7,), generator=g)
    lg = ex.forward([("a", 90), ("b", 7)], torch.cat([a, b]))
    torch.testing.assert_close(lg[0], reference_forward([w], a)[-1], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(lg[1], reference_forward([w], b)[-1], atol=1e-4, rtol=1e-4)
    for _ in range(3):  # decode steps: dense all-experts combine
        nxt = torch.argmax(lg, -1)
        a, b = torch.cat([a, nxt[:1]]), torch.cat([b, nxt[1:]])
        lg = ex.forward([("a", 1), ("b", 1)], nxt)
        torch.testing.assert_close(lg[0], reference_forward([w], a)[-1], atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(lg[1], reference_forward([w], b)[-1], atol=1e-4, rtol=1e-4)


def test_two_stage_split_equals_single_stage():
    cfg = resolve_model("tiny-mixtral")
    L = cfg.num_hidden_layers
    full = _w(cfg, 0, L, True, True)
    s0, s1 = _w(cfg, 0, 2, True, False), _w(cfg, 2, L, False, True)
    mk = lambda w: StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=2,  # noqa
                                 max_seq_len=128)
    ef, e0, e1 = mk(full), mk(s0), mk(s1)
    ids = torch.arange(20) * 7 % cfg.vocab_size
    torch.testing.assert_close(e1.forward([("s", 20)], e0.forward([("s", 20)], ids)), ef.forward([("s", 20)], ids),
                               atol=1e-5, rtol=1e-5)


def test_autograd_stage_moe_forward_and_grad():
    cfg = resolve_model("tiny-mixtral")
    w = _w(cfg, 0, 2, False, False, dtype=torch.float64)
    st = AutogradStage(cfg, w, "cpu", dtype=torch.float64)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 9, cfg.hidden_size, generator=g, dtype=torch.float64) * 0.5
    out = st.forward(x)
    assert out.shape == x.shape
    gx, _ = st.backward(x, torch.ones_like(out))
    # finite-difference check of d(sum out)/dx along a random direction
    d = torch.randn(x.shape, generator=g, dtype=torch.float64) * 1e-3
    fd = (st.forward(x + d).sum() - st.forward(x - d).sum()) / 2
    torch.testing.assert_close((gx * d).sum(), fd, atol=1e-6, rtol=1e-2)


def test_hf_mixtral_checkpoint_parity(tmp_path):
    """Save a tiny random HF MixtralForCausalLM as safetensors, load it through this framework's
    per-stage loader (two stages) and compare logits with transformers' own forward."""
    tr = pytest.importorskip("transformers")
    hcfg = tr.MixtralConfig(vocab_size=128, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                            num_attention_heads=4, num_key_value_heads=2, num_local_experts=4,
                            num_experts_per_tok=2, max_position_embeddings=256, sliding_window=None,
                            tie_word_embeddings=False)
    torch.manual_seed(0)
    model = tr.MixtralForCausalLM(hcfg).float().eval()
    with torch.no_grad():  # make the routing decisive so fp32 summation order cannot flip an expert
        for layer in model.model.layers:
            layer.mlp.gate.weight.mul_(20) if hasattr(layer, "mlp") and hasattr(layer.mlp, "gate") else \
                layer.block_sparse_moe.gate.weight.mul_(20)
    model.save_pretrained(tmp_path, safe_serialization=True)
    cfg = resolve_model(str(tmp_path))
    assert cfg.model_type == "mixtral" and cfg.num_local_experts == 4
    s0 = build_stage_weights(cfg, str(tmp_path), 0, 1, has_embed=True, has_head=False, device="cpu",
                             dtype=torch.float32)
    s1 = build_stage_weights(cfg, str(tmp_path), 1, 2, has_embed=False, has_head=True, device="cpu",
                             dtype=torch.float32)
    ids = torch.randint(0, 128, (24,), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        ref = model(ids[None]).logits[0]
    torch.testing.assert_close(reference_forward([s0, s1], ids), ref, atol=1e-4, rtol=1e-4)
    mk = lambda w: StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=2,  # noqa
                                 max_seq_len=128)
    e0, e1 = mk(s0), mk(s1)
    out = e1.forward([("s", 24)], e0.forward([("s", 24)], ids))
    torch.testing.assert_close(out[-1], ref[-1], atol=1e-4, rtol=1e-4)


def test_sliding_window_caps_session_length():
    cfg = dataclasses.replace(resolve_model("tiny-llama"), model_type="mistral", sliding_window=96)
    w = _w(cfg, 0, 1, True, False)
    ex = StageExecutor(cfg, w, "cpu", dtype=torch.float32, kv_cache_bytes=8 << 20, max_sessions=2)
    assert ex.max_seq_len == 96


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
def test_mixtral_gpu_matches_fp32_reference(graphs):
    cfg = resolve_model("tiny-mixtral")
    w = _w(cfg, 0, cfg.num_hidden_layers, True, True, device="cuda", dtype=torch.bfloat16, seed=4)
    ex = StageExecutor(cfg, w, "cuda", kv_cache_bytes=128 << 20, max_sessions=4, max_seq_len=256, use_graphs=graphs)
    assert w.layers[0].router_p is not None and w.layers[0].gate_up_p.shape[0] == cfg.num_local_experts
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(0, cfg.vocab_size, (n,), generator=g) for n in (80, 9)]
    logits = ex.forward([("a", 80), ("b", 9)], torch.cat(prompts).cuda())
    seqs = [p.clone() for p in prompts]
    for _ in range(5):
        for i, p in enumerate(seqs):
            r = reference_forward([w], p.cuda())[-1]
            torch.testing.assert_close(logits[i].float(), r, atol=0.06, rtol=0.05)
        nxt = torch.argmax(logits.float(), -1)
        seqs = [torch.cat([s, nxt[i:i + 1].cpu()]) for i, s in enumerate(seqs)]
        logits = ex.forward([("a", 1), ("b", 1)], nxt)

"""Parity against transformers' own forward on real HF checkpoint layouts (CPU, fp32).

A tiny random ``LlamaForCausalLM`` (with and without llama3 ``rope_scaling``) and a tiny
``GPT2LMHeadModel`` are written with ``save_pretrained`` (safetensors) or as
``pytorch_model.bin`` (single file and sharded index), loaded TWO-STAGE through
``load_stage_model`` (the reference's API, src/llama_partition.py:477-550) and compared with
transformers' logits for the prompt and for greedy decode steps.  This pins the parts the
framework's own fp32 oracle cannot: the HF key names, the GPT-2 Conv1D transposes, the
gate/up interleave on real checkpoints and the llama3 RoPE frequency scaling.
"""
import json
import os

import pytest
import torch

tr = pytest.importorskip("transformers")

from src.llama_partition import StageLast, StageSegment, Stage0, load_stage_model  # noqa: E402
from src.models.config import resolve_model  # noqa: E402
from src.runtime.executor import StageExecutor  # noqa: E402

LLAMA3_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                  "original_max_position_embeddings": 64}


def _llama(scaling=None, tie=False):
    hcfg = tr.LlamaConfig(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=3,
                          num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512,
                          rope_theta=50000.0, rope_scaling=scaling, tie_word_embeddings=tie, rms_norm_eps=1e-5)
    torch.manual_seed(0)
    m = tr.LlamaForCausalLM(hcfg).float().eval()
    with torch.no_grad():  # non-trivial norm weights so a dropped / misplaced norm shows
        for n, p in m.named_parameters():
            if "norm" in n:
                p.uniform_(0.5, 1.5)
    return m


def _gpt2():
    hcfg = tr.GPT2Config(vocab_size=256, n_embd=128, n_layer=3, n_head=4, n_positions=256)
    torch.manual_seed(0)
    m = tr.GPT2LMHeadModel(hcfg).float().eval()
    with torch.no_grad():  # random biases / LN params so every transpose and bias is exercised
        for n, p in m.named_parameters():
            if n.endswith(".bias"):
                p.normal_(0, 0.02)
            if "ln_" in n and n.endswith(".weight"):
                p.uniform_(0.5, 1.5)
    return m


def _save_bin(model, path, sharded: bool):
    model.config.save_pretrained(path)
    sd = {k: v.contiguous() for k, v in model.state_dict().items()}
    if not sharded:
        torch.save(sd, os.path.join(path, "pytorch_model.bin"))
        return
    keys = sorted(sd)
    half = len(keys) // 2
    wm = {}
    for i, part in enumerate((keys[:half], keys[half:])):
        fn = f"pytorch_model-0000{i + 1}-of-00002.bin"
        torch.save({k: sd[k] for k in part}, os.path.join(path, fn))
        wm.update({k: fn for k in part})
    with open(os.path.join(path, "pytorch_model.bin.index.json"), "w") as f:
        json.dump({"metadata": {}, "weight_map": wm}, f)


def _two_stage(path, cut):
    kw = dict(kv_cache_bytes=8 << 20, max_sessions=2, max_seq_len=128)
    f0 = load_stage_model(path, "cpu", "stage0", end=cut, dtype=torch.float32, **kw)
    f1 = load_stage_model(path, "cpu", "last", start=cut, dtype=torch.float32, **kw)
    return Stage0(f0, cut), StageLast(f1, cut)


def _check_generation(model, path, cut=1, steps=4, prompt_len=19):
    s0, s1 = _two_stage(str(path), cut)
    ids = torch.randint(0, model.config.vocab_size, (1, prompt_len), generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        ref = model(ids).logits[0, -1]
        h, p0 = s0(ids, torch.arange(prompt_len)[None], None, None)
        lg, p1 = s1(h, torch.arange(prompt_len)[None], None, None)
    torch.testing.assert_close(lg[0, -1], ref, atol=2e-4, rtol=2e-4)
    seq = ids
    for _ in range(steps):
        nxt = torch.argmax(lg[0, -1]).view(1, 1)
        seq = torch.cat([seq, nxt], 1)
        pos = torch.tensor([[seq.shape[1] - 1]])
        with torch.no_grad():
            ref = model(seq).logits[0, -1]
            h, p0 = s0(nxt, pos, None, p0)
            lg, p1 = s1(h, pos, None, p1)
        torch.testing.assert_close(lg[0, -1], ref, atol=2e-4, rtol=2e-4)


@pytest.mark.parametrize("scaling", [None, LLAMA3_SCALING], ids=["rope-default", "rope-llama3"])
def test_llama_safetensors_two_stage_matches_transformers(tmp_path, scaling):
    m = _llama(scaling)
    m.save_pretrained(tmp_path)
    cfg = resolve_model(str(tmp_path))
    if scaling:
        assert cfg.rope_scaling and cfg.rope_scaling.get("rope_type") == "llama3"
    # prompt + decode crosses original_max_position_embeddings (64): the scaled band matters
    _check_generation(m, tmp_path, cut=1, steps=4, prompt_len=70 if scaling else 19)


@pytest.mark.parametrize("sharded", [False, True], ids=["single-bin", "sharded-bin"])
def test_llama_pytorch_bin_two_stage_matches_transformers(tmp_path, sharded):
    m = _llama(tie=False)
    _save_bin(m, str(tmp_path), sharded)
    assert not any(f.endswith(".safetensors") for f in os.listdir(tmp_path))
    _check_generation(m, tmp_path, cut=2)


def test_llama_tied_embeddings(tmp_path):
    m = _llama(tie=True)
    m.save_pretrained(tmp_path)
    _check_generation(m, tmp_path, cut=1, steps=2)


def test_gpt2_two_stage_matches_transformers(tmp_path):
    m = _gpt2()
    m.save_pretrained(tmp_path)
    _check_generation(m, tmp_path, cut=2)


def test_gpt2_pytorch_bin(tmp_path):
    m = _gpt2()
    _save_bin(m, str(tmp_path), sharded=False)
    _check_generation(m, tmp_path, cut=1, steps=2)


def test_directory_without_weights_raises(tmp_path):
    """A real config with no weight files must not silently fall back to random weights."""
    _llama().config.save_pretrained(tmp_path)
    with pytest.raises(FileNotFoundError, match="without"):
        load_stage_model(str(tmp_path), "cpu", "stage0", end=1, dtype=torch.float32)


def test_stage_wrappers_reject_mismatched_spans(tmp_path):
    m = _llama()
    m.save_pretrained(tmp_path)
    kw = dict(kv_cache_bytes=8 << 20, max_sessions=2, max_seq_len=128)
    f0 = load_stage_model(str(tmp_path), "cpu", "stage0", end=1, dtype=torch.float32, **kw)
    with pytest.raises(ValueError, match="end"):
        Stage0(f0, 2)
    fs = load_stage_model(str(tmp_path), "cpu", "segment", start=1, end=2, dtype=torch.float32, **kw)
    with pytest.raises(ValueError, match="start"):
        StageSegment(fs, start=0, end=2)
    seg = StageSegment(fs, start=1, end=2, gpu_device="cpu")
    assert isinstance(seg.executor, StageExecutor) and (seg.executor.start, seg.executor.end) == (1, 2)
    with pytest.raises(ValueError, match="keep_layers_on_gpu"):
        StageSegment(fs, start=1, end=2, keep_layers_on_gpu=5)

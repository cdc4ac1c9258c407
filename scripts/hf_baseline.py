#!/usr/bin/env python3
"""Reference-equivalent baseline on one MI355X: HF-eager Llama decode (random init, bf16).

Follows the reference's own correctness/perf oracle, scripts/single_gpu_check.py:183-315
(prefill with ``use_cache=True``, then one ``model(input_ids=[[next]], past_key_values=...)``
call per generated token, torch softmax/top-k/top-p/multinomial sampling on the GPU,
``.item()`` per token), with weights resident on the GPU (i.e. WITHOUT the reference's
per-token CPU<->GPU layer streaming, so this is an upper bound for the reference).
Measured at batch 1 (the reference's only mode) and at the benchmark's batch (HF batched
decode) so ``bench.py``'s ``vs_baseline`` compares equal work.

Prints one JSON line.  transformers is installed offline; no weights/tokenizer are needed.
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def sample(logits, temperature, top_p, top_k):
    if temperature <= 0:
        return torch.argmax(logits, -1, keepdim=True)
    probs = torch.softmax(logits.float() / max(temperature, 1e-5), -1)
    if 0 < top_k < probs.size(-1):
        tv, ti = torch.topk(probs, top_k, -1)
        probs = torch.zeros_like(probs).scatter(-1, ti, tv)
    if 0 < top_p < 1:
        sp, si = torch.sort(probs, descending=True, dim=-1)
        keep = torch.cumsum(sp, -1) <= top_p
        keep[..., 0] = True
        probs = torch.zeros_like(probs).scatter(-1, si, sp * keep)
    return torch.multinomial(probs / probs.sum(-1, keepdim=True), 1)


def run(model, batch, prompt_len, new_tokens, vocab, args):
    ids = torch.randint(0, vocab, (batch, prompt_len), device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.inference_mode():
        out = model(input_ids=ids, use_cache=True)
        past = out.past_key_values
        nxt = sample(out.logits[:, -1, :], args.temperature, args.top_p, args.top_k)
        _ = nxt[0, 0].item()
    ttft = time.perf_counter() - t0
    t1 = time.perf_counter()
    with torch.inference_mode():
        for _ in range(new_tokens):
            out = model(input_ids=nxt, past_key_values=past, use_cache=True)
            past = out.past_key_values
            nxt = sample(out.logits[:, -1, :], args.temperature, args.top_p, args.top_k)
            _ = nxt[0, 0].item()  # the reference syncs per token (int(...item()))
    dt = time.perf_counter() - t1
    return ttft, batch * new_tokens / dt, dt / new_tokens


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--new-tokens", type=int, default=32)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--top-p", type=float, default=0.92)
    ap.add_argument("--top-k", type=int, default=50)
    args = ap.parse_args()
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=args.layers,
                      num_attention_heads=32, num_key_value_heads=32, max_position_embeddings=4096,
                      rms_norm_eps=1e-5, torch_dtype=torch.bfloat16)
    torch.set_default_dtype(torch.bfloat16)
    with torch.device("cuda"):
        model = LlamaForCausalLM(cfg)
    torch.set_default_dtype(torch.float32)
    model.eval()
    res = {"model": f"Llama-2-7B ({args.layers} layers) HF eager, random init, bf16", "prompt_len": args.prompt_len,
           "new_tokens": args.new_tokens}
    run(model, 1, 16, 4, cfg.vocab_size, args)  # warm-up
    ttft1, tps1, ms1 = run(model, 1, args.prompt_len, args.new_tokens, cfg.vocab_size, args)
    res.update(batch1_ttft_s=round(ttft1, 4), batch1_decode_tokens_per_s=round(tps1, 2),
               batch1_ms_per_token=round(1000 * ms1, 3))
    if args.batch > 1:
        run(model, args.batch, 16, 2, cfg.vocab_size, args)
        ttftb, tpsb, msb = run(model, args.batch, args.prompt_len, args.new_tokens, cfg.vocab_size, args)
        res.update(batch=args.batch, batch_ttft_s=round(ttftb, 4), batch_decode_tokens_per_s=round(tpsb, 2),
                   batch_ms_per_step=round(1000 * msb, 3))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

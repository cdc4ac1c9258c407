"""Write the committed decode-kernel table (``ops.KERNEL_TABLE``) on an MI355X.

    python -m src.ops.tune                       # every preset the benches and tests run
    python -m src.ops.tune --models llama2-7b --batches 64 --out /tmp/t.json

For each model a full-depth stage with random-init weights is built with no table loaded
(``MPAMD_KERNEL_TABLE=0``), so its executor times every decode GEMM shape it uses (``autotune_gemm``
/ ``autotune_w8`` / ``autotune_qkv_fold``: M buckets 4..64), then ``warmup_serving`` runs the
end-to-end qkv-fold A/B of each decode batch in ``--batches``.  The resulting choices - one entry
per (row bucket, N, K, epilogue) and one fold decision per (graph batch bucket, N, K) - are
written as JSON.  Executors load that file by default, so every box running the tree runs the
same kernel mix (``ops.load_kernel_table``) and bench records carry its sha.
"""
from __future__ import annotations

import argparse
import gc
import os
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--models", default="small-llama,tiny-llama,llama2-7b,llama3-8b,llama3-70b:fp8",
                    help="comma-separated presets; ':fp8' = fp8 (W8A16) projection weights")
    ap.add_argument("--batches", default="64", help="decode batches whose qkv-fold A/B is pinned")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--out", default=None, help="default: the committed table path")
    a = ap.parse_args(argv)
    os.environ["MPAMD_KERNEL_TABLE"] = "0"   # time everything: nothing pre-loaded
    os.environ.setdefault("MPAMD_GEMM_AUTOTUNE", "1")
    import torch

    from .. import ops
    from ..models.config import resolve_model
    from ..models.weights import random_stage_weights
    from ..runtime.executor import StageExecutor

    if not torch.cuda.is_available():
        print("tune: needs an MI355X", file=sys.stderr)
        return 2
    batches = [int(b) for b in a.batches.split(",") if b]
    for spec in [m for m in a.models.split(",") if m]:
        name, _, opt = spec.partition(":")
        cfg = resolve_model(name)
        t0 = time.time()
        w = random_stage_weights(cfg, 0, cfg.num_hidden_layers, has_embed=True, has_head=True, device="cuda",
                                 seed=0, fp8=opt == "fp8")
        B = max(batches)
        ex = StageExecutor(cfg, w, "cuda", max_sessions=B + 8, max_seq_len=512, kv_cache_bytes=8 << 30,
                           graph_max_batch=B, max_tokens_per_step=B * a.prompt_len, warmup=False)
        if cfg.model_type != "gpt2":
            for b in batches:
                ex.warmup_serving(b, a.prompt_len)
        print(f"tune: {spec} done in {time.time() - t0:.1f}s; fold {ex.qkv_fold_by_bucket} "
              f"ab {getattr(ex, 'qkv_fold_ab_ms', {})}", file=sys.stderr, flush=True)
        del ex, w
        gc.collect()
        torch.cuda.empty_cache()
    out = a.out or ops.KERNEL_TABLE
    sha = ops.save_kernel_table(out)
    print(f"tune: wrote {out} (sha {sha})", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

#!/usr/bin/env python3
"""W8A8-MX vs W8A16 decode projections, isolated, under decode conditions (fp8 weights rotated over
~1 GiB of copies, so neither L2 nor the Infinity Cache serves them): per shape and row count, us per
call of the W8A16 GEMM (the committed table's kernel), the MX GEMM alone, and quant_mx + MX GEMM.

    python lab/tools/mx_ab.py --ms 64,32,1
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from src import ops  # noqa: E402

SHAPES = {  # name: (N, K, epilogue)
    "70b.qkv": (10240, 8192, 0), "70b.o": (8192, 8192, 3), "70b.down": (8192, 28672, 3),
    "7b.qkv": (12288, 4096, 0), "7b.o": (4096, 4096, 3), "7b.down": (4096, 11008, 3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="64,32,1")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    ops.load_library()
    ops.load_kernel_table()
    dev = torch.device("cuda")
    ops.gemm_workspace(dev)
    out = []
    for name in a.shapes.split(","):
        N, K, epi = SHAPES[name]
        copies = max(2, (1 << 30) // (N * K))
        ws = []
        for _ in range(copies):
            wq, wsc = ops.pack_weight_fp8(torch.randn(N, K, device=dev) * 0.02)
            ws.append((ops.w8_from_fp8(wq), wsc))
        for M in [int(m) for m in a.ms.split(",")]:
            x = (torch.randn(M, K, device=dev)).to(torch.bfloat16)
            xp = ops.pack_act(x)
            ax, as_ = ops.mx_buffers(M, K, dev)
            res = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            kw = {}
            if epi == 3:
                kw = dict(residual=res, ap_out=torch.zeros(ops.packed_numel(M, N), dtype=torch.bfloat16, device=dev),
                          ss_out=ops.norm_stats_buffer(dev, 2)[0], ss_zero=ops.norm_stats_buffer(dev, 2)[1])
            else:
                kw = dict(ss_in=ops.norm_stats_buffer(dev)[0], eps=1e-5)

            def w8a16(i):
                w8, wsc = ws[i % copies]
                ops.linear_w8(xp, w8, wsc, M, out=res, epilogue=epi, **kw)

            def mx_only(i, rot=False):
                w8, wsc = ws[i % copies]
                ops.linear_mx(ax, as_, w8, wsc, M, out=res, epilogue=epi, rot=rot, **kw)

            def mx_rot(i):
                mx_only(i, True)

            def mx_quant(i):
                ops.quant_mx(xp, M, K, ax, as_)
                mx_only(i)

            def quant_only(i):
                ops.quant_mx(xp, M, K, ax, as_)

            row = {"shape": name, "M": M, "N": N, "K": K}
            for label, fn in (("w8a16", w8a16), ("mx", mx_only), ("mx+r", mx_rot), ("quant+mx", mx_quant), ("quant", quant_only)):
                try:
                    for i in range(4):
                        fn(i)
                    ts = []
                    for rep in range(3):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for i in range(a.iters):
                            fn(i)
                        e1.record()
                        e1.synchronize()
                        ts.append(1000 * e0.elapsed_time(e1) / a.iters)
                    row[label] = round(min(ts), 2)
                except Exception as e:  # noqa: BLE001 - a shape the MX form does not cover
                    row[label] = f"n/a: {str(e)[:60]}"
            print(json.dumps(row), flush=True)
            out.append(row)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    with torch.no_grad():
        main()

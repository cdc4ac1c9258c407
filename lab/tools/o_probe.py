#!/usr/bin/env python3
"""One decode projection under decode conditions, for rocprofv3 --pmc passes: the packed weight
rotated over enough copies that the 256 MB Infinity Cache never serves it (a decode step streams
GBs between two uses of a layer's weights), the kernel the committed table picks per row bucket
(or --kern), the fused-norm producer epilogue of o / down (--epi 3) or none (--epi 0)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from src import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--N", type=int, default=4096)
ap.add_argument("--K", type=int, default=4096)
ap.add_argument("--epi", type=int, default=3)
ap.add_argument("--ms", default="1,64")
ap.add_argument("--kern", default="auto")
ap.add_argument("--iters", type=int, default=24)
ap.add_argument("--copies", type=int, default=0, help="weight copies rotated (0: enough for 1 GiB, i.e. cold)")
a = ap.parse_args()
ops.load_library()
ops.load_kernel_table()
ops.set_gemm_sk(a.kern)
dev = torch.device("cuda")
ops.gemm_workspace(dev)
copies = a.copies or max(2, (1 << 30) // (a.N * a.K * 2))
wps = [ops.pack_weight((torch.randn(a.N, a.K, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(copies)]
for M in [int(m) for m in a.ms.split(",")]:
    xp = ops.pack_act(torch.randn(M, a.K, device=dev).to(torch.bfloat16))
    res = torch.zeros(M, a.N, dtype=torch.bfloat16, device=dev)
    extra = {}
    if a.epi == 3:
        extra = dict(ap_out=torch.zeros(ops.packed_numel(M, a.N), dtype=torch.bfloat16, device=dev),
                     ss_out=ops.norm_stats_buffer(dev)[0], ss_zero=ops.norm_stats_buffer(dev)[0], residual=res)
    out = res if a.epi == 3 else torch.empty(M, a.N, dtype=torch.bfloat16, device=dev)
    print(f"M={M} kernel={ops._kernel_for(M, a.N, a.K, a.epi)}", flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(4):
        ops.linear(xp, None, out=out, epilogue=a.epi, wp=wps[i % copies], a_rows=M, **extra)
    e0.record()
    for i in range(a.iters):
        ops.linear(xp, None, out=out, epilogue=a.epi, wp=wps[i % copies], a_rows=M, **extra)
    e1.record()
    e1.synchronize()
    us = 1000 * e0.elapsed_time(e1) / a.iters
    print(f"N={a.N} K={a.K} copies={copies} M={M}: {us:.2f} us/launch, {a.N * a.K * 2 / us / 1e6:.2f} TB/s weights", flush=True)
torch.cuda.synchronize()

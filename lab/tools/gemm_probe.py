#!/usr/bin/env python3
"""Run one decode GEMM shape a few times per M (for rocprofv3 --pmc counter collection)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from src import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--N", type=int, default=12288)
ap.add_argument("--K", type=int, default=4096)
ap.add_argument("--ms", default="1,64")
ap.add_argument("--sk", default="on")
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
ops.load_library()
ops.set_gemm_sk(a.sk)
w = (torch.randn(a.N, a.K, device="cuda") * 0.02).to(torch.bfloat16)
wp = ops.pack_weight(w)
for M in [int(m) for m in a.ms.split(",")]:
    xp = ops.pack_act(torch.randn(M, a.K, device="cuda").to(torch.bfloat16))
    y = torch.empty(M, a.N, device="cuda", dtype=torch.bfloat16)
    for _ in range(a.iters):
        ops.linear(xp, None, out=y, wp=wp, a_rows=M)
torch.cuda.synchronize()

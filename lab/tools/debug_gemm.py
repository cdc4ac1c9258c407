import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from src import ops
from src.ops import reference as ref
torch.manual_seed(0)
for (N, K) in [(4096, 4096), (12288, 4096), (768, 768)]:
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    wp = ops.pack_weight(w)
    for M in [1, 7, 16, 17, 33, 64]:
        x = torch.randn(M, K, device="cuda").bfloat16()
        yr = x.float() @ w.float().t()
        y = ops.linear(x, None, wp=wp, policy="native")
        ap = ops.pack_act(x)
        y2 = ops.linear(ap, None, wp=wp, a_rows=M)
        e1 = (y.float() - yr).abs().max().item()
        e2 = (y2.float() - yr).abs().max().item()
        print(f"N={N} K={K} M={M} rowmajor_err={e1:.4f} packed_err={e2:.4f} nan={torch.isnan(y.float()).sum().item()}", flush=True)

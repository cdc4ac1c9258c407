import os, sys
sys.path.insert(0, os.getcwd())
import torch
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from src import ops
import test_qkv_fold_gpu as T

for (nh, nkv, D, gqa) in [(32, 8, 128, True), (32, 32, 128, False)]:
    for M in (1, 16):
        c = T._case(nh, nkv, D, M, seed=M)
        N, K = c["N"], c["K"]
        wp = ops.pack_weight(c["w"])
        ops.set_gemm_sk("rwk")
        qkv = ops.linear(c["xp"], None, wp=wp, a_rows=M, ss_in=c["ss"], eps=1e-5)
        ops.set_gemm_sk("auto")
        dummy = torch.zeros_like(qkv)
        part = ops.linear_partials(c["xp"], M, wp=wp, out=dummy)
        red = ops.reduce_qkv_part((part, c["ss"], 1.0 / K, 1e-5))
        print(nh, nkv, M, "S", part.shape[0], "qkv vs torch-reduce maxdiff", float((qkv.float() - red.float()).abs().max()),
              "bitdiff", int((qkv != red).sum()), flush=True)
        o1, k1, v1 = T._attend(c, nh, nkv, D, qkv, None, gqa)
        o2, k2, v2 = T._attend(c, nh, nkv, D, dummy, (part, c["ss"], 1.0 / K, 1e-5), gqa)
        o3, k3, v3 = T._attend(c, nh, nkv, D, red, None, gqa)
        d = (o1.float() - o2.float()).abs()
        print("  o fold-vs-ref maxdiff", float(d.max()), "n", int((o1 != o2).sum()), "of", o1.numel(),
              "| o redtorch-vs-ref", int((o1 != o3).sum()), "| k diff", int((k1 != k2).sum()), "v diff", int((v1 != v2).sum()),
              flush=True)
        if int((o1 != o2).sum()):
            o1u = ops.unpack_act(o1, M, nh * D).float().view(M, nh, D)
            o2u = ops.unpack_act(o2, M, nh * D).float().view(M, nh, D)
            bad = ((o1u - o2u).abs() > 0).nonzero()
            print("  first bad (tok, head, d):", bad[:8].tolist(), flush=True)

"""hipGraphLaunch host time vs the number of kernel nodes in the graph (~4 ms of GPU work each):
does a graph of ~200 kernels (the decode step's size) block the host at launch while the previous
graph still runs (AQL packet ring full), where an 8-kernel graph does not (graph_launch_probe.py)?"""
import time

import torch

x = torch.randn(512, 4096, device="cuda", dtype=torch.bfloat16)
w = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)


def body(n, reps):
    y = x
    for _ in range(n):
        for _ in range(reps):
            y = torch.mm(y, w) * 1e-3
    return y


for n_k, reps in ((8, 16), (64, 2), (128, 1), (256, 1), (512, 1)):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(n_k, reps)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(n_k, reps)
    torch.cuda.synchronize()
    a = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    one = time.perf_counter() - a
    launch = []
    t0 = time.perf_counter()
    for i in range(6):
        b = time.perf_counter()
        g.replay()
        launch.append(time.perf_counter() - b)
    issued = time.perf_counter() - t0
    torch.cuda.synchronize()
    print(f"{2 * n_k * reps:4d} kernels/graph ({1e3 * one:6.2f} ms GPU): host per launch {1e3 * sum(launch) / 6:7.3f} ms "
          f"(first {1e3 * launch[0]:6.3f}, last {1e3 * launch[-1]:6.3f}); 6 issued after {1e3 * issued:7.2f} ms",
          flush=True)
    del g

"""Does hipGraphLaunch block the host until the previous launch of the SAME graph has finished?
Replays one captured ~2 ms graph back to back (host time per launch call) vs two identical graphs
in alternation.  profiles/r5f: the decode step's hipGraphLaunch holds the host ~4 ms per step."""
import time

import torch

x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
w = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)


def body():
    y = x
    for _ in range(8):
        y = torch.mm(y, w) * 1e-3
    return y


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
graphs = []
for _ in range(2):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    graphs.append(g)
torch.cuda.synchronize()
for mode in ("same", "alternate", "same", "alternate"):
    torch.cuda.synchronize()
    launch = []
    t0 = time.perf_counter()
    for i in range(20):
        g = graphs[0] if mode == "same" else graphs[i % 2]
        a = time.perf_counter()
        g.replay()
        launch.append(time.perf_counter() - a)
    issued = time.perf_counter() - t0
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    print(f"{mode:9s}: host per launch call {1e6 * sum(launch) / len(launch):8.1f} us (max {1e6 * max(launch):8.1f}), "
          f"all 20 issued after {1e3 * issued:7.2f} ms, done after {1e3 * total:7.2f} ms", flush=True)

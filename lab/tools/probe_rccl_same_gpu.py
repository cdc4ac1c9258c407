"""Probe: can two RCCL ranks share one GPU (the 1-GPU box)?  Prints the outcome; exit 0 either way."""
import os
import socket
import sys
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(rank, port, q):
    from src.parallel.channel import Channel, make_store

    try:
        ch = Channel(make_store("127.0.0.1", port, 2, rank == 0), "probe", rank, 2, "cuda:0", timeout_s=20)
        if rank == 0:
            ch.send(1, torch.arange(8, device="cuda", dtype=torch.float32))
            ch.flush(20)
        else:
            _, wt = ch.recv(0, (8,), torch.float32)
            t = wt()
            torch.cuda.synchronize()
            q.put(("ok", t.tolist()))
        ch.close()
    except Exception as e:  # noqa: BLE001
        q.put(("error", f"rank {rank}: {type(e).__name__}: {str(e)[:300]}"))


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=run, args=(r, port, q)) for r in range(2)]
    [p.start() for p in ps]
    try:
        print("RCCL same-GPU probe:", q.get(timeout=45), flush=True)
    except Exception as e:  # noqa: BLE001
        print("RCCL same-GPU probe: no result", e, flush=True)
    for p in ps:
        p.join(10)
        if p.is_alive():
            p.kill()

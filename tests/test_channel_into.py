"""``Channel.recv(..., into=(buffer, free_event))`` lands the payload in the caller's buffer on every
backend: the receive-into-graph-input hand-off the stages use must not depend on
the direct-RCCL backend, or the gloo-staged rehearsals never exercise it.

CPU, two gloo processes: plain gloo receives straight into the buffer; the host-staged path
(``staged``: a CPU rank standing in for a GPU rank that shares its card) copies the host payload
into it; a buffer of another shape is ignored; ``waiter.host_wait()`` (the blocking part a stage
runs outside its executor lock) followed by ``waiter()`` gives the same tensor.  The device
backends (ProcessGroupNCCL, direct RCCL) are exercised on the GPU by tests/test_rccl_gpu.py."""
import socket

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q):
    from src.parallel.channel import Channel, make_store

    try:
        ch = Channel(make_store("127.0.0.1", port, 2, rank == 0), "into", rank, 2, "cpu", timeout_s=30.0)
        payloads = [torch.arange(12, dtype=torch.float32).view(3, 4) + 100 * i for i in range(4)]
        if rank == 0:
            for p in payloads:
                ch.send(1, p)
            ch.flush(timeout_s=30.0)
            q.put(("ok", 0, None))
        else:
            res = []
            buf = torch.zeros(3, 4)
            t, w = ch.recv(0, (3, 4), torch.float32, into=(buf, None))        # plain gloo
            w.host_wait()
            y = w()
            res.append(y is buf and t is buf and torch.equal(buf, payloads[0]))
            ch.staged = True                                                # host-staged hand-off
            buf2 = torch.zeros(3, 4)
            t, w = ch.recv(0, (3, 4), torch.float32, into=(buf2, None))
            y = w()
            res.append(y is buf2 and t is buf2 and torch.equal(buf2, payloads[1]))
            ch.staged = False
            wrong = torch.zeros(4, 3)                                       # shape mismatch: ignored
            t, w = ch.recv(0, (3, 4), torch.float32, into=(wrong, None))
            y = w()
            res.append(t is None and y is not wrong and torch.equal(y, payloads[2]) and not wrong.any())
            t, w = ch.recv(0, (3, 4), torch.float32)                        # no target
            res.append(torch.equal(w(), payloads[3]))
            q.put(("ok", 1, res))
        ch.close()
    except Exception as e:  # noqa: BLE001
        q.put(("error", rank, repr(e)))


def test_recv_into_every_host_backend():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(2):
        status, rank, res = q.get(timeout=120)
        assert status == "ok", res
        out[rank] = res
    for p in ps:
        p.join(30)
    assert out[1] == [True, True, True, True], out[1]

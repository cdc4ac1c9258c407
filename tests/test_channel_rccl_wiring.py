"""Wiring of the direct-RCCL channel backend (``MPAMD_CHANNEL_DATA=rccl``) on the CPU: which
two-rank communicators every rank of a P-stage pipeline builds, in which order (a blocking init
must pair with the neighbour's FIRST init), and which pair / peer each hop uses.  The
communicators themselves are faked here; the real ones run in tests/test_rccl_gpu.py."""
import pytest
import torch

from src.parallel import channel as chmod
from src.parallel import rccl


class _FakeComm:
    log = []

    def __init__(self, store, prefix, rank, world, device, timeout_s=0):
        self.prefix, self.rank, self.world = prefix, rank, world
        _FakeComm.log.append((prefix, rank))


def _channel(rank, P, monkeypatch):
    monkeypatch.setattr(rccl, "RcclComm", _FakeComm)
    monkeypatch.setattr(torch.cuda, "Stream", lambda *a, **k: object())
    ch = chmod.Channel.__new__(chmod.Channel)
    ch.rank, ch.world, ch.device = rank, P, torch.device("cpu")
    ch._rc = {}
    _FakeComm.log = []
    ch._init_rccl(None, "p", 10.0)
    return ch, list(_FakeComm.log)


@pytest.mark.parametrize("P", [2, 3, 8])
def test_pairs_and_init_order(P, monkeypatch):
    inits = {}
    for r in range(P):
        ch, log = _channel(r, P, monkeypatch)
        inits[r] = log
        keys = set(ch._rc)
        want = set()
        if r > 0:
            want.add(("data", "recv"))
        if r < P - 1:
            want.add(("data", "send"))
        if r == 0:
            want.add(("ret", "recv"))
        if r == P - 1:
            want.add(("ret", "send"))
        assert keys == want
        # peers inside the two-rank communicators
        for (which, d), (comm, peer) in ch._rc.items():
            assert comm.world == 2 and peer == 1 - comm.rank
            assert (comm.rank == 0) == (d == "send")
    # every data pair is initialised by exactly its two ranks, each as its first data init
    for k in range(P - 1):
        pre = f"p/rdata/{k}"
        assert [r for r in range(P) if any(x[0] == pre for x in inits[r])] == [k, k + 1]
        assert inits[k + 1][0][0] == pre  # the receiver's first init pairs with the sender's
    # data pairs come in increasing k on every rank, the return pair last
    for r in range(P):
        names = [x[0] for x in inits[r]]
        data = [n for n in names if "/rdata/" in n]
        assert data == sorted(data, key=lambda n: int(n.rsplit("/", 1)[1]))
        if "p/rret" in names:
            assert names[-1] == "p/rret"


def test_hop_routing_checks_peer(monkeypatch):
    ch, _ = _channel(1, 3, monkeypatch)
    ch._rstreams = {k: None for k in ch._rc}
    comm, peer, _ = ch._rccl_pair("data", "send", 2)
    assert comm.prefix == "p/rdata/1" and peer == 1
    comm, peer, _ = ch._rccl_pair("data", "recv", 0)
    assert comm.prefix == "p/rdata/0" and peer == 0
    with pytest.raises(chmod.ChannelError):
        ch._rccl_pair("data", "send", 0)
    with pytest.raises(chmod.ChannelError):
        ch._rccl_pair("ret", "send", 0)  # only the tail returns tokens

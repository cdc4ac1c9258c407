"""Wire format, RPC, and the replicated TTL registry."""
import asyncio
import time

import pytest
import torch

from src import native
from src.comm.registry import DHT, get_dht_time
from src.comm.rpc import RemoteError, RpcClient, RpcServer, get_loop
from src.comm.wire import Message, encode, make_maddr, parse_peer_address, split_for_streaming


@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32,
                                torch.uint8, torch.bool])
def test_wire_roundtrip(dt):
    t = (torch.randn(3, 5, 7) * 10).to(dt)

    async def go():
        srv = await RpcServer("127.0.0.1", 0).start()

        async def echo(m):
            return Message({"x": m.metadata["x"] + 1}, m.tensors)

        srv.add_handler("echo", echo)
        cli = RpcClient()
        r = await cli.call(srv.maddrs[0], "echo", Message({"x": 41}, [t, t[0]]), timeout=5)
        big = torch.arange(300000, dtype=torch.float32).view(3000, 100)
        r2 = await cli.call(srv.maddrs[0], "echo", Message({"x": 0}, [big]), timeout=5, stream_chunk_bytes=65536)
        with pytest.raises(RemoteError):
            await cli.call(srv.maddrs[0], "nope", Message({}), timeout=5)
        await cli.close()
        await srv.shutdown()
        return r, r2, big

    r, r2, big = get_loop().run(go())
    assert r.metadata["x"] == 42 and torch.equal(r.tensors[0], t) and torch.equal(r.tensors[1], t[0])
    assert torch.equal(r2.tensors[0], big)


def test_frame_prefix_native_matches_python():
    hdr = b"abc" * 10
    assert native.pack_prefix(hdr, [1, 2, 3])[:12] == native.pack_prefix(hdr, [1, 2, 3])[:12]
    hl, n = native.unpack_fixed(native.pack_prefix(hdr, [5, 6])[:12])
    assert (hl, n) == (30, 2)
    with pytest.raises(Exception):
        native.unpack_fixed(b"\x00" * 12)


def test_addresses_and_split():
    assert parse_peer_address("/ip4/10.0.0.1/tcp/8000/p2p/QmX") == ("10.0.0.1", 8000, "QmX")
    assert parse_peer_address("127.0.0.1:9") == ("127.0.0.1", 9, None)
    assert parse_peer_address(make_maddr("1.2.3.4", 5, "id")) == ("1.2.3.4", 5, "id")
    with pytest.raises(ValueError):
        parse_peer_address("nohostport")
    parts = split_for_streaming(torch.zeros(100, 10), 400)
    assert sum(p.shape[0] for p in parts) == 100 and len(parts) == 10


def test_rpc_timeout_and_dead_peer():
    async def go():
        srv = await RpcServer("127.0.0.1", 0).start()

        async def slow(m):
            await asyncio.sleep(2)
            return Message({})

        srv.add_handler("slow", slow)
        cli = RpcClient()
        with pytest.raises(asyncio.TimeoutError):
            await cli.call(srv.maddrs[0], "slow", Message({}), timeout=0.2)
        addr = srv.maddrs[0]
        await srv.shutdown()
        with pytest.raises((ConnectionError, OSError, asyncio.TimeoutError)):
            await cli.call(addr, "slow", Message({}), timeout=1)
        await cli.close()

    get_loop().run(go())


def test_registry_replication_ttl_subkeys():
    a = DHT(start=True, sync_period=0.3)
    b = DHT(start=True, initial_peers=[a.address], sync_period=0.3)
    c = DHT(start=True, initial_peers=[b.address], sync_period=0.3)
    try:
        a.store("k", {"v": 1}, get_dht_time() + 30)
        b.store("mod", {"p": "b"}, get_dht_time() + 30, subkey="b")
        c.store("mod", {"p": "c"}, get_dht_time() + 30, subkey="c")
        deadline = time.time() + 5
        while time.time() < deadline and (a.get("mod") is None or len(a.get("mod").value) < 2):
            time.sleep(0.05)
        assert set(a.get("mod").value) == {"b", "c"}
        assert c.get("k").value == {"v": 1}
        # newer expiration wins, older is ignored
        assert a.store("k", {"v": 2}, get_dht_time() + 60)
        assert not b._merge("k", None, {"v": 0}, get_dht_time() + 1)
        # expiry
        a.store("short", 1, get_dht_time() + 0.2)
        time.sleep(0.4)
        assert b.get("short") is None and a.get("short") is None
        assert a.store("past", 1, get_dht_time() - 1) is False
        # late joiner converges from a snapshot
        d = DHT(start=True, initial_peers=[c.address], sync_period=0.3)
        assert set(d.get("mod").value) == {"b", "c"}
        d.shutdown()
    finally:
        for n in (a, b, c):
            n.shutdown()

"""Session placement over replicated pipelines (parallel/pipeline.py, failover.ReplicaRouter).

The multi-process pipeline protocol itself is covered by tests/test_engine_gloo.py (N stages
== 1 stage, slots S / S+1 / 2S, dead-stage detection), tests/test_router_gloo.py (replicas +
failover) and tests/test_bench_contract.py (pp2, pp2xdp2, pp2xtp2 through bench.py)."""
from src.parallel.failover import ReplicaRouter
from src.parallel.pipeline import assign_sessions


def test_assign_sessions_proportional():
    a = assign_sessions(10, [1.0, 1.0])
    assert a.count(0) == 5 and a.count(1) == 5
    a = assign_sessions(9, [2.0, 1.0])
    assert a.count(0) == 6 and a.count(1) == 3
    assert assign_sessions(3, [0.0, 0.0]).count(0) == 2


def test_place_one_follows_throughput_and_skips_dead():
    r = ReplicaRouter(3, throughputs=[2.0, 1.0, 1.0])
    got = [r.place_one(f"s{i}", [1]) for i in range(8)]
    assert got.count(0) == 4 and got.count(1) == 2 and got.count(2) == 2
    plans = r.fail(1)
    assert {p.replica for p in plans} <= {0, 2} and len(plans) == 2
    assert all(r.place_one(f"t{i}", [1]) != 1 for i in range(5))


def test_assign_sessions_capacity_redistributes_overflow():
    a = assign_sessions(12, [7.0, 5.0], capacity=6)
    assert a.count(0) == 6 and a.count(1) == 6
    a = assign_sessions(12, [10.0, 1.0, 1.0], capacity=5)
    assert [a.count(r) for r in range(3)] == [5, 4, 3] or sorted(a.count(r) for r in range(3)) == [3, 4, 5]
    assert len(a) == 12 and max(a.count(r) for r in range(3)) <= 5
    import pytest

    with pytest.raises(ValueError):
        assign_sessions(13, [1.0, 1.0], capacity=6)

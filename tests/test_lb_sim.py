"""Load-balancing simulator: the balancing rules keep the swarm near its upper bound."""
from src.lb_sim import SimServer, compare, simulate, swarm_throughput, upper_bound


def test_metrics():
    s = {"a": SimServer("a", 2.0, 2, 0), "b": SimServer("b", 3.0, 2, 2)}
    assert swarm_throughput(s, 4) == 2.0 and upper_bound(s, 4) == 2.5


def test_balancing_beats_random_and_full_recovers_from_departures():
    kw = dict(n_servers=12, total_blocks=24, blocks_range=(4, 8), leave_frac=0.34)
    res = compare(range(3), **kw)
    assert res["new"]["after_join"] > res["none"]["after_join"] + 0.3
    assert res["full"]["after_join"] > 0.6
    assert res["full"]["after_leave"] >= res["new"]["after_leave"]
    r = simulate("full", seed=1, **kw)
    assert r["servers"] == 12 - int(0.34 * 12) and 0 < r["after_leave"] <= 1.0 + 1e-9

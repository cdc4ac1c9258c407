#!/usr/bin/env python3
"""Manual fault-tolerance drill (reference scripts/test_fault_tolerance.py).

Start the servers (e.g. with two replicas of one stage), run this client, and kill the
replica in use mid-generation with ``scripts/kill_stage.py N``: the client re-routes, replays
the session's history into the survivor and keeps generating.  The automated version of
this drill is ``tests/test_swarm.py::test_failover_to_replica_replays_kv``.

    python scripts/test_fault_tolerance.py --dht_initial_peers /ip4/127.0.0.1/tcp/29802/p2p/<id>
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from src.main import main  # noqa: E402


if __name__ == "__main__":
    argv = sys.argv[1:]
    defaults = {"--model": "gpt2", "--splits": "6", "--stage": "0", "--max_new_tokens": "50", "--temperature": "0"}
    for k, v in defaults.items():
        if k not in argv:
            argv += [k, v]
    main(argv)

"""CLI surface parity with the reference (src/main.py:776-819) and the multi-process launcher."""
import os
import subprocess
import sys

import pytest

from src.main import build_parser

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REFERENCE_FLAGS = {
    "--model": None, "--splits": None, "--dtype": "fp16", "--max_new_tokens": 64, "--prompt": "Hello, how are you?",
    "--dht_initial_peers": "", "--public_ip": "", "--public_dht_port": None, "--public_rpc_port": None,
    "--dht_port": 8000, "--rpc_port": 8001, "--stage": None, "--request_timeout": 30.0, "--temperature": 1.0,
    "--top_p": 0.92, "--top_k": 50, "--use_cpu_offload": False, "--keep_layers_on_gpu": 0,
    "--use_load_balancing": False, "--num_blocks": None, "--total_blocks": None, "--balance_quality": 0.75,
    "--mean_balance_check_period": 120.0, "--network_bandwidth_mbps": None,
}


def test_reference_flags_and_defaults():
    args = build_parser().parse_args(["--model", "gpt2", "--splits", "6", "--stage", "1"])
    for flag, default in REFERENCE_FLAGS.items():
        name = flag[2:]
        assert hasattr(args, name), flag
        if default is not None:
            assert getattr(args, name) == default, (flag, getattr(args, name))


@pytest.mark.timeout(300)
def test_run_all_launcher_three_processes(tmp_path):
    r = subprocess.run([sys.executable, "scripts/run_all.py", "--model", "tiny-gpt2", "--splits", "1,2",
                        "--max_new_tokens", "6", "--base_port", "29930", "--log_dir", str(tmp_path)],
                       cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "GENERATED:" in r.stdout and "TTFT" in r.stdout
    assert "hop mini_petals:stage2" in r.stdout


def test_kill_stage_dry_run():
    r = subprocess.run([sys.executable, "scripts/kill_stage.py", "7", "--dry_run"], cwd=ROOT, capture_output=True,
                       text=True, timeout=60)
    assert "no stage 7 server found" in r.stdout


@pytest.mark.timeout(300)
def test_sigkill_replica_process_mid_decode(tmp_path):
    """Fault injection at process level (reference scripts/test_fault_tolerance.py + kill_stage.py):
    two OS processes serve stage 1; the one on the session's route is SIGKILLed mid-decode and the
    generation continues on the other replica with identical (greedy) output."""
    import re
    import signal
    import time

    import torch

    from tests.test_swarm import MODEL, _client, _generate, _reference

    def start(i, peers=None):
        log = tmp_path / f"s{i}.log"
        cmd = [sys.executable, "-m", "src.main", "--model", MODEL, "--splits", "2", "--stage", "1", "--dht_port", "0",
               "--rpc_port", "0", "--host", "127.0.0.1", "--device", "cpu", "--kv_cache_gb", "0.05",
               "--max_sessions", "8"]
        if peers:
            cmd += ["--dht_initial_peers", peers]
        p = subprocess.Popen(cmd, cwd=ROOT, stdout=open(log, "w"), stderr=subprocess.STDOUT)
        t0 = time.time()
        while time.time() - t0 < 120:
            txt = log.read_text()
            m = re.search(r"handlers registered .*peer (\S+),", txt)
            d = re.search(r"DHT visible multiaddrs: \['([^']+)'", txt)
            if m and d:
                return p, m.group(1), d.group(1)
            assert p.poll() is None, txt[-2000:]
            time.sleep(0.2)
        raise TimeoutError(txt[-2000:])

    p1, id1, maddr = start(1)
    p2, id2, _ = start(2, maddr)
    procs = {id1: p1, id2: p2}
    try:
        cfg, ex, tx = _client(maddr, [2])
        t0 = time.time()
        while time.time() - t0 < 30:
            if len(tx._candidates(tx.stage_keys[0])) == 2:
                break
            time.sleep(0.2)
        killed = []

        def kill_current(i):
            if i == 3:
                pid = tx.session_routes[next(iter(tx.session_routes))][0].peer_id
                procs[pid].send_signal(signal.SIGKILL)
                procs[pid].wait(10)
                killed.append(pid)

        gen = _generate(ex, tx, 10, kill_current)
        assert killed and tx.failed_peers
        assert gen == _reference(10)
        tx.shutdown()
    finally:
        for p in (p1, p2):
            if p.poll() is None:
                p.terminate()
                p.wait(10)


@pytest.mark.timeout(300)
def test_lb_swarm_recipe(tmp_path):
    """Reference scripts/elice_test_load_balancing.sh on one host: servers pick disjoint spans."""
    r = subprocess.run([sys.executable, "scripts/lb_swarm.py", "--model", "tiny-llama", "--servers", "3",
                        "--num_blocks", "1", "--splits", "1", "--base_port", "29970", "--log_dir", str(tmp_path)],
                       cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    spans = sorted(set(__import__("re").findall(r"Selected blocks \[(\d+), (\d+)\)", r.stdout)))
    assert spans == [("1", "2"), ("2", "3"), ("3", "4")], r.stdout
    assert "GENERATED:" in r.stdout


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_run_all_launcher_on_gpu_matches_single_process(tmp_path):
    """The reference's main flow on the GPU: two stage servers and the CLI client (stage 0) as
    separate processes on cuda:0 (all stages on one node: the client opens a device channel to
    them), greedy decoding; the text is a prefix of the single-process generator's
    (scripts/single_gpu_check.py, the reference's S4 tool) for the same synthetic weights - the
    CLI stops early on repeated tokens, as the reference client does (src/main.py:160-204).  Synthetic weights are
    seeded per device (the CUDA generator is not the CPU one), so GPU runs compare with GPU runs.
    Reference flow: src/main.py:776-819, scripts/run_all.py; single-GPU check:
    scripts/single_gpu_check.py."""
    import ast
    import re

    ref = subprocess.run([sys.executable, "scripts/single_gpu_check.py", "--model", "small-llama", "--max_new_tokens",
                          "12", "--device", "cuda"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert ref.returncode == 0, ref.stderr[-3000:]
    want = ast.literal_eval(re.search(r"Generated: (.*)", ref.stdout).group(1))
    r = subprocess.run([sys.executable, "scripts/run_all.py", "--model", "small-llama", "--splits", "2,4", "--gpus",
                        "--max_new_tokens", "12", "--base_port", "29890", "--log_dir", str(tmp_path),
                        "--extra", "--kv_cache_gb 1"], cwd=ROOT, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "TTFT" in r.stdout and ("device channel" in r.stdout or "hop mini_petals:stage2" in r.stdout), \
        r.stdout[-3000:]
    got = re.search(r"GENERATED: (.*?)\n={10,}", r.stdout, re.S).group(1)
    assert got and want.startswith(got), (got, want)

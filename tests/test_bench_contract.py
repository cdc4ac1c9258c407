"""bench.py's driver contract on CPU: torchrun multi-rank (gloo), rank 0 prints ONE JSON line
with the required keys; the pipeline (pp2), replica (pp2 x dp2) and tensor-parallel (pp2 x tp2)
layouts all complete."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


@pytest.mark.parametrize("nproc,extra,par,gb", [(2, [], "pp2", 6), (4, ["--replicas", "2"], "pp2xdp2", 12),
                                                (4, ["--tp", "2"], "pp2xtp2", 6)])
def test_bench_torchrun_gloo(nproc, extra, par, gb):
    port = 29650 + nproc
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", "bench.py", "--gpus", str(nproc), "--steps", "3",
           "--warmup", "1", "--model", "tiny-llama", "--device", "cpu", "--batch", "2", "--prompt-len", "8", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == nproc and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True and rec["scaling"] == "weak"
    assert rec["config"]["parallelism"] == par
    assert rec["config"]["global_batch"] == gb  # (stages + 1) slots x batch x replicas (TP lanes share)


def test_bench_spawns_its_own_ranks():
    """``python bench.py --gpus 2`` with no launcher: bench.py starts the two ranks itself, rank 0's
    JSON line is forwarded (data plane reported), the command exits 0."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--model", "tiny-llama",
           "--device", "cpu", "--batch", "2", "--prompt-len", "8"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec) and rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "pp2"
    assert rec["data_plane"].startswith("gloo") and rec["graph_hop"] is False
    # hop statistics cover exactly the timed steps: rank 0 sends one [B, H] bf16 hidden-state hop
    # per micro-batch slot per step (tiny-llama H = 256; M = stages + 1 = 3 slots, B = 2), nothing
    # from the prefill or warm-up rounds
    steps, M, B, H = 3, rec["config"]["micro_batches"], 2, 256
    assert rec["hop_sends_per_rank"][0] == steps * M
    assert rec["hop_bytes_sent_per_rank"][0] == steps * M * B * H * 2
    assert rec["hop_sends_per_rank"][1] == steps * M  # the tail's token returns
    assert rec["hop_bytes_sent_per_rank"][1] == steps * M * B * 8


def test_bench_spawn_fails_loudly():
    """A rank that dies makes the launcher exit non-zero (here: cut points for 4 stages on 2 ranks)."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--model", "tiny-llama",
           "--device", "cpu", "--batch", "1", "--prompt-len", "4", "--splits", "1,2,3"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def _spawn2(extra, timeout=240):
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--model", "tiny-llama",
           "--device", "cpu", "--batch", "2", "--prompt-len", "8", *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec) and rec["value"] > 0 and rec["data_plane"].startswith("gloo")  # the headline stands
    return rec


def test_bench_second_phase_same_tokens():
    """The second timed phase runs the same sessions on a second channel in the same processes and
    draws exactly the headline phase's tokens."""
    rec = _spawn2(["--phase2", "gloo"])
    p2 = rec["phase2"]
    assert p2["ok"] is True and p2["data_plane"].startswith("gloo"), p2
    assert p2["tokens_match_headline"] is True and p2["sessions_compared"] == 6
    assert p2["ms_per_step"] > 0 and p2["value"] > 0
    assert p2["hop_sends_per_rank"][0] == 3 * 3  # steps x slots, counted for the timed steps only


@pytest.mark.parametrize("extra,stage", [(["--phase2", "rccl"], "init"),
                                         (["--phase2", "gloo", "--phase2-inject", "init"], "init"),
                                         (["--phase2", "gloo", "--phase2-inject", "run", "--phase2-hop-timeout", "5"],
                                          None)])
def test_bench_second_phase_failure_keeps_headline(extra, stage):
    """A second phase that cannot set up its communicators (the RCCL data plane on a CPU run; an
    injected set-up error on one rank) or loses a rank mid-run is reported as ``phase2.ok = false``
    with its reason; the command still exits 0 with the headline numbers."""
    rec = _spawn2(extra)
    p2 = rec["phase2"]
    assert p2["ok"] is False and p2["reason"], p2
    if stage:
        assert p2["stage"] == stage

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

"""BASELINE config 5 as a runnable drill: ``bench.py --replicas 2 --kill RANK@STEPS`` (2 replicas x
2 stages, ranks spawned by bench.py itself so one rank's SIGKILL does not tear the others down).

* CPU (gloo, fp32 reference ops): every session finishes and every token equals the uninterrupted
  run's (``--drill`` without a kill) - the re-placed sessions included.
* GPU rehearsal on ONE MI355X (4 ranks on the card, payloads host-staged over gloo: RCCL refuses
  two ranks per device): every session finishes, the failed replica's sessions are re-placed, and
  every token a session had before the failure equals the uninterrupted run's.  After a
  re-placement the GPU logits differ in their last bits (the survivor runs another batch size, so
  another decode GEMM form, and rebuilds the KV by a prefill): the exactness contract there is
  the teacher-forced logit tolerance of ``test_failover_gpu.py``.
Reference FT loop: /root/reference/src/rpc_transport.py:587-712,
/root/reference/scripts/test_fault_tolerance.py:24-88, /root/reference/scripts/kill_stage.py:16-67."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _drill(tmp_path, name, extra, device, model, env_extra=None, timeout=300):
    dump = str(tmp_path / f"{name}.json")
    cmd = [sys.executable, "bench.py", "--gpus", "4", "--replicas", "2", "--model", model, "--device", device,
           "--batch", "2", "--prompt-len", "8", "--steps", "16", "--dump-tokens", dump, *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", MPAMD_DRILL_TIMEOUT="30", **(env_extra or {}))
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    with open(dump) as f:
        return json.loads(lines[0]), json.load(f)


def _check(ref, ref_dump, rec, dump, exact):
    fo = rec["failover"]
    assert rec["ms_per_step"] is not None and rec["ms_per_step"] > 0  # the pre-failure window's step time
    assert fo["failed_replicas"] == [1]
    assert fo["sessions_completed"] == fo["sessions_total"] == 12
    assert fo["sessions_replaced"] > 0 and fo["recovery_s"] is not None and fo["recovery_s"] < 30
    assert ref["failover"]["failed_replicas"] == [] and ref["failover"]["sessions_completed"] == 12
    assert set(dump["replaced"]) <= set(dump["tokens"])
    for rid, toks in dump["tokens"].items():
        want = ref_dump["tokens"][rid]
        assert len(toks) == len(want) == 16
        n = dump["at_failure"][rid]
        assert toks[:n] == want[:n], rid  # every token produced before the failure is unchanged
        if exact:
            assert toks == want, rid


@pytest.mark.timeout(900)
def test_failover_drill_cpu_exact(tmp_path):
    ref, ref_dump = _drill(tmp_path, "ref", ["--drill"], "cpu", "tiny-llama")
    rec, dump = _drill(tmp_path, "kill", ["--kill", "3@10"], "cpu", "tiny-llama")
    _check(ref, ref_dump, rec, dump, exact=True)


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_failover_drill_one_gpu_rehearsal(tmp_path):
    env = dict(MPAMD_DIST_BACKEND="gloo", MPAMD_CHANNEL_DATA="gloo", MPAMD_KV_GB="1", MPAMD_GEMM_AUTOTUNE="0")
    ref, ref_dump = _drill(tmp_path, "ref", ["--drill"], "cuda", "small-llama", env)
    rec, dump = _drill(tmp_path, "kill", ["--kill", "3@10"], "cuda", "small-llama", env)
    _check(ref, ref_dump, rec, dump, exact=False)
    same = sum(dump["tokens"][k] == ref_dump["tokens"][k] for k in dump["tokens"])
    print(f"failover drill (1-GPU rehearsal): {json.dumps(rec['failover'])}; sessions identical end to end: "
          f"{same}/{len(dump['tokens'])}")

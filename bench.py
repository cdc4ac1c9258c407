#!/usr/bin/env python3
"""Flagship benchmark: whole-node decode tokens/s + per-stage ms, Llama-2-7B split over N stages.

Metric/config from BASELINE.json: "tokens/sec (whole node) + per-stage ms, Llama-7B split
over 1/2/4/8 stages".  One process per GPU (torchrun); rank r serves an even contiguous block
range of Llama-2-7B (bf16, synthetic random-init weights: no checkpoints on the box), hidden
states hop stage->stage over RCCL (xGMI), the last stage samples server-side with the
reference CLI's defaults (temperature 1.0, top_p 0.92, top_k 50, repetition penalty 1.5) and
returns token ids to rank 0.

Work per GPU is fixed as N grows ("weak" scaling): N+1 micro-batches x --batch sessions are in
flight (one slot of slack for the token hop), so every GPU processes N+1 micro-batch ticks of
its 32/N blocks per step (continuous-batching engine, parallel/engine.py).  A step
advances every session by one token; value = generated tokens/s over the whole node.

    python bench.py                       # N=1 (defaults finish in ~1-2 minutes)
    python bench.py --gpus N              # spawns the N ranks itself (no launcher needed)
    torchrun --nproc-per-node N bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import sys
import time
from typing import Optional

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "tokens/sec (whole node) + per-stage ms, Llama-7B split over 1/2/4/8 stages"


def baseline_value(batch: int = 64):
    """Reference-equivalent per-GPU tokens/s recorded in BASELINE.json (a measured run) at THIS
    batch: the same-batch number at its batch (64), the batch-1 number at 1, None otherwise."""
    try:
        with open(os.path.join(HERE, "BASELINE.json")) as f:
            m = json.load(f).get("measured_reference_equivalent", {})
    except Exception:
        return None
    if batch == 1:
        v = m.get("batch1_decode_tokens_per_s")
    elif batch == int(m.get("batch", 64)):
        v = m.get("decode_tokens_per_s_same_batch")
    else:
        v = None
    return float(v) if v else None


def data_plane_name(ch, eng) -> str:
    if ch is None:
        return "none"
    b = getattr(ch, "data_backend", "")
    if b == "rccl":
        return "rccl-graph-hop" if getattr(eng, "graph_hop", False) else "rccl-direct"
    if b == "nccl":
        return "pgnccl"
    return "gloo" + ("(host-staged)" if getattr(ch, "staged", False) else "")


def fp8_label(ex) -> str:
    """The precision path the executor actually runs for fp8 weights."""
    if getattr(ex, "_mx", False):
        return "fp8-w8a8-mx (e4m3 weights; o projection on MX e4m3 activations with e8m0 block scales, others bf16)"
    if getattr(ex, "_w8", False):
        return "fp8-w8a16 (e4m3 weights, bf16 activations/KV)"
    return "fp8-w8a8 (e4m3 weights and activations, bf16 KV)"


def run_failover_drill(a, cfg, eng, ex, rank, world, S, R, M, B, device, load_s):
    """BASELINE config 5 as a runnable drill: R replica pipelines of S stages; global rank 0 (replica
    0's head) runs the replica front end (parallel/router.py ReplicaFrontend) with host links to the
    other heads (serve_replica_head); stage rank K is SIGKILLed after running N micro-batch steps;
    the front end marks its replica dead and re-places the unfinished sessions on the survivors
    (re-prefill of prompt + generated tokens).  Reference FT loop: /root/reference/src/
    rpc_transport.py:587-712, /root/reference/scripts/test_fault_tolerance.py:24-88,
    /root/reference/scripts/kill_stage.py:16-67.  No collective runs after the kill (a dead rank
    would hang it): every rank leaves with os._exit."""
    import signal

    from torch.distributed import distributed_c10d as c10d

    from src.parallel.channel import HostLink
    from src.parallel.engine import PipelineFailure, Request
    from src.parallel.router import ReplicaFrontend, gather_replica_throughput, serve_replica_head
    from src.runtime.sampler import SamplingParams

    kill_rank, _, kill_steps = (a.kill or "-1@0").partition("@")
    kill_rank, kill_steps = int(kill_rank), int(kill_steps or 8)
    if a.kill and (not (0 < kill_rank < world) or kill_rank % S == 0):
        raise SystemExit(f"--kill {a.kill}: pick a non-head stage rank (rank % {S} != 0)")
    store = c10d._get_default_store()
    lane, stage = rank // S, rank % S
    link = HostLink(store, "bench/all", rank, world, timeout_s=600.0)
    thr = gather_replica_throughput(link, ex, lane, stage, R, batch=min(B, 16))
    link.close()
    timeout = float(os.environ.get("MPAMD_DRILL_TIMEOUT", "60"))
    code = 0
    if rank == 0:
        links = {r: HostLink(store, f"bench/link{r}", 0, 2, timeout_s=timeout) for r in range(1, R)}
        fe = ReplicaFrontend(R, eng, links, throughputs=thr, timeout_s=timeout)
        sp = SamplingParams(a.temperature, a.top_p, a.top_k, a.repetition_penalty)
        gen = torch.Generator().manual_seed(1234)
        n_total = R * M * B
        reqs = []
        stamps = []  # (time, rid) of every delivered token
        for i in range(n_total):
            prompt = torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=gen).tolist()
            reqs.append(fe.submit(Request(prompt, max_new_tokens=a.steps, params=sp, stop_on_repeat=0,
                                          seed=a.seed * 1000003 + i, rid=f"s{i}")))
        fe.on_token = lambda req, t: stamps.append((time.perf_counter(), req.rid))
        t0 = time.perf_counter()
        fe.run()
        t1 = time.perf_counter()
        fails = list(fe.failures)
        t_fail = fe.failure_times[0] if fails else None
        moved = {reqs[k].rid for k in fe.replaced}
        before = sum(1 for ts, _ in stamps if t_fail is None or ts < t_fail)
        rec = [ts for ts, rid in stamps if t_fail is not None and ts >= t_fail and rid in moved]
        t_rec = rec[0] if rec else None
        after = sum(1 for ts, _ in stamps if t_rec is not None and ts >= t_rec)
        done = sum(1 for r in reqs if r.done and len(r.generated) >= a.steps)
        total_tokens = sum(len(r.generated) for r in reqs)
        # ms per decode step of the pre-failure window (every session advances one token per step):
        # wall time before the kill / tokens delivered per session in it; the whole drill without a kill
        win_s, win_tok = ((t_fail - t0), before) if t_fail is not None else ((t1 - t0), total_tokens)
        ms_step = round(1000.0 * win_s / (win_tok / n_total), 3) if win_tok else None
        out = {
            "metric": METRIC, "value": round(total_tokens / (t1 - t0), 2), "unit": "tokens/s", "n_gpus": world,
            "steps": a.steps, "warmup": 0, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": fp8_label(ex) if a.fp8 else "bf16",
            "data": f"synthetic (random-init {cfg.name} weights, random prompt ids)",
            "config": {"model": cfg.name, "global_batch": n_total, "seq_len": a.prompt_len,
                       "parallelism": f"pp{S}xdp{R}", "micro_batches": M, "sessions_per_micro_batch": B,
                       "engine": "ReplicaFrontend over PipelineServingEngine replicas (failover drill)"},
            "failover": {
                "killed_rank": kill_rank, "kill_after_steps": kill_steps,
                "failed_replicas": [f[0] for f in fails], "failure_reasons": [f[1] for f in fails],
                "sessions_total": n_total, "sessions_completed": done, "sessions_replaced": len(moved),
                "tokens_per_s_before": round(before / (t_fail - t0), 2) if t_fail else None,
                "tokens_per_s_after": round(after / max(t1 - t_rec, 1e-9), 2) if t_rec else None,
                "recovery_s": round(t_rec - t_fail, 4) if (t_rec and t_fail) else None,
                "drill_s": round(t1 - t0, 3),
            },
            "load_s": round(load_s, 1),
        }
        print(json.dumps(out), flush=True)
        if a.dump_tokens:  # per session: tokens, and for re-placed ones how many preceded the failure
            with open(a.dump_tokens, "w") as f:
                json.dump({"tokens": {r.rid: list(r.generated) for r in reqs},
                           "replaced": {reqs[k].rid: n for k, n in fe.replaced.items()},
                           "at_failure": {reqs[k].rid: n for k, n in fe.at_failure.items()}}, f)
        code = 0 if done == n_total else 3
    elif stage == 0:
        link = HostLink(store, f"bench/link{lane}", 1, 2, timeout_s=timeout)
        serve_replica_head(eng, link, timeout_s=timeout)
    elif rank == kill_rank:
        try:
            for _ in range(kill_steps):
                if not eng._stage_step():
                    break
        finally:
            os.kill(os.getpid(), signal.SIGKILL)
    else:
        try:
            eng.serve()
        except PipelineFailure:
            pass  # a stage of the failed replica: its neighbour died
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _drill_victim(argv):
    """The rank a ``--kill RANK@STEPS`` drill kills on purpose (its SIGKILL is not a failure)."""
    for i, v in enumerate(argv):
        spec = v.split("=", 1)[1] if v.startswith("--kill=") else (argv[i + 1] if v == "--kill" and i + 1 < len(argv)
                                                                  else None)
        if spec:
            return int(spec.partition("@")[0])
    return None


def spawn_ranks(n: int, argv) -> int:
    """``--gpus N`` without a launcher (no WORLD_SIZE in the environment): start the N ranks as
    child processes here - one per GPU, torchrun's environment contract (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT) - forward rank 0's stdout (the one JSON
    line) and return non-zero if any rank fails, after stopping the others.  Runs before this
    process touches the GPU (no ``torch.cuda`` call here).  Reference launcher:
    /root/reference/scripts/run_all.py:164-208 (one subprocess per stage, logs streamed)."""
    import signal
    import subprocess

    port = _free_port()
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", ROLE_RANK="0")
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), ROLE_WORLD_SIZE=str(n))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno(), start_new_session=True))
    rc = 0
    victim = _drill_victim(argv)
    try:
        while True:
            codes = [p.poll() for p in procs]
            if victim is not None and codes[victim] == -signal.SIGKILL:
                codes[victim] = 0  # the drill's own kill
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                rc = bad[0][1] or 1
                print(f"bench: rank {bad[0][0]} exited with {bad[0][1]}; stopping the other ranks", file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                return 0
            time.sleep(0.2)
    except KeyboardInterrupt:
        rc = 130
    for p in procs:  # only the process groups started above
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + 20
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
    return rc if rc > 0 else 1


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=None)
    known, _ = pre.parse_known_args(argv)
    if known.gpus and known.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(spawn_ranks(known.gpus, argv))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batch", type=int, default=64, help="sessions per micro-batch")
    ap.add_argument("--micro", type=int, default=None, help="micro-batches in flight (default: stages + 1, or 1 on one GPU)")
    ap.add_argument("--replicas", type=int, default=1,
                    help="independent pipelines (data parallel): N GPUs = replicas x stages, e.g. 8 = 2 x 4")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--top-p", type=float, default=0.92)
    ap.add_argument("--top-k", type=int, default=50)
    ap.add_argument("--repetition-penalty", type=float, default=1.5)
    ap.add_argument("--gemm", default=os.environ.get("MPAMD_GEMM", "auto"), choices=["auto", "native", "hipblaslt"])
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree inside each stage (RCCL all-reduce after o / down)")
    ap.add_argument("--fp8", action="store_true",
                    help="fp8 (OCP e4m3) projection weights (the 70B config): W8A16 by default, W8A8 with "
                         "MPAMD_FP8_MODE=w8a8")
    ap.add_argument("--splits", default="auto",
                    help="'auto' (cost-balanced: lm_head + sampler weigh on the tail, partition.balanced_splits), "
                         "'even', or explicit cut points")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default=None)
    ap.add_argument("--kill", default=None, metavar="RANK@STEPS",
                    help="replica failover drill (BASELINE config 5): SIGKILL this stage rank after it has run STEPS "
                         "micro-batch steps; replica 0's head routes the sessions (ReplicaFrontend), re-places the "
                         "failed replica's sessions on the survivors, and the JSON reports tokens/s before / after, "
                         "recovery seconds and sessions completed.  Ranks are this launcher's own children")
    ap.add_argument("--drill", action="store_true",
                    help="run the failover drill's front end without killing anyone (the uninterrupted reference)")
    ap.add_argument("--dump-tokens", default=None, help="drill: write every session's tokens (JSON) here")
    ap.add_argument("--channel-data", default=os.environ.get("MPAMD_CHANNEL_DATA", "auto"),
                    choices=["auto", "nccl", "rccl", "gloo"],
                    help="stage-hop data plane: ProcessGroupNCCL (nccl, the GPU default), the framework's own "
                         "RCCL communicators (rccl; + MPAMD_GRAPH_HOP=1 records the hop inside the decode graph), "
                         "or host-staged gloo")
    ap.add_argument("--phase2", default="auto", choices=["auto", "off", "rccl", "nccl", "gloo"],
                    help="after the headline phase, a second timed phase of the same pipelines on another stage-hop "
                         "data plane, in the same processes: auto = the framework's RCCL communicators with the hop "
                         "recorded in the decode graphs (rccl + graph hop) whenever the headline ran on "
                         "ProcessGroupNCCL with >= 2 stages; reported under 'phase2' (ok or the failure reason), "
                         "never replacing the headline value")
    ap.add_argument("--phase2-timeout", type=float, default=180.0,
                    help="wall-clock bound of the second phase: past it every rank leaves (rank 0 printing the "
                         "headline line with phase2 = timeout)")
    ap.add_argument("--phase2-hop-timeout", type=float, default=60.0,
                    help="second phase: timeout of every channel wait (a dead or stuck peer becomes a failure)")
    ap.add_argument("--phase2-recv-into", default="on", choices=["on", "off"],
                    help="second phase: receive decode hops straight into the graph input (on) or through a "
                         "receive slab + copy (off) - with the headline on, 'off' checks both give the same tokens")
    ap.add_argument("--phase2-inject", default="none", choices=["none", "init", "run"],
                    help="test hook: make the second phase fail on the last stage rank at communicator set-up "
                         "(init) or in the middle of its timed steps (run)")
    a = ap.parse_args(argv)

    from src import ops
    from src.models.config import resolve_model
    from src.models.weights import random_stage_weights
    from src.parallel import dist as pdist
    from src.parallel.channel import Channel
    from src.parallel.engine import PipelineServingEngine, Request
    from src.parallel.tensor_parallel import make_tp_groups, shard_stage_weights
    from src.partition import balanced_splits, even_splits, parse_splits, stage_ranges
    from src.runtime.executor import StageExecutor
    from src.runtime.sampler import SamplingParams

    dev_type = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    rank, world, local, device = pdist.init_distributed(dev_type)
    n = a.gpus or world
    if n != world:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}: launch with torchrun --nproc-per-node {n}")
    ops.set_gemm_policy(a.gemm)
    cfg = resolve_model(a.model)
    R = max(1, a.replicas)
    if world % R:
        raise SystemExit(f"--replicas {R} does not divide {world} GPUs")
    TP = max(1, a.tp)
    if world % (R * TP):
        raise SystemExit(f"--replicas {R} x --tp {TP} does not divide {world} GPUs")
    S = world // (R * TP)
    tpg = make_tp_groups(world, S, TP, device=device)
    stage = rank % S
    lane = rank // S                      # pipeline index: replica * TP + tensor-parallel shard
    M = a.micro or (S + 1 if S > 1 else 1)  # one slot of slack for the token-return hop
    B = a.batch
    if a.splits == "auto":
        cuts = balanced_splits(cfg, S, batch=B, ctx=a.prompt_len + (a.warmup + a.steps) // 2, fp8=a.fp8)
    elif a.splits == "even":
        cuts = even_splits(cfg.num_hidden_layers, S)
    else:
        cuts = parse_splits(a.splits, cfg.num_hidden_layers)
        if len(cuts) != S - 1:
            raise SystemExit(f"--splits {a.splits} defines {len(cuts) + 1} stages, the run has {S}")
    start, end = stage_ranges(cuts, cfg.num_hidden_layers)[stage]
    dtype = torch.bfloat16
    t0 = time.time()
    w = random_stage_weights(cfg, start, end, has_embed=stage == 0, has_head=stage == S - 1, device=device,
                             dtype=dtype, seed=a.seed, fp8=a.fp8 and TP == 1)
    if TP > 1:  # shard the stage's blocks over the TP group (fp8: quantize the shard)
        w = shard_stage_weights(w, lane % TP, TP)
        if a.fp8:
            w.quantize_fp8()
    rounds = 2 + a.warmup + a.steps
    max_len = a.prompt_len + rounds + 8
    max_len = 64 * math.ceil(max_len / 64)
    kv_bytes = None if device.type == "cuda" else 256 << 20
    if os.environ.get("MPAMD_KV_GB"):  # cap the KV pool (e.g. several ranks sharing one GPU in a rehearsal)
        kv_bytes = int(float(os.environ["MPAMD_KV_GB"]) * (1 << 30))
    ex = StageExecutor(w.cfg, w, device, dtype=dtype, max_sessions=M * B + 8, max_seq_len=max(max_len, 256),
                       kv_cache_bytes=kv_bytes, use_graphs=not a.no_graphs, graph_max_batch=max(B, 1),
                       max_tokens_per_step=max(B * a.prompt_len, B), tp=tpg)
    if rank == 0 and device.type == "cuda":
        print("gemm kernel choice:", {f"M{k[0]}:N{k[1]}xK{k[2]}e{k[3]}": v
                                                   for k, v in sorted(ops._SK_CHOICE.items())}, file=sys.stderr)
        if ops._FP8_CHOICE:
            print("fp8 gemm kernel choice:", {f"M{k[0]}:N{k[1]}xK{k[2]}e{k[3]}": v
                                              for k, v in sorted(ops._FP8_CHOICE.items())}, file=sys.stderr)
        if ops._W8_CHOICE:
            print("w8a16 gemm kernel choice:", {f"M{k[0]}:N{k[1]}xK{k[2]}e{k[3]}": v
                                                for k, v in sorted(ops._W8_CHOICE.items())}, file=sys.stderr)
    ch = None
    if S > 1:  # this pipeline's device channel: ranks [lane*S, (lane+1)*S) over RCCL / xGMI
        from torch.distributed import distributed_c10d as c10d

        ch = Channel(c10d._get_default_store(), f"bench/pipe{lane}", stage, S, device, timeout_s=600.0,
                     data_backend=None if a.channel_data == "auto" else a.channel_data)
    eng = PipelineServingEngine(ex, ch, n_slots=M, batch=B, max_step_tokens=B * a.prompt_len, name=f"p{lane}")
    eng.freeze_heap = True  # a driver process: freeze the setup heap once before the first step
    if a.kill or a.drill:
        if R < 2 or TP != 1:
            raise SystemExit("--kill needs --replicas >= 2 (and no --tp): a failover needs a survivor")
        run_failover_drill(a, cfg, eng, ex, rank, world, S, R, M, B, device, time.time() - t0)
        return
    n_sessions = M * B
    if R > 1:
        # replica placement from measured throughput: every rank times its stage's decode step,
        # the node all-gathers them (host control group) and the sessions are split in
        # proportion to each replica's slowest stage (parallel/router.py, parallel/pipeline.py)
        from torch.distributed import distributed_c10d as c10d

        from src.parallel.channel import HostLink
        from src.parallel.failover import ReplicaRouter
        from src.parallel.router import gather_replica_throughput

        link = HostLink(c10d._get_default_store(), "bench/all", rank, world, timeout_s=600.0)
        thr = gather_replica_throughput(link, ex, lane // TP, stage, R, batch=min(B, 16))
        # the replica front end's online placement (ReplicaRouter.place_one: lowest
        # throughput-normalised load), capped at a pipeline's M slots x B sessions
        router = ReplicaRouter(R, thr)
        counts = [0] * R
        for i in range(M * B * R):
            r = router.place_one(f"s{i}", [])
            if counts[r] >= M * B:  # full: the next-best replica with room takes it
                r = min((k for k in range(R) if counts[k] < M * B),
                        key=lambda k: ((counts[k] + 1) / max(thr[k], 1e-9), k))
                router.placement[f"s{i}"] = r
            counts[r] += 1
        n_sessions = counts[lane // TP]
        link.close()
        if rank == 0:
            print(f"replica throughput (tok/s, probe batch {min(B, 16)}): {[round(t, 1) for t in thr]} -> "
                  f"sessions {counts}", file=sys.stderr)
    reqs1 = []
    sp = SamplingParams(a.temperature, a.top_p, a.top_k, a.repetition_penalty)
    if stage == 0:
        # synthetic requests: every pipeline of a TP group submits the same ones (same seeds),
        # so its shards take identical scheduling decisions and sample identical tokens
        gen = torch.Generator().manual_seed(1234 + (lane // TP))
        for i in range(n_sessions):
            prompt = torch.randint(0, cfg.vocab_size, (a.prompt_len,), generator=gen).tolist()
            reqs1.append(eng.submit(Request(prompt, max_new_tokens=rounds + 8, params=sp, stop_on_repeat=0,
                                            seed=a.seed * 1000003 + (lane // TP) * 7919 + i, rid=f"s{i}")))
    load_s = time.time() - t0

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()

    # prefill (TTFT of the whole batch through the pipeline) + first decode round (graph capture),
    # timed separately as well; the one-time heap freeze (a full collection, ~45 ms) is setup,
    # done before the clock starts rather than inside the first round
    eng._settle_heap()
    pdist.barrier(device)
    sync()
    tp0 = time.perf_counter()
    eng.run_rounds(1)
    sync()
    pdist.barrier(device)
    tp1 = time.perf_counter()
    eng.run_rounds(1)
    sync()
    pdist.barrier(device)
    prefill_s = time.perf_counter() - tp0
    prefill_only_s = pdist.all_max(tp1 - tp0, device)

    eng.run_rounds(a.warmup)
    sync()
    pdist.barrier(device)
    sync()
    if ch is not None:
        ch.stats(reset=True)
        ch.timing = True
    gc_runs = [0, 0, 0]  # collections per generation inside the timed window (host-side stalls)

    def _gc_cb(phase, info):
        if phase == "start":
            gc_runs[info["generation"]] += 1

    gc.callbacks.append(_gc_cb)
    t1 = time.perf_counter()
    eng.timing = True
    eng.run_rounds(a.steps)
    sync()
    pdist.barrier(device)
    sync()
    dt_local = time.perf_counter() - t1
    gc.callbacks.remove(_gc_cb)
    eng.timing = False
    if ch is not None:
        ch.timing = False
    stage_ms = eng.stage_ms() or 0.0
    recv_into = (eng.recvs_into, eng.recvs)  # (into a graph input, all) payload receives, whole run
    hop = ch.stats() if ch is not None else {"backend": "none", "bytes_sent": 0, "sends": 0, "recv_wait_ms": 0.0}
    data_plane = data_plane_name(ch, eng)
    n_tokens = 0
    if stage == 0:
        eng.drain()
        n_tokens = eng.tokens_generated
        if any(r.done for r in eng.finished):
            raise SystemExit("a benchmark session finished early: the timed rounds would be short of work")
        eng.stop()
    else:
        eng.serve()  # until the head's STOP
    if ch is not None:
        ch.close()
    dt = pdist.all_max(dt_local, device)
    counted = float(n_sessions) if (stage == 0 and lane % TP == 0) else 0.0  # TP lanes mirror one replica
    per_stage = pdist.all_gather_floats([stage_ms, float(end - start), counted, float(hop["bytes_sent"]),
                                         float(hop["sends"]), float(hop["recv_wait_ms"]), float(recv_into[0]),
                                         float(recv_into[1])], device)
    global_batch = int(sum(p[2] for p in per_stage))
    n_sessions_total = global_batch
    tokens = a.steps * global_batch  # every session advances one token per round
    value = tokens / dt
    # the baseline is a Llama-2-7B bf16 number at batch 64 (and 1)
    base = baseline_value(B) if a.model == "llama2-7b" and not a.fp8 else None
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * dt / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / (base * world), 3) if base else None),
            "baseline_tokens_per_s_per_gpu": base,
            "dtype": fp8_label(ex) if a.fp8 else "bf16",
            "data": f"synthetic (random-init {cfg.name} weights, random prompt ids)",
            "config": {
                "model": {"llama2-7b": "Llama-2-7B", "llama3-70b": "Llama-3-70B", "llama3-8b": "Llama-3-8B"}.get(
                    a.model, a.model),
                "global_batch": global_batch,
                "seq_len": a.prompt_len,
                "parallelism": f"pp{S}" + (f"xtp{TP}" if TP > 1 else "") + (f"xdp{R}" if R > 1 else ""),
                "micro_batches": M,
                "engine": "PipelineServingEngine (continuous batching, device channel)",
                "sessions_per_micro_batch": B,
                "splits": cuts,
                "sampling": {"temperature": a.temperature, "top_p": a.top_p, "top_k": a.top_k,
                             "repetition_penalty": a.repetition_penalty},
                "gemm": a.gemm,
                "graphs": not a.no_graphs,
            },
            "per_stage_ms": [round(p[0], 3) for p in per_stage],
            "per_stage_blocks": [int(p[1]) for p in per_stage],
            "gc_collections_timed": gc_runs,
            # the device channel of every pipeline: which backend carried the hops (RCCL over
            # xGMI on a multi-GPU node), payload bytes each rank sent during the timed steps,
            # and how long each rank's stream waited for its incoming payload per step
            "channel_backend": hop["backend"],
            # which data plane carried the stage hops: pgnccl (ProcessGroupNCCL send/recv),
            # rccl-direct (framework RCCL communicators on a side stream), rccl-graph-hop (the
            # send recorded inside every decode hipGraph), gloo (host), none (one stage)
            "data_plane": data_plane,
            "graph_hop": bool(getattr(eng, "graph_hop", False)),
            "hop_bytes_sent_per_rank": [int(p[3]) for p in per_stage],
            "hop_sends_per_rank": [int(p[4]) for p in per_stage],
            "hop_recv_wait_ms_per_rank": [round(p[5], 4) for p in per_stage],
            # payload receives that landed straight in the static input of the decode graph the step
            # replayed, per rank: [into graph input, all receives] over the whole run (decode steps
            # only: prefill chunks run eagerly, so they always take a receive slab)
            "hop_recv_into_graph_per_rank": [[int(p[6]), int(p[7])] for p in per_stage],
            # the qkv fold per decode row bucket, as the warm-up's decode-graph A/B left it
            "qkv_fold": {f"M{k}": bool(v) for k, v in sorted(ex.qkv_fold_by_bucket.items())},
            # the warm-up A/B behind it: (folded, unfolded) ms per step
            "qkv_fold_ab_ms": {f"M{k}": v for k, v in sorted(getattr(ex, "qkv_fold_ab_ms", {}).items())},
            # the decode-kernel mix: the committed table (ops/tuned/decode_kernels_gfx950.json) this run
            # loaded, the sha of the choices it actually ran, and any shape it had to time itself
            **{k: v for k, v in ops.kernel_table_report().items()},
            "prefill_plus_first_token_s": round(prefill_s, 3),
            # the prefill round alone: every session's prompt through the whole pipeline
            # (micro-batch slots x batch x prompt-len tokens), max over ranks
            "prefill_round_s": round(prefill_only_s, 4),
            "prefill_tokens_per_s": round(n_sessions_total * a.prompt_len / max(prefill_only_s, 1e-9), 1),
            "load_s": round(load_s, 1),
        }
    p2 = phase2_backend(a, S, R, TP, device, data_plane)
    if p2 is not None:
        ctx = dict(ex=ex, rank=rank, world=world, S=S, stage=stage, lane=lane, M=M, B=B, device=device,
                   rounds=rounds, reqs1=reqs1, sp=sp)
        guard = _Phase2Guard(a.phase2_timeout, rec if rank == 0 else None)
        phase2 = run_phase2(a, p2, ctx)
        if rank == 0:
            rec["phase2"] = phase2
            guard.print_once(rec)
        guard.cancel()
    elif rank == 0:
        print(json.dumps(rec), flush=True)
    pdist.shutdown()


def phase2_backend(a, S, R, TP, device, data_plane):
    """The second phase's data plane, or None: only pure pipelines (no replicas / TP)."""
    if a.phase2 == "off" or S < 2 or R != 1 or TP != 1:
        return None
    if a.phase2 == "auto":
        return "rccl" if (device.type == "cuda" and data_plane == "pgnccl") else None
    return a.phase2


class _Phase2Guard:
    """Wall-clock bound of the second phase: a peer stuck inside a device wait (an RCCL receive that
    never completes blocks ``torch.cuda.synchronize``) must not cost the run its headline line.  Past
    the deadline rank 0 prints the headline record with ``phase2 = timeout`` and every rank leaves
    with exit code 0 (no exec, no GPU call from this thread)."""

    def __init__(self, limit_s: float, rec: Optional[dict]):
        import threading

        self.rec = rec
        self.printed = False
        self.lock = threading.Lock()
        self.timer = threading.Timer(max(1.0, float(limit_s)), self._fire)
        self.timer.daemon = True
        self.timer.start()

    def print_once(self, rec: dict) -> None:
        with self.lock:
            if not self.printed:
                self.printed = True
                print(json.dumps(rec), flush=True)

    def _fire(self) -> None:
        if self.rec is not None:
            out = dict(self.rec)
            out["phase2"] = {"ok": False, "stage": "timeout",
                             "reason": "the second phase did not finish within --phase2-timeout"}
            self.print_once(out)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)

    def cancel(self) -> None:
        self.timer.cancel()


def run_phase2(a, backend: str, ctx: dict) -> dict:
    """Second timed phase: the same pipeline, the same synthetic sessions (same prompts and seeds,
    so the same tokens), on another stage-hop data plane - by default the designed one, the
    framework's own RCCL communicators with every hop recorded inside the sender's decode graph
    and received straight into the receiver's graph input (the reference hop it
    replaces: /root/reference/src/rpc_transport.py:738-766).  Built only after the headline phase
    has been timed and reported; every wait is bounded (channel timeouts, the host agreement link,
    ``_Phase2Guard``), a failure aborts this phase's communicators and is reported, never raised.
    Returns the phase's record (rank 0's is the one printed)."""
    from torch.distributed import distributed_c10d as c10d

    from src.parallel.channel import Channel, HostLink
    from src.parallel.engine import PipelineServingEngine, Request

    ex, rank, world, S, stage, lane = ctx["ex"], ctx["rank"], ctx["world"], ctx["S"], ctx["stage"], ctx["lane"]
    M, B, device = ctx["M"], ctx["B"], ctx["device"]
    store = c10d._get_default_store()
    link = HostLink(store, "bench/p2ctl", rank, world, timeout_s=max(30.0, 2 * a.phase2_hop_timeout))

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()

    def agree(vals):
        return link.all_gather_floats([float(v) for v in vals])

    out = {"data_plane": None, "ok": False}
    ch2 = eng2 = None
    ok, reason, where = 1.0, "", "init"
    try:
        with ex.exec_lock:  # the headline phase's sessions (never finished) give their rows / pages back
            for sid in list(ex.sessions.sessions):
                ex.sessions.close(sid)
        if a.phase2_inject == "init" and stage == S - 1:
            raise RuntimeError("injected communicator set-up failure (--phase2-inject init)")
        if backend == "rccl":
            os.environ["MPAMD_GRAPH_HOP"] = "1"  # record the send in the decode graphs (every stage agrees)
        ch2 = Channel(store, f"bench/p2pipe{lane}", stage, S, device, timeout_s=a.phase2_hop_timeout,
                      data_backend=backend)
    except Exception as e:  # noqa: BLE001 - reported in the JSON, never fatal to the headline
        ok, reason = 0.0, f"rank {rank}: {type(e).__name__}: {e}"
    try:
        allv = agree([ok])
    except Exception as e:  # noqa: BLE001
        allv, reason = [[0.0]], reason or f"rank {rank}: agreement failed: {e}"
    if not all(v[0] for v in allv):
        if ch2 is not None:
            ch2.abort()
        out.update(stage="init", reason=reason or "another rank failed to set up its communicators",
                   ranks_failed=[r for r, v in enumerate(allv) if not v[0]])
        link.close()
        return out
    dt_local, tokens_match, n_cmp, hop = 0.0, None, 0, {"bytes_sent": 0, "sends": 0}
    try:
        where = "warmup"
        eng2 = PipelineServingEngine(ex, ch2, n_slots=M, batch=B, max_step_tokens=B * a.prompt_len,
                                     timeout_s=a.phase2_hop_timeout, name=f"q{lane}")
        eng2.recv_into = a.phase2_recv_into == "on"
        out["data_plane"] = data_plane_name(ch2, eng2)
        out["graph_hop"] = bool(eng2.graph_hop)
        out["recv_into"] = eng2.recv_into
        reqs2 = []
        if stage == 0:
            for r in ctx["reqs1"]:
                reqs2.append(eng2.submit(Request(list(r.prompt), max_new_tokens=r.max_new_tokens, params=ctx["sp"],
                                                 stop_on_repeat=0, seed=r.seed, rid=r.rid)))
        eng2.run_rounds(2 + a.warmup)
        if eng2.failed:
            raise RuntimeError(eng2.failed)
        sync()
        agree([1])  # host barrier
        ch2.stats(reset=True)
        where = "timed"
        t1 = time.perf_counter()
        if a.phase2_inject == "run" and stage == S - 1:
            eng2.run_rounds(max(1, a.steps // 2))
            raise RuntimeError("injected failure in the middle of the timed steps (--phase2-inject run)")
        eng2.run_rounds(a.steps)
        if eng2.failed:
            raise RuntimeError(eng2.failed)
        sync()
        dt_local = time.perf_counter() - t1
        hop = ch2.stats()
        where = "drain"
        if stage == 0:
            eng2.drain()
            n_cmp = len(reqs2)
            tokens_match = all(list(r2.generated) == list(r1.generated) for r1, r2 in zip(ctx["reqs1"], reqs2))
            eng2.stop()
        else:
            eng2.serve()
        ch2.close()
    except Exception as e:  # noqa: BLE001 - a peer failure of this phase: abort, report
        ok, reason = 0.0, f"rank {rank} ({where}): {type(e).__name__}: {e}"
        if ch2 is not None:
            ch2.abort()
    try:
        rows = agree([ok, dt_local, float(hop["bytes_sent"]), float(hop["sends"]),
                      float(bool(tokens_match)) if tokens_match is not None else -1.0,
                      float(eng2.recvs_into if eng2 is not None else 0), float(eng2.recvs if eng2 is not None else 0)])
    except Exception as e:  # noqa: BLE001
        rows = [[0.0, 0.0, 0.0, 0.0, -1.0, 0.0, 0.0]]
        reason = reason or f"rank {rank}: agreement failed: {e}"
    link.close()
    if not all(r[0] for r in rows):
        out.update(stage=where if not ok else "peer", reason=reason or "another rank's second phase failed",
                   ranks_failed=[r for r, v in enumerate(rows) if not v[0]])
        return out
    dt = max(r[1] for r in rows)
    n_sess = len(ctx["reqs1"]) if stage == 0 else 0
    out.update(ok=True, value=round(a.steps * n_sess / dt, 2) if n_sess else None,
               ms_per_step=round(1000 * dt / a.steps, 3), steps=a.steps, warmup=a.warmup,
               hop_bytes_sent_per_rank=[int(r[2]) for r in rows], hop_sends_per_rank=[int(r[3]) for r in rows],
               hop_recv_into_graph_per_rank=[[int(r[5]), int(r[6])] for r in rows],
               tokens_match_headline=bool(tokens_match) if tokens_match is not None else None,
               sessions_compared=n_cmp)
    return out


if __name__ == "__main__":
    main()

"""CLI: ``python -m src.main --model M --splits S --stage K [...]`` (reference src/main.py:775-838).

* ``--stage 0``: the client ("rank0"): runs blocks [0, splits[0]) + embeddings locally,
  drives prefill and the token loop through the swarm, prints the generation and TTFT /
  decode / total time (reference run_rank0, src/main.py:62-227).
* ``--stage K >= 1``: a stage server for blocks [splits[K-1], splits[K]) (the last stage
  also applies the final norm + lm_head and samples).  Registers ``mini_petals:stage{K}``
  (TTL 45 s, heartbeat 15 s) and serves ``StageConnectionHandler.rpc_forward[_stream]``
  (reference src/main.py:230-555).
* ``--use_load_balancing``: the server instead picks ``--num_blocks`` blocks with
  ``choose_best_blocks`` (>= splits[0]), publishes ``petals:server:*`` / ``petals:module:*``
  records with its measured throughput, and every U(0, 2 x period) s re-checks
  ``should_choose_other_blocks``; on imbalance it reloads a better span (reference
  src/main.py:281-423, :558-772).  The client then routes by modules.

The reference hard-wires 4 stages (3 cut points); here the stage count follows the number
of cut points (``--splits 6`` for gpt2 = 2 stages, ``8,16,24`` = 4 stages, ...).
Same-node fast path (``--device_channel auto``, default): servers announce their machine and
device; when every hop of the client's route is on the client's machine, the client opens a
device channel through them (one ``rpc_channel_open`` handshake per hop over TCP) and the
generation runs on the continuous-batching pipeline engine with hidden states moving
GPU -> GPU over RCCL and token ids returning on the channel (``parallel/channel.py``,
``parallel/engine.py``).  Off-node routes use the TCP path below.
"""
from __future__ import annotations

import argparse
import logging
import os
import random
import signal
import sys
import threading
import time
import uuid
from typing import List, Optional

import torch

from .comm.wire import Message
from .comm.registry import DHT, get_dht_time
from .comm.rpc import RpcServer, get_loop
from .dht_utils import (DEFAULT_TTL, get_module_entries, get_remote_module_infos, get_stage_key, register_blocks_on_dht,
                        register_model_on_dht, register_server_on_dht, register_stage_on_dht)
from .llama_partition import load_stage_model, resolve_dtype
from .load_balancing import ServerState, choose_best_blocks, should_choose_other_blocks
from .models.config import resolve_model
from .models.tokenizer import load_tokenizer
from .partition import parse_splits, resolve_splits, stage_ranges  # noqa: F401 (parse_splits: API)
from .rpc_handler import StageConnectionHandler
from .rpc_transport import RpcTransport
from .runtime.executor import StageExecutor
from .throughput_measurement import FALLBACK_THROUGHPUT, get_server_throughput
from .utils import setup_logging

logger = logging.getLogger("src.main")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X-native Mini-Petals: pipeline-parallel LLM inference")
    p.add_argument("--model", required=True, help="local HF directory or preset (llama2-7b, llama3-8b, gpt2, ...)")
    p.add_argument("--splits", required=True,
                   help="comma-separated cut points, e.g. 10,20,30 (N cuts -> N+1 stages), or auto:N = the "
                        "cost-balanced cuts for N stages (partition.balanced_splits: the tail's lm_head + sampler "
                        "count against its blocks); every process must pass the same value")
    p.add_argument("--dtype", default="fp16", choices=["fp16", "bf16", "fp32"])
    p.add_argument("--max_new_tokens", type=int, default=64)
    p.add_argument("--prompt", type=str, default="Hello, how are you?")
    p.add_argument("--dht_initial_peers", type=str, default="",
                   help="comma-separated peer addresses (/ip4/H/tcp/P[/p2p/ID] or host:port)")
    p.add_argument("--public_ip", type=str, default="")
    p.add_argument("--public_dht_port", type=int, default=None)
    p.add_argument("--public_rpc_port", type=int, default=None)
    p.add_argument("--dht_port", type=int, default=8000)
    p.add_argument("--rpc_port", type=int, default=8001)
    p.add_argument("--stage", type=int, required=True)
    p.add_argument("--request_timeout", type=float, default=30.0)
    p.add_argument("--temperature", type=float, default=1.0)
    p.add_argument("--top_p", type=float, default=0.92)
    p.add_argument("--top_k", type=int, default=50)
    p.add_argument("--use_cpu_offload", action="store_true")
    p.add_argument("--keep_layers_on_gpu", type=int, default=0)
    p.add_argument("--use_load_balancing", action="store_true")
    p.add_argument("--num_blocks", type=int, default=None)
    p.add_argument("--total_blocks", type=int, default=None)
    p.add_argument("--balance_quality", type=float, default=0.75)
    p.add_argument("--mean_balance_check_period", type=float, default=120.0)
    p.add_argument("--network_bandwidth_mbps", type=float, default=None)
    # --- beyond the reference ---
    p.add_argument("--host", type=str, default="0.0.0.0", help="bind address of the registry / RPC servers")
    p.add_argument("--device", type=str, default=None, help="cuda:N / cpu (default: cuda:LOCAL_RANK if available)")
    p.add_argument("--seed", type=int, default=0, help="synthetic-weight seed (must match across stages)")
    p.add_argument("--kv_cache_gb", type=float, default=None, help="KV cache budget per stage (default: 90%% free HBM)")
    p.add_argument("--max_sessions", type=int, default=256)
    p.add_argument("--max_seq_len", type=int, default=None)
    p.add_argument("--repetition_penalty", type=float, default=None, help="sent to the last stage (server default 1.5)")
    p.add_argument("--batch_window_ms", type=float, default=0.5, help="continuous-batching collection window")
    p.add_argument("--ttl", type=float, default=DEFAULT_TTL)
    p.add_argument("--push", action="store_true",
                   help="client: server-to-server forwarding along the route (one client round trip per token)")
    p.add_argument("--alloc_timeout", type=float, default=5.0, help="server: wait this long for free KV pages")
    p.add_argument("--auto_num_blocks", action="store_true",
                   help="LB server: size the span from free HBM (upstream Petals num_blocks=None behaviour)")
    p.add_argument("--throughput_cache", type=str, default=None,
                   help="LB server: JSON cache of throughput measurements ('' disables; default: no cache)")
    p.add_argument("--log_level", type=str, default=None)
    # upstream Petals Server options (petals/server/server.py:58-86,197-228,403-414)
    p.add_argument("--block_indices", type=str, default=None,
                   help="load balancing: serve exactly blocks start:end (never rebalanced)")
    p.add_argument("--mean_block_selection_delay", type=float, default=0.0,
                   help="load balancing: sleep U(0, 2*delay) s before choosing blocks (joining servers spread out)")
    p.add_argument("--inference_max_length", type=int, default=None,
                   help="server: longest session (tokens) a client may open; alias of --max_seq_len")
    p.add_argument("--public_name", type=str, default=None, help="server: human-readable name in announcements")
    p.add_argument("--device_channel", choices=["auto", "on", "off"], default="auto",
                   help="same-node fast path: hidden states GPU->GPU over RCCL (xGMI) instead of TCP. Servers "
                        "announce it; the client uses it when every hop runs on its machine (auto) or always (on)")
    p.add_argument("--channel_data", choices=["nccl", "rccl"], default=None,
                   help="device channel data plane on GPUs: nccl (ProcessGroupNCCL send/recv, default) or rccl "
                        "(the framework's own RCCL communicators on a side stream; MPAMD_GRAPH_HOP=1 records the hop "
                        "in the decode graphs). Default: MPAMD_CHANNEL_DATA or nccl")
    p.add_argument("--throughput_batch", type=int, default=16,
                   help="LB server: concurrent one-token steps of the compute-throughput probe (tokens/s)")
    p.add_argument("--num_sessions", type=int, default=1,
                   help="client: generate this many sessions concurrently (prompt repeated, distinct seeds)")
    p.add_argument("--dump_tokens", type=str, default=None,
                   help="client: write every session's generated token ids (JSON) here (harnesses, fault tests)")
    p.add_argument("--max_replicas", type=int, default=0,
                   help="client, device channel: pipelines to open over disjoint same-node routes (0 = all found)")
    p.add_argument("--replay_cache", action="store_true",
                   help="client, device channel: stage-local recovery - every non-tail stage keeps its output "
                        "rows in HBM, so when ONE server of a pipeline dies only its spare is rebuilt (the stage "
                        "before it replays its rows; every other stage keeps its KV) instead of re-prefilling "
                        "every session on every stage.  Costs sessions x max_seq_len x hidden x 2 bytes of HBM "
                        "per stage and one row copy per step")
    return p


def pick_device(args) -> torch.device:
    if args.device:
        dev = torch.device(args.device)
    elif torch.cuda.is_available():
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    else:
        dev = torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    return dev


def _peers(s: str) -> List[str]:
    return [p.strip() for p in (s or "").split(",") if p.strip()]


def _executor_kwargs(args) -> dict:
    kw = dict(max_sessions=args.max_sessions)
    if args.kv_cache_gb is not None:
        kw["kv_cache_bytes"] = int(args.kv_cache_gb * (1 << 30))
    if args.max_seq_len is not None:
        kw["max_seq_len"] = args.max_seq_len
    if getattr(args, "inference_max_length", None) is not None:
        kw["max_seq_len"] = min(kw.get("max_seq_len", args.inference_max_length), args.inference_max_length)
    return kw


def parse_block_indices(s: Optional[str], total: int) -> Optional[List[int]]:
    """``start:end`` -> list of block ids (upstream Server ``block_indices``, server.py:221-227)."""
    if not s:
        return None
    try:
        a, b = [int(x.strip()) for x in s.split(":")]
    except ValueError:
        raise SystemExit(f"--block_indices {s!r}: expected start:end, e.g. 8:16")
    if not 0 <= a < b <= total:
        raise SystemExit(f"--block_indices {s!r} outside [0, {total}]")
    return list(range(a, b))


def _start_dht(args) -> DHT:
    host_maddrs = [f"/ip4/{args.host}/tcp/{args.dht_port}"]
    announce = None
    if args.public_ip:
        announce = [f"/ip4/{args.public_ip}/tcp/{args.public_dht_port or args.dht_port}"]
    dht = DHT(start=True, initial_peers=_peers(args.dht_initial_peers), host_maddrs=host_maddrs,
              announce_maddrs=announce)
    logger.info(f"DHT visible multiaddrs: {dht.get_visible_maddrs()}")
    return dht


# ================================================================================ client
@torch.inference_mode()
def run_rank0(args, device, cuts: List[int], on_token=None, results: Optional[list] = None):
    """``on_token(request, token)`` / ``results`` (filled with every session's tokens) are
    hooks for embedding the client (tests, fault-injection harnesses) on the device-channel path."""
    cfg = resolve_model(args.model)
    L = cfg.num_hidden_layers
    stage0_end = cuts[0]
    n_servers = len(cuts)
    dtype = resolve_dtype(args.dtype, device)
    full = load_stage_model(args.model, device, "stage0", end=stage0_end, dtype=dtype, seed=args.seed,
                            **_executor_kwargs(args))
    w = full.weights
    ex = StageExecutor(cfg, w, device, dtype=dtype, **full.executor_kwargs)
    tok = load_tokenizer(args.model, cfg)
    total_blocks = args.total_blocks or L
    tx = RpcTransport(device, 0, _peers(args.dht_initial_peers), args.dht_port, args.rpc_port,
                      timeout=args.request_timeout, temperature=args.temperature, top_p=args.top_p,
                      top_k=args.top_k, stage_keys=[get_stage_key(i) for i in range(1, n_servers + 1)],
                      routing="module" if args.use_load_balancing else "stage", model_name=args.model,
                      total_blocks=total_blocks, start_block=stage0_end, repetition_penalty=args.repetition_penalty,
                      push=args.push)
    ids = tok(args.prompt, return_tensors="pt").input_ids.reshape(-1)
    Lp = int(ids.numel())
    sid = str(uuid.uuid4())
    max_length = Lp + args.max_new_tokens
    if args.device_channel != "off":
        route = tx._get_route(sid)
        if args.device_channel == "on" or tx.device_channel_possible(route, device):
            return _run_rank0_channel(args, device, ex, tok, tx, route, ids, on_token=on_token, results=results)
        logger.info("device channel not possible (a hop is on another machine or did not announce one): TCP path")
    if int(args.num_sessions) > 1:
        return _run_rank0_tcp_sessions(args, device, ex, tok, tx, ids)
    t0 = time.perf_counter()
    hidden = ex.forward([(sid, Lp)], ids.to(device), reset=[True], max_length=max_length)
    tx.send_prefill(Lp, hidden, session_id=sid, max_length=max_length)
    next_id = tx.recv_token()
    generated = [next_id]
    ttft = time.perf_counter() - t0
    logger.info(f"Prefill completed in {ttft:.3f}s; first token {next_id}")
    eos = getattr(tok, "eos_token_id", None)
    cur_len = Lp + 1
    repeat, last = 0, None
    t1 = time.perf_counter()
    for _ in range(args.max_new_tokens - 1):
        if eos is not None and next_id == eos:
            logger.info("EOS token generated, stopping generation")
            break
        hidden = ex.forward([(sid, 1)], torch.tensor([next_id], device=device), starts=[cur_len - 1])
        tx.send_decode_step(cur_len, hidden, session_id=sid, max_length=max_length, generated_tokens=generated)
        next_id = tx.recv_token()
        if eos is not None and next_id == eos:
            logger.info("EOS token generated, stopping generation")
            break
        if next_id == last:
            repeat += 1
            if repeat >= 5:
                logger.warning(f"Consecutive repetition detected (token {next_id}), stopping generation")
                break
        else:
            repeat, last = 0, next_id
        generated.append(next_id)
        cur_len += 1
    t2 = time.perf_counter()
    text = tok.decode(generated, skip_special_tokens=True)
    print(f"\n{'=' * 80}\nPROMPT: {args.prompt}\nGENERATED: {text}\n{'=' * 80}\n", flush=True)
    n_dec = max(len(generated) - 1, 0)
    logger.info(f"Decode completed in {t2 - t1:.3f}s ({n_dec / max(t2 - t1, 1e-9):.2f} tokens/s)")
    logger.info(f"Total time: {t2 - t0:.3f}s")
    logger.info(f"TTFT (Time to First Token): {ttft:.3f}s")
    if tx.decode_stage_history:
        keys = [k for k, _ in tx.decode_stage_history[-1]]
        for i, k in enumerate(keys):
            vals = [h[i][1] for h in tx.decode_stage_history if len(h) > i]
            logger.info(f"hop {k}: mean {1000 * sum(vals) / len(vals):.2f} ms over {len(vals)} steps")
    tx.close_session(sid)
    tx.shutdown()
    return generated


def _run_rank0_tcp_sessions(args, device, ex, tok, tx, ids):
    """``--num_sessions N`` over the TCP RPC path: N sessions of the same prompt advance in
    lockstep; stage 0 runs all of them as one ragged step and every hop receives the N
    per-session requests concurrently (``RpcTransport.send_steps``), so each server batches
    them inside its window.  Each session keeps its own route, history and recovery."""
    n = int(args.num_sessions)
    Lp = int(ids.numel())
    max_length = Lp + args.max_new_tokens
    sids = [str(uuid.uuid4()) for _ in range(n)]
    eos = getattr(tok, "eos_token_id", None)
    t0 = time.perf_counter()
    hidden = ex.forward([(s, Lp) for s in sids], ids.repeat(n).to(device), reset=[True] * n,
                        max_length=max_length)
    rows = hidden.reshape(n, Lp, -1)
    nxt = tx.send_steps([(s, rows[i], Lp, Lp, max_length, None) for i, s in enumerate(sids)])
    ttft = time.perf_counter() - t0
    gen = {s: [t] for s, t in zip(sids, nxt)}
    live = [s for s, t in zip(sids, nxt) if t != eos]
    t1 = time.perf_counter()
    n_dec = 0
    for _ in range(args.max_new_tokens - 1):
        if not live:
            break
        toks = torch.tensor([gen[s][-1] for s in live], device=device)
        hidden = ex.forward([(s, 1) for s in live], toks)
        out = tx.send_steps([(s, hidden[i:i + 1], 1, Lp + len(gen[s]), max_length, gen[s])
                             for i, s in enumerate(live)])
        n_dec += len(live)
        for s, t in zip(live, out):
            gen[s].append(t)
        live = [s for s, t in zip(live, out) if t != eos]
    t2 = time.perf_counter()
    text = tok.decode(gen[sids[0]], skip_special_tokens=True)
    print(f"\n{'=' * 80}\nPROMPT: {args.prompt}\nGENERATED: {text}\n{'=' * 80}\n", flush=True)
    logger.info(f"TCP path: {len(tx.stage_keys) + 1} stages, {n} concurrent session(s)")
    logger.info(f"Decode completed in {t2 - t1:.3f}s ({n_dec / max(t2 - t1, 1e-9):.2f} tokens/s over {n} session(s))")
    logger.info(f"Total time: {t2 - t0:.3f}s ({(n_dec + n) / max(t2 - t0, 1e-9):.2f} tokens/s end to end)")
    logger.info(f"TTFT (Time to First Token): {ttft:.3f}s")
    if tx.decode_stage_history:
        keys = [k for k, _ in tx.decode_stage_history[-1]]
        for i, k in enumerate(keys):
            vals = [h[i][1] for h in tx.decode_stage_history if len(h) > i]
            logger.info(f"hop {k}: mean {1000 * sum(vals) / len(vals):.2f} ms over {len(vals)} session-steps")
    for s in sids:
        tx.close_session(s)
    tx.shutdown()
    return gen[sids[0]]


def _run_rank0_channel(args, device, ex, tok, tx, route, ids, on_token=None, results=None):
    """Same-node fast path of run_rank0: this process heads a device channel
    (parallel/channel.py) through the servers of every complete same-node route - one
    pipeline replica per disjoint route - and generation runs on the continuous-batching
    engine (parallel/engine.py) under the replica front end (parallel/router.py): sessions
    are placed by throughput (measured tokens/s of each replica, EMA) and, when a pipeline
    loses a stage, its dead servers are found over TCP (``rpc_echo``), a replacement route
    is opened if the registry has one, and the unfinished sessions are re-prefilled
    (prompt + generated tokens) on the surviving / rebuilt replicas - the fast-path form of
    the reference client's exclude / rediscover / replay failover (src/rpc_transport.py:
    587-712).  The TCP RPC only does discovery, liveness probes and the channel handshake."""
    from .parallel.engine import PipelineServingEngine, Request, request_seed
    from .parallel.router import ReplicaFrontend
    from .runtime.sampler import SamplingParams

    n = max(1, int(args.num_sessions))
    same_node = args.device_channel == "auto"
    max_rep = int(getattr(args, "max_replicas", 0) or 0) or None
    routes = tx.channel_routes(device, max_routes=max_rep, same_node=same_node) or [route]
    S = len(routes[0]) + 1
    M = max(1, min(S + 1, n))
    B = (n + M - 1) // M  # every replica can hold ALL sessions: a lone survivor takes them over
    timeout = max(30.0, args.request_timeout * 2)
    rep_routes = {}
    counter = [0]

    replay = bool(getattr(args, "replay_cache", False))

    def open_replica(rt, old=None):
        k = counter[0]
        counter[0] += 1
        ch = tx.open_device_channel(rt, device, n_slots=M, batch=B, timeout=timeout, timing=True,
                                    data_backend=getattr(args, "channel_data", None), replay_cache=replay,
                                    resume_prefix=old.ch.prefix if old is not None else None)
        eng = PipelineServingEngine(ex, ch, n_slots=M, batch=B, name=f"client-r{k}", timeout_s=timeout,
                                    replay_cache=replay,
                                    resume={"prefix": old.name, "cache": old.replay} if old is not None else None)
        eng.freeze_heap = True  # the client is a driver process: one heap freeze per process
        eng.timing = True
        ch.timing = True
        thr = min((float(h.info.get("throughput") or 0.0) for h in rt), default=0.0)
        return eng, thr

    engines, thrs = {}, []
    for r, rt in enumerate(routes):
        engines[r], t = open_replica(rt)
        rep_routes[r] = rt
        thrs.append(t)
    known = all(t > 0 for t in thrs)

    def recover(r):
        """Replica r lost a stage: probe its servers, exclude the dead ones, open a replacement
        route over servers no live replica uses (wait for one only if nothing else is left)."""
        dead = [h for h in rep_routes[r] if not tx.hop_alive(h)]
        for h in dead:
            tx.failed_peers.setdefault(h.key, set()).add(h.peer_id)
        logger.warning(f"replica {r} failed; dead servers: {[h.peer_id[:8] for h in dead] or 'none answered dead'}")
        old = engines.get(r)
        if old is not None and old.ch is not None:
            old.ch.close()
        live = [k for k in fe.alive_locals() if k != r]
        busy = set().union(*[{h.peer_id for h in rep_routes[k]} for k in live]) if live else set()
        if replay and len(dead) == 1 and old is not None and old.failed_sessions:
            # stage-local recovery: swap only the dead hop; the survivors adopt their sessions and
            # the stage before the spare replays its cached rows into it
            k = rep_routes[r].index(dead[0])
            hop = tx.replacement_hop(dead[0], device, exclude=busy | {h.peer_id for h in rep_routes[r]},
                                     same_node=same_node, wait_s=0.0 if live else max(10.0, args.request_timeout))
            if hop is not None:
                rt = rep_routes[r][:k] + [hop] + rep_routes[r][k + 1:]
                try:
                    eng, thr = open_replica(rt, old=old)
                except (ConnectionError, OSError, RuntimeError) as e:
                    logger.warning(f"stage-local rebuild through {hop.peer_id[:8]} failed ({e}); full rebuild")
                else:
                    eng.resume_target = k + 1
                    eng.resume_from = old
                    r2 = fe.router.n
                    rep_routes[r2] = rt
                    engines[r2] = eng
                    logger.info(f"rebuilt a pipeline over {[h.peer_id[:8] for h in rt]} (stage {k + 1} replaced, "
                                f"the other stages keep their KV)")
                    return eng, thr if thr > 0 else (max(fe.router.throughput) if fe.router.throughput else 1.0)
        new = tx.channel_routes(device, max_routes=1, exclude=busy, same_node=same_node,
                                wait_s=0.0 if live else max(10.0, args.request_timeout))
        if not new:
            return None
        eng, thr = open_replica(new[0])
        r2 = fe.router.n  # the index add_replica will hand out
        rep_routes[r2] = new[0]
        engines[r2] = eng
        logger.info(f"rebuilt a pipeline over {[h.peer_id[:8] for h in new[0]]}")
        return eng, thr if thr > 0 else (max(fe.router.throughput) if fe.router.throughput else 1.0)

    fe = ReplicaFrontend(len(engines), locals=engines, throughputs=thrs if known else None, timeout_s=timeout,
                         recover=recover)
    engines[0]._settle_heap()  # the one-time heap freeze before t0, not inside the first round (TTFT)
    progress = {"n": 0, "t": time.perf_counter()}

    def _on_token(req, tok_id):
        progress["n"] += 1
        now = time.perf_counter()
        if now - progress["t"] >= 1.0:
            progress["t"] = now
            logger.info(f"progress: {progress['n']} tokens generated")
        if on_token is not None:
            on_token(req, tok_id)

    fe.on_token = _on_token
    eos = getattr(tok, "eos_token_id", None)
    rp = args.repetition_penalty if args.repetition_penalty is not None else 1.5
    sp = SamplingParams(args.temperature, args.top_p, args.top_k, rp)
    t0 = time.perf_counter()
    reqs = [fe.submit(Request(ids.tolist(), max_new_tokens=args.max_new_tokens, params=sp, eos_token_id=eos,
                              seed=request_seed(args.seed, f"s{i}"), rid=f"s{i}")) for i in range(n)]
    try:
        with torch.inference_mode():
            fe.run(stop=False)
        t2 = time.perf_counter()
        for r, eng in fe.alive_locals().items():
            try:
                _log_stage_stats(r, eng.gather_stage_stats(), rep_routes.get(r, []))
            except Exception as e:  # noqa: BLE001 - stats are diagnostics
                logger.warning(f"replica {r}: stage stats unavailable ({e})")
    finally:
        for r, eng in fe.alive_locals().items():
            eng.stop()
        for eng in engines.values():
            if eng.ch is not None:
                eng.ch.close()
    gen = reqs[0].generated
    if results is not None:
        results.extend(r.generated for r in reqs)
    if getattr(args, "dump_tokens", None):
        import json

        with open(args.dump_tokens, "w") as f:
            json.dump({r.rid: {"tokens": r.generated, "finish": r.finish_reason} for r in reqs}, f)
    text = tok.decode(gen, skip_special_tokens=True)
    print(f"\n{'=' * 80}\nPROMPT: {args.prompt}\nGENERATED: {text}\n{'=' * 80}\n", flush=True)
    ttft = (reqs[0].t_first or t2) - t0
    total = sum(len(r.generated) for r in reqs)
    logger.info(f"device channel: {S} stages x {len(routes)} replica(s), {n} session(s), {M} slot(s) x {B}; "
                f"tokens per replica {fe.replica_tokens}")
    if fe.failures:
        logger.info(f"failover: {len(fe.failures)} replica failure(s) recovered "
                    f"({'; '.join(f'replica {r}: {w[:80]}' for r, w in fe.failures)}); "
                    f"{len(fe.resumed)} session(s) resumed in place, {len(fe.replaced)} re-prefilled")
    # decode rate counts tokens after each session's first one over the time after the first
    # session's first token (as the TCP path does); end-to-end counts everything from t0
    logger.info(f"Decode completed in {t2 - t0 - ttft:.3f}s ({(total - n) / max(t2 - t0 - ttft, 1e-9):.2f} tokens/s "
                f"over {n} session(s))")
    logger.info(f"Total time: {t2 - t0:.3f}s ({total / max(t2 - t0, 1e-9):.2f} tokens/s end to end)")
    logger.info(f"TTFT (Time to First Token): {ttft:.3f}s")
    tx.shutdown()
    return gen


def _log_stage_stats(replica: int, rows, route) -> None:
    """Per-stage ms of a device-channel pipeline (the reference client's per-hop times,
    src/rpc_transport.py:98-103, 824-839): compute per micro-batch step, how long the stage
    waited for its input, bytes it sent downstream."""
    names = ["stage0 (client)"] + [f"{h.key} {h.peer_id[:8]}" for h in route]
    for row in rows:
        k = int(row["stage"])
        name = names[k] if k < len(names) else f"stage{k}"
        logger.info(f"replica {replica} {name}: blocks {int(row['blocks'])}, compute {row['compute_ms']:.3f} ms/step "
                    f"over {int(row['steps'])} steps, input wait {row['recv_wait_ms']:.3f} ms/step, "
                    f"sent {row['bytes_sent'] / 2**20:.1f} MiB")


# ================================================================================ servers
class _Server:
    """RPC server + handler + heartbeat for one loaded span."""

    def __init__(self, args, dht: DHT, executor: StageExecutor, final: bool, stage_idx: int,
                 throughput: Optional[float] = None, lb: bool = False, announce: bool = True):
        self.args, self.dht, self.ex, self.final, self.stage_idx = args, dht, executor, final, stage_idx
        self.throughput, self.lb = throughput, lb
        self.link_mbps: Optional[float] = getattr(args, "network_bandwidth_mbps", None)
        self.loop = get_loop()
        self.server = RpcServer(args.host, args.rpc_port, announce_host=args.public_ip or None,
                                announce_port=args.public_rpc_port)
        self.handler = StageConnectionHandler(dht, executor, executor.device, args.request_timeout, final,
                                              batch_window_ms=args.batch_window_ms, seed=args.seed,
                                              alloc_timeout=getattr(args, "alloc_timeout", 5.0))
        self.loop.run(self.server.start())
        self.handler.add_p2p_handlers(self.server)
        self.maddrs = self.server.maddrs
        if args.host in ("0.0.0.0", "") and not args.public_ip:
            self.maddrs = [m.replace("/ip4/0.0.0.0/", "/ip4/127.0.0.1/") for m in self.maddrs]
        self.peer_id = self.server.peer_id
        self.next_pings: dict = {}
        self._stop = threading.Event()
        if announce:
            self.store_once()
        logger.info(f"StageConnectionHandler handlers registered (stage {stage_idx}, blocks "
                    f"[{executor.start},{executor.end}), final={final}, peer {self.peer_id}, maddrs {self.maddrs})")
        self._hb = threading.Thread(target=self._heartbeat, daemon=True)
        self._hb.start()

    def store_once(self, state: ServerState = ServerState.ONLINE):
        a, ex = self.args, self.ex
        exp = get_dht_time() + a.ttl
        extra = dict(start_block=ex.start, end_block=ex.end, final_stage=self.final,
                     cache_tokens_left=int(ex.sessions.cache_tokens_left()))
        if self.next_pings:
            extra["next_pings"] = dict(self.next_pings)
        if self.lb:
            extra.update(blocks=[ex.start, ex.end], throughput=self.throughput)
        if getattr(a, "public_name", None):
            extra["public_name"] = a.public_name
        chan = {}
        if getattr(a, "device_channel", "auto") != "off":
            from .parallel.channel import host_id

            chan = dict(channel_host=host_id(), device=str(ex.device))
            extra.update(chan)
        if state == ServerState.ONLINE:
            register_stage_on_dht(self.dht, self.stage_idx, self.peer_id, self.maddrs, ttl=a.ttl, **extra)
        register_model_on_dht(self.dht, a.model, getattr(a, "total_blocks", None) or ex.cfg.num_hidden_layers,
                              public_name=getattr(a, "public_name", None), ttl=a.ttl)
        if self.lb:
            register_server_on_dht(self.dht, self.peer_id, ex.start, ex.end, self.throughput or FALLBACK_THROUGHPUT,
                                   a.model, p2p_maddrs=self.maddrs, final_stage=self.final, state=state,
                                   expiration_time=exp)
            register_blocks_on_dht(self.dht, self.peer_id, list(range(ex.start, ex.end)), a.model, self.maddrs,
                                   ex.start, ex.end, self.throughput, self.final, state, exp, extra=chan)

    def measure_next_pings(self, max_peers: int = 5, timeout: float = 2.0) -> dict:
        """RTT (s) to servers hosting the block right after this span (upstream Petals
        ModuleAnnouncerThread ``next_pings``, petals/server/server.py:674-767): routing hints."""
        if self.final:
            return {}
        from .comm.rpc import RpcClient

        ents = get_module_entries(self.dht, self.ex.end, self.args.model)
        if not ents:  # fixed-split swarm: the next stage's records
            res = self.dht.get(get_stage_key(self.stage_idx + 1), latest=True)
            if res is not None and isinstance(res.value, dict):
                ents = {str(k): (v.value if hasattr(v, "value") else v) for k, v in res.value.items()}
        pings = {}

        async def probe(client, addr):
            t0 = time.perf_counter()
            await client.call(addr, "StageConnectionHandler.rpc_echo", Message({"ping": True}), timeout=timeout)
            return time.perf_counter() - t0

        client = RpcClient()
        try:
            for pid, e in list(ents.items())[:max_peers]:
                addrs = (e or {}).get("p2p_maddrs") or []
                if pid == self.peer_id or not addrs:
                    continue
                try:
                    pings[pid] = round(self.loop.run(probe(client, addrs[0]), timeout=timeout + 1), 6)
                except Exception:  # unreachable peers are simply absent
                    pass
        finally:
            try:
                self.loop.run(client.close(), timeout=2)
            except Exception:
                pass
        self.next_pings = pings
        return pings

    def _heartbeat(self):
        period = self.args.ttl / 3
        while not self._stop.wait(period):
            try:
                self.measure_next_pings()
                self.store_once()
                self.ex.sessions.evict_expired()
            except Exception as e:  # pragma: no cover
                logger.warning(f"heartbeat failed: {e}")

    def stop(self, announce_offline: bool = True):
        self._stop.set()
        if announce_offline and self.lb:
            try:
                self.store_once(ServerState.OFFLINE)
            except Exception:
                pass
        try:
            self.loop.run(self.server.shutdown(), timeout=5)
        except Exception:
            pass
        self.handler.shutdown()


def _install_signal_handlers(stop: threading.Event):
    def _h(signum, frame):
        logger.info(f"signal {signum}: shutting down")
        stop.set()

    for s in (signal.SIGTERM, signal.SIGINT):
        try:
            signal.signal(s, _h)
        except ValueError:
            pass


def run_stage_server_fixed(args, device, cuts: List[int], stop: Optional[threading.Event] = None, on_ready=None):
    cfg = resolve_model(args.model)
    ranges = stage_ranges(cuts, cfg.num_hidden_layers)
    k = args.stage
    if not 1 <= k < len(ranges):
        raise SystemExit(f"--stage {k} out of range: splits {cuts} define stages 0..{len(ranges) - 1}")
    s, e = ranges[k]
    final = k == len(ranges) - 1
    role = "last" if final else "segment"
    dtype = resolve_dtype(args.dtype, device)
    full = load_stage_model(args.model, device, role, start=s, end=e, dtype=dtype, seed=args.seed,
                            use_cpu_offload=args.use_cpu_offload, **_executor_kwargs(args))
    off = bool(args.use_cpu_offload) and device.type == "cuda"
    ex = StageExecutor(cfg, full.weights if off or not args.use_cpu_offload else _onto(full, device), device,
                       dtype=dtype, offload=off, keep_layers_on_gpu=args.keep_layers_on_gpu, **full.executor_kwargs)
    dht = _start_dht(args)
    srv = _Server(args, dht, ex, final, k)
    stop = stop or threading.Event()
    _install_signal_handlers(stop)
    if on_ready is not None:
        on_ready(dht, srv)
    stop.wait()
    srv.stop()
    dht.shutdown()


def _onto(full, device):
    from .llama_partition import _to_device

    return _to_device(full.weights, device)


def run_stage_server_with_load_balancing(args, device, cuts: List[int], stop: Optional[threading.Event] = None,
                                         on_ready=None):
    cfg = resolve_model(args.model)
    total = args.total_blocks or cfg.num_hidden_layers
    min_block = cuts[0] if cuts else 0
    dtype = resolve_dtype(args.dtype, device)
    if args.num_blocks is None and getattr(args, "auto_num_blocks", False) and device.type == "cuda":
        from .block_utils import auto_num_blocks

        num_blocks = auto_num_blocks(cfg, dtype=dtype, device=device, total_blocks=total - min_block)
        logger.info(f"auto num_blocks = {num_blocks}")
    else:
        num_blocks = args.num_blocks or 4
    tcache = None
    if getattr(args, "throughput_cache", None):
        from .throughput_measurement import ThroughputCache

        tcache = ThroughputCache(args.throughput_cache)
    dht = _start_dht(args)
    stop = stop or threading.Event()
    _install_signal_handlers(stop)
    strict = parse_block_indices(getattr(args, "block_indices", None), total)
    while not stop.is_set():
        sel_delay = getattr(args, "mean_block_selection_delay", 0.0)
        if strict is None and sel_delay > 0 and stop.wait(random.uniform(0, 2 * sel_delay)):
            break
        infos = []
        delay = 2.0
        for attempt in range(3):
            try:
                infos = get_remote_module_infos(dht, args.model, total)
                break
            except Exception as e:  # pragma: no cover
                logger.warning(f"module info query failed ({e}); retry in {delay:.1f}s")
                time.sleep(delay)
                delay *= 1.5
        if strict is not None:
            blocks = strict
        elif infos:
            blocks = choose_best_blocks(num_blocks, infos, total, min_block=min_block)
        else:
            blocks = list(range(min_block, min(min_block + num_blocks, total)))
        s, e = blocks[0], min(blocks[-1] + 1, total)
        final = e >= total
        logger.info(f"Selected blocks [{s}, {e}) (final={final})")
        full = load_stage_model(args.model, device, "last" if final else "segment", start=s, end=e, dtype=dtype,
                                seed=args.seed, **_executor_kwargs(args))
        ex = StageExecutor(cfg, full.weights, device, dtype=dtype, **full.executor_kwargs)
        tb = max(1, int(getattr(args, "throughput_batch", 16)))
        srv = _Server(args, dht, ex, final, args.stage, throughput=FALLBACK_THROUGHPUT, lb=True, announce=False)
        mbps = args.network_bandwidth_mbps
        if mbps is None:  # measure the link instead of assuming 100 Mbit/s
            mbps = _measure_network(args, dht, srv, ex, total)
        thr = get_server_throughput(ex, mbps, cache=tcache, batch=tb)
        srv.throughput = thr
        srv.link_mbps = mbps
        srv.store_once()
        logger.info(f"Announced blocks [{s}, {e}) throughput={thr:.1f} rps link={mbps} Mbit/s")
        if on_ready is not None:
            on_ready(dht, srv)
        rebalance = False
        if strict is not None:  # pinned span: heartbeat only, never rebalanced (upstream server.py:414)
            stop.wait()
        while strict is None and not stop.is_set():
            if stop.wait(random.uniform(0, 2 * args.mean_balance_check_period)):
                break
            try:
                srv.throughput = get_server_throughput(ex, srv.link_mbps, n_steps=3, batch=tb)
                infos = get_remote_module_infos(dht, args.model, total)
                if should_choose_other_blocks(srv.peer_id, infos, args.balance_quality, total, min_block):
                    logger.info("Rebalancing: choosing other blocks")
                    rebalance = True
                    break
            except Exception as e:  # pragma: no cover
                logger.warning(f"rebalance check failed: {e}")
        srv.stop()
        del ex, full
        if device.type == "cuda":
            torch.cuda.empty_cache()
        if not rebalance:
            break
    dht.shutdown()


def _measure_network(args, dht, srv, ex, total) -> Optional[float]:
    """Measured Mbit/s for the network term: echo round trips to another server of the swarm
    (the span after ours first, else any), or to our own RPC endpoint when we are alone (the
    local stack's ceiling).  None (-> the reference's 100 Mbit/s) if nothing answers."""
    from .throughput_measurement import measure_peer_bandwidth

    addrs = []
    try:
        for e in get_module_entries(dht, min(ex.end, total - 1), args.model).values():
            if str(e.get("peer_id")) != srv.peer_id:
                addrs.extend(e.get("p2p_maddrs") or [])
        if not addrs:
            for b in range(total):
                for e in get_module_entries(dht, b, args.model).values():
                    if str(e.get("peer_id")) != srv.peer_id:
                        addrs.extend(e.get("p2p_maddrs") or [])
                if addrs:
                    break
    except Exception as e:  # pragma: no cover
        logger.warning(f"peer lookup for the bandwidth probe failed: {e}")
    mbps = measure_peer_bandwidth((addrs or list(srv.maddrs))[:3], ex.cfg.hidden_size, ex.dtype)
    logger.info(f"measured link bandwidth: {mbps if mbps is None else round(mbps, 1)} Mbit/s "
                f"({'peer' if addrs else 'loopback'})")
    return mbps


def run_stage_server(args, device, cuts, stop=None, on_ready=None):
    if args.use_load_balancing:
        return run_stage_server_with_load_balancing(args, device, cuts, stop, on_ready)
    return run_stage_server_fixed(args, device, cuts, stop, on_ready)


def main(argv=None):
    args = build_parser().parse_args(argv)
    setup_logging(args.log_level)
    device = pick_device(args)
    cfg = resolve_model(args.model)
    try:
        cuts = resolve_splits(args.splits, cfg)  # model defaults only: every process derives the same cuts
    except ValueError as e:
        raise SystemExit(f"--splits {args.splits}: {e}")
    if not cuts:
        raise SystemExit("--splits must contain at least one cut point")
    if str(args.splits).startswith("auto"):
        logger.info(f"--splits {args.splits} -> {','.join(map(str, cuts))}")
    if args.stage == 0:
        run_rank0(args, device, cuts)
    else:
        run_stage_server(args, device, cuts)


if __name__ == "__main__":
    main()

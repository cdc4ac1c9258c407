"""Replica router and failover for single-node pipelines (BASELINE configs "4 stages x 2
replicas, load_balancing.py routing over RCCL subgroups" and "... + fault-tolerance replica
failover").

Reference: servers hosting the same blocks register under the same keys; the client routes
each session greedily over the live spans (src/rpc_transport.py:393-501), and when a hop
fails it excludes the peer, re-discovers a replacement and replays the session's cached
inputs to rebuild its KV (src/rpc_transport.py:587-712).

On one node a replica is a whole pipeline (its own device channel), so routing and
recovery work one level up, in a front end on global rank 0 (which is also replica 0's
head):

* **Throughput registry.** Every rank measures its stage's decode rate and the node
  all-gathers them on a host control group (``gather_replica_throughput``); a replica's
  rate is its slowest stage's.  Running replica heads keep reporting their measured
  tokens/s, and the router's placement weights follow (EMA).
* **Placement.** New sessions go to live replicas in proportion to throughput
  (``ReplicaRouter`` / ``assign_sessions``); a per-replica host link (gloo) carries
  admissions (prompt, generated-so-far, sampling parameters, seed) to remote heads and
  token / finish reports back, one exchange per head round, each on its own router thread
  so replicas never wait on each other.
* **Failure detection.** A head whose pipeline loses a stage reports it (its channel
  aborted, see ``engine.PipelineFailure``); a head that dies shows up as a link error or
  timeout.  Either way the replica is marked dead and its unfinished sessions are
  re-placed on the survivors by **re-prefilling prompt + generated tokens** (token history
  is all a pipeline needs to rebuild KV).  Sampling is seeded by (session seed, position),
  so the survivors produce exactly the tokens the failed replica would have.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..runtime.sampler import SamplingParams
from .channel import ChannelError, HostLink
from .engine import PipelineFailure, PipelineServingEngine, Request, _f2i, _i2f
from .failover import ReplicaRouter

logger = logging.getLogger(__name__)

REPORT, CMD = 1, 2
REASONS = {"eos": 1, "length": 2, "repeat": 3, "max_length": 4, "done": 5}
REASON_OF = {v: k for k, v in REASONS.items()}


def gather_replica_throughput(link: HostLink, executor, replica: int, stage: int, n_replicas: int,
                              batch: int = 16) -> List[float]:
    """All-gather every rank's measured decode rate; replica tokens/s = batch x its slowest
    stage's steps/s (the C3 "throughput registry over an all-gather")."""
    from ..throughput_measurement import measure_compute_throughput

    sps = measure_compute_throughput(executor, n_warmup=1, n_steps=3, batch=batch)
    rows = link.all_gather_floats([float(replica), float(stage), float(sps)])
    per = [float("inf")] * n_replicas
    for r, _, v in rows:
        per[int(r)] = min(per[int(r)], v)
    return [batch * v for v in per]


# ------------------------------------------------------------------ wire format (int64)
def encode_cmd(reqs: Sequence[Tuple[int, Request]], stop: bool) -> np.ndarray:
    out = [CMD, int(stop), len(reqs)]
    for rid, r in reqs:
        p = r.params
        out += [rid, r.max_new_tokens, r.seed, -1 if r.eos_token_id is None else int(r.eos_token_id),
                r.stop_on_repeat, _f2i(p.temperature), _f2i(p.top_p), int(p.top_k), _f2i(p.repetition_penalty),
                len(r.prompt), len(r.generated)]
        out += list(r.prompt) + list(r.generated)
    return np.asarray(out, dtype=np.int64)


def decode_cmd(a: np.ndarray) -> Tuple[bool, List[Request]]:
    assert int(a[0]) == CMD
    stop, n = bool(a[1]), int(a[2])
    off, reqs = 3, []
    for _ in range(n):
        rid, mx, seed, eos, rep, t, tp, tk, rp, lp, lg = (int(v) for v in a[off:off + 11])
        off += 11
        prompt = a[off:off + lp].tolist()
        gen = a[off + lp:off + lp + lg].tolist()
        off += lp + lg
        reqs.append(Request(prompt, max_new_tokens=mx, params=SamplingParams(_i2f(t), _i2f(tp), tk, _i2f(rp)),
                            eos_token_id=None if eos < 0 else eos, stop_on_repeat=rep, seed=seed, rid=str(rid),
                            generated=gen))
    return stop, reqs


def encode_report(tokens: Sequence[Tuple[int, int]], finished: Sequence[Tuple[int, int]], failed: bool,
                  tok_per_s: float) -> np.ndarray:
    out = [REPORT, int(failed), len(tokens), len(finished), int(tok_per_s * 1000)]
    for a, b in tokens:
        out += [a, b]
    for a, b in finished:
        out += [a, b]
    return np.asarray(out, dtype=np.int64)


def decode_report(a: np.ndarray):
    assert int(a[0]) == REPORT
    failed, nt, nf, thr = bool(a[1]), int(a[2]), int(a[3]), int(a[4]) / 1000.0
    toks = a[5:5 + 2 * nt].reshape(nt, 2).tolist()
    fin = a[5 + 2 * nt:5 + 2 * nt + 2 * nf].reshape(nf, 2).tolist()
    return failed, toks, fin, thr


# ------------------------------------------------------------------ remote replica head
def serve_replica_head(engine: PipelineServingEngine, link: HostLink, timeout_s: float = 120.0) -> str:
    """Loop of a replica head (global rank r*S, r >= 1): report tokens, take admissions,
    run one round.  Returns "stopped" or "failed"."""
    toks: List[Tuple[int, int]] = []
    fin: List[Tuple[int, int]] = []
    engine.on_token = lambda req, t: toks.append((int(req.rid), int(t)))
    engine.on_finish = lambda req: fin.append((int(req.rid), REASONS.get(req.finish_reason, 5)))
    failed = False
    t_last, n_last = time.perf_counter(), 0
    while True:
        now = time.perf_counter()
        rate = (engine.tokens_generated - n_last) / max(now - t_last, 1e-6) if engine.is_head else 0.0
        t_last, n_last = now, engine.tokens_generated
        link.send_msg(0, encode_report(toks, fin, failed, rate))
        toks.clear()
        fin.clear()
        if failed:
            link.close()
            return "failed"
        stop, adm = decode_cmd(link.recv_msg(0, timeout_s))
        for r in adm:
            try:
                engine.submit(r)
            except ValueError as e:  # cannot fit this pipeline: report it finished, keep serving
                logger.error(f"replica head: session {r.rid} rejected: {e}")
                fin.append((int(r.rid), REASONS["max_length"]))
        if stop:
            engine.drain()
            engine.stop()
            link.close()
            return "stopped"
        try:
            if engine.idle:
                time.sleep(0.002)
            else:
                engine.run_rounds(1)
        except PipelineFailure as e:
            logger.error(f"replica head: pipeline failed ({e}); reporting to the router")
            failed = True


# ------------------------------------------------------------------ front end (global rank 0)
class ReplicaFrontend:
    """Routes sessions over replica pipelines and fails them over.

    ``locals``: replica index -> a pipeline head engine driven by THIS thread (the CLI client
    heads every same-node replica itself; bench / multi-process runs head replica 0 here);
    ``links``: replica index -> host link to a remote replica head (``serve_replica_head``).
    ``recover(r)`` (optional) is called when replica ``r`` fails, before its sessions are
    re-placed: it may rebuild a pipeline (new route, excluding dead servers) and return
    ``(engine, throughput)``, which joins as a new replica."""

    def __init__(self, n_replicas: int, local: Optional[PipelineServingEngine] = None,
                 links: Optional[Dict[int, HostLink]] = None, throughputs: Optional[Sequence[float]] = None,
                 timeout_s: float = 120.0, *, locals: Optional[Dict[int, PipelineServingEngine]] = None,
                 recover: Optional[Callable[[int], Optional[Tuple[PipelineServingEngine, float]]]] = None):
        self.n = int(n_replicas)
        self.router = ReplicaRouter(self.n, throughputs, timeout_s)
        self.locals: Dict[int, PipelineServingEngine] = dict(locals or {})
        if local is not None:
            self.locals[0] = local
        self.links = dict(links or {})
        self.recover = recover
        self.timeout_s = timeout_s
        self.lock = threading.RLock()
        self.requests: Dict[int, Request] = {}
        self.pending: Dict[int, List[int]] = {r: [] for r in range(self.n)}
        self.failures: List[Tuple[int, str]] = []
        self.failure_times: List[float] = []  # perf_counter() of each failure (drill reporting)
        self.replaced: Dict[int, int] = {}    # re-placed session -> tokens it had at its failure
        self.at_failure: Dict[int, int] = {}  # every session -> tokens it had at the first failure
        self.resumed: Dict[int, int] = {}     # session resumed in place (stage-local) -> tokens at failure
        self._next = 0
        self._threads: List[threading.Thread] = []
        self.replica_tokens = [0] * self.n
        self._rate_mark: Dict[int, Tuple[float, int]] = {}
        self._measured = [throughputs is not None] * self.n
        self.on_token: Optional[Callable[[Request, int], None]] = None
        for r, eng in self.locals.items():
            self._attach(r, eng)

    @property
    def local(self) -> Optional[PipelineServingEngine]:
        return self.locals.get(0)

    def _attach(self, r: int, eng: PipelineServingEngine) -> None:
        eng.on_token = lambda req, t, r=r: self._token(r, int(req.rid), t)
        eng.on_finish = lambda req, r=r: self._finish(r, int(req.rid), req.finish_reason or "done")

    # ---------------------------------------------------------------- API
    def submit(self, req: Request) -> Request:
        with self.lock:
            rid = self._next
            self._next += 1
            req.rid = req.rid or f"q{rid}"
            self.requests[rid] = req
            rep = self.router.place_one(str(rid), req.prompt)
            self.pending[rep].append(rid)
        return req

    def all_done(self) -> bool:
        with self.lock:
            return all(r.done for r in self.requests.values())

    def alive_locals(self) -> Dict[int, PipelineServingEngine]:
        return {r: e for r, e in self.locals.items() if self.router.alive[r]}

    def run(self, poll_s: float = 0.002, stop: bool = True) -> List[Request]:
        for r, link in self.links.items():
            t = threading.Thread(target=self._remote_loop, args=(r, link), daemon=True, name=f"router-{r}")
            t.start()
            self._threads.append(t)
        while not self.all_done():
            busy = False
            for r, eng in list(self.alive_locals().items()):
                self._feed_local(r, eng)
                if eng.idle:
                    continue
                busy = True
                try:
                    eng.run_rounds(1)
                except PipelineFailure as e:
                    self._fail(r, f"local pipeline: {e}")
            self._update_rates()
            if not busy:
                if not any(self.router.alive):
                    raise RuntimeError("every replica failed")
                time.sleep(poll_s)
        for eng in self.alive_locals().values():
            eng.drain()
            if stop:
                eng.stop()
        for t in self._threads:
            t.join(self.timeout_s)
        return [self.requests[k] for k in sorted(self.requests)]

    # ---------------------------------------------------------------- bookkeeping
    def _token(self, r: int, rid: int, tok: int) -> None:
        with self.lock:
            req = self.requests.get(rid)
            if req is None or req.done or self.router.placement.get(str(rid)) != r:
                return
            if req.t_first is None:
                req.t_first = time.perf_counter()
            req.generated.append(int(tok))
            self.router.record(str(rid), int(tok))
            self.replica_tokens[r] += 1
            if self.on_token is not None:
                self.on_token(req, int(tok))

    def _finish(self, r: int, rid: int, reason: str) -> None:
        with self.lock:
            req = self.requests.get(rid)
            if req is None or req.done or self.router.placement.get(str(rid)) != r:
                return
            req.done, req.finish_reason, req.t_done = True, reason, time.perf_counter()
            self.router.close(str(rid))  # finished sessions no longer count as replica load

    def _update_rates(self, period_s: float = 0.5) -> None:
        """Throughput EMA of the locally driven replicas from their delivered tokens/s (remote
        heads report theirs): placement weights follow the measured rates."""
        now = time.perf_counter()
        for r in self.alive_locals():
            t0, n0 = self._rate_mark.get(r, (now, self.replica_tokens[r]))
            if r not in self._rate_mark:
                self._rate_mark[r] = (t0, n0)
                continue
            if now - t0 < period_s:
                continue
            rate = (self.replica_tokens[r] - n0) / (now - t0)
            self._rate_mark[r] = (now, self.replica_tokens[r])
            if rate > 0:
                with self.lock:
                    old = self.router.throughput[r]
                    self.router.throughput[r] = rate if not self._measured[r] else 0.8 * old + 0.2 * rate
                    self._measured[r] = True
                    self.router.heartbeat(r)

    def _take(self, r: int) -> List[Tuple[int, Request]]:
        with self.lock:
            rids, self.pending[r] = self.pending.get(r, []), []
            return [(rid, self.requests[rid]) for rid in rids if not self.requests[rid].done]

    def _feed_local(self, r: int, eng: PipelineServingEngine) -> None:
        for rid, m in self._take(r):
            try:
                eng.submit(Request(list(m.prompt), max_new_tokens=m.max_new_tokens, params=m.params,
                                   eos_token_id=m.eos_token_id, stop_on_repeat=m.stop_on_repeat, seed=m.seed,
                                   rid=str(rid), generated=list(m.generated)))
            except ValueError as e:  # cannot fit this pipeline: finish it instead of killing the front end
                logger.error(f"session {rid} rejected by replica {r}: {e}")
                self._finish(r, rid, "max_length")

    def _fail(self, r: int, why: str) -> None:
        with self.lock:
            if not self.router.alive[r]:
                return
            logger.error(f"replica {r} failed: {why}; re-placing its sessions")
            self.failures.append((r, why))
            self.failure_times.append(time.perf_counter())
            if not self.at_failure:
                self.at_failure = {k: len(q.generated) for k, q in self.requests.items()}
            if self.recover is not None:
                rep = None
                try:
                    rep = self.recover(r)
                except Exception as e:  # noqa: BLE001 - a failed rebuild leaves the survivors
                    logger.error(f"replica {r}: rebuilding a pipeline failed: {e}")
                if rep is not None:
                    eng, thr = rep
                    r2 = self.router.add_replica(thr)
                    self.pending[r2] = []
                    self.replica_tokens.append(0)
                    self._measured.append(False)
                    self.locals[r2] = eng
                    self._attach(r2, eng)
                    logger.info(f"replica {r2} joined (rebuilt after replica {r} failed)")
                    self._resume(r, r2, eng)
            # every unfinished session placed on r (delivered or still pending) moves to a
            # survivor, which re-prefills prompt + generated tokens (the master copies)
            plans = self.router.fail(r)
            self.pending[r] = []
            for plan in plans:
                rid = int(plan.session_id)
                self.pending[plan.replica].append(rid)
                self.replaced.setdefault(rid, len(self.requests[rid].generated))

    def _resume(self, r: int, r2: int, eng: PipelineServingEngine) -> None:
        """Stage-local recovery: a rebuilt replica that replaced only the dead stage of replica
        ``r`` (``eng.resume_target`` = that stage's rank, ``eng.resume_from`` = r's failed head)
        continues r's unfinished sessions from their KV (``PipelineServingEngine.resume_sessions``)
        - no re-prefill; whatever it cannot resume is re-placed by ``router.fail`` as usual."""
        target, old = int(getattr(eng, "resume_target", 0) or 0), getattr(eng, "resume_from", None)
        if target <= 0 or old is None:
            return
        items = []
        for rid_s, (oh, _) in old.failed_sessions.items():
            rid = int(rid_s)
            m = self.requests.get(rid)
            if m is None or m.done or self.router.placement.get(str(rid)) != r or not m.generated:
                continue
            req = Request(list(m.prompt), max_new_tokens=m.max_new_tokens, params=m.params,
                          eos_token_id=m.eos_token_id, stop_on_repeat=m.stop_on_repeat, seed=m.seed,
                          rid=str(rid), generated=list(m.generated))
            items.append((req, int(oh), len(m.prompt) + len(m.generated) - 1))
        for req in eng.resume_sessions(items, target):
            rid = int(req.rid)
            self.router.placement[str(rid)] = r2
            if rid in self.pending.get(r, []):
                self.pending[r].remove(rid)
            self.resumed[rid] = len(req.generated)

    def _remote_loop(self, r: int, link: HostLink) -> None:
        try:
            while True:
                failed, toks, fin, thr = decode_report(link.recv_msg(1, self.timeout_s))
                for rid, t in toks:
                    self._token(r, rid, t)
                for rid, code in fin:
                    self._finish(r, rid, REASON_OF.get(code, "done"))
                if failed:
                    self._fail(r, "head reported a pipeline failure")
                    return
                if thr > 0:
                    with self.lock:
                        self.router.throughput[r] = 0.8 * self.router.throughput[r] + 0.2 * thr
                        self.router.heartbeat(r)
                stop = self.all_done()
                link.send_msg(1, encode_cmd(self._take(r), stop))
                if stop:
                    link.close()
                    return
        except ChannelError as e:
            self._fail(r, f"link: {e}")

"""Split semantics: ``--splits`` cut points -> per-stage block ranges.

Reference: ``--splits`` holds the cut points of a hard-wired 4-stage pipeline
(reference src/main.py:91,248-276,795): stage 0 = [0, s0) + embeddings, stage k =
[s_{k-1}, s_k), the last stage = [s_last, L) + final norm + lm_head.  Generalised here to
any number of cuts (N cuts -> N+1 stages).  A trailing cut equal to L is allowed (the
last stage then only holds norm + head: an *empty* span is an error, as in
src/llama_partition.py:540-541, so a trailing cut == L is dropped instead).
(The reference also exposes ``src/partition.py`` as a re-export shim of
``load_stage_model``; ``load_stage_model`` is re-exported here for the same reason.)
"""
from __future__ import annotations

from typing import List, Sequence, Tuple


def parse_splits(splits, num_layers: int) -> List[int]:
    if isinstance(splits, str):
        parts = [p.strip() for p in splits.split(",") if p.strip()]
        cuts = [int(p) for p in parts]
    else:
        cuts = [int(c) for c in splits]
    if not cuts:
        return []
    if any(c <= 0 for c in cuts):
        raise ValueError(f"split points must be positive: {cuts}")
    if any(b <= a for a, b in zip(cuts, cuts[1:])):
        raise ValueError(f"split points must be strictly increasing: {cuts}")
    if cuts[-1] > num_layers:
        raise ValueError(f"split point {cuts[-1]} exceeds num_layers={num_layers}")
    if cuts[-1] == num_layers:
        cuts = cuts[:-1]
    return cuts


def stage_ranges(cuts: Sequence[int], num_layers: int) -> List[Tuple[int, int]]:
    bounds = [0] + list(cuts) + [num_layers]
    rng = [(bounds[i], bounds[i + 1]) for i in range(len(bounds) - 1)]
    for s, e in rng:
        if e <= s:
            raise ValueError(f"empty stage span [{s}, {e}) from splits {list(cuts)}")
    return rng


def even_splits(num_layers: int, num_stages: int) -> List[int]:
    """Cut points that spread ``num_layers`` over ``num_stages`` as evenly as possible."""
    if num_stages < 1 or num_stages > num_layers:
        raise ValueError(f"cannot split {num_layers} layers into {num_stages} stages")
    base, extra = divmod(num_layers, num_stages)
    cuts, acc = [], 0
    for i in range(num_stages - 1):
        acc += base + (1 if i < extra else 0)
        cuts.append(acc)
    return cuts


# ----------------------------------------------------------------------------- cost model
STREAM_BPS = 5.0e12      # sustained decode-GEMM streaming rate of one MI355X (bytes/s, measured 4.5-5.6)
LAUNCH_S = 2.5e-6        # per-launch cost inside a replayed hipGraph
SAMPLER_FIXED_S = 15e-6  # batched sampler: fixed part (penalty, top-k select, Philox draw)


def stage_cost_model(cfg, *, batch: int = 64, ctx: int = 256, fp8: bool = False) -> Tuple[float, float, float]:
    """Seconds per decode micro-batch step contributed by (one block, the head's extras, the
    tail's extras) - what a pipeline stage actually streams from HBM:

    * block: its weights (1 byte per projection weight on the fp8 W8A16 path, else 2) + the
      micro-batch's KV (``batch`` sessions x ``ctx`` tokens) + 5 launches;
    * head: the embedding gather (``batch`` rows: negligible, the table is not streamed);
    * tail: final norm + ``lm_head`` (bf16, also in fp8 mode) on the last rows + the sampler,
      which makes several passes over ``batch`` x vocab fp32 logits.
    """
    H, V = cfg.hidden_size, cfg.vocab_size
    if fp8 and cfg.model_type != "gpt2":
        wbytes = cfg.layer_param_bytes(1.0) + 2 * H  # e4m3 projections, bf16 norm weights
    else:
        wbytes = cfg.layer_param_bytes(2.0)
    kv = batch * ctx * cfg.kv_bytes_per_token_per_layer(2)
    block = (wbytes + kv) / STREAM_BPS + 5 * LAUNCH_S
    head = batch * H * 2 / STREAM_BPS + LAUNCH_S
    tail = (V * H * 2 + batch * V * 4 * 4) / STREAM_BPS + SAMPLER_FIXED_S + 3 * LAUNCH_S
    return block, head, tail


def balanced_splits(cfg, num_stages: int, *, batch: int = 64, ctx: int = 256, fp8: bool = False,
                    num_layers: int = None) -> List[int]:
    """Cut points that minimise the slowest stage's modelled step time (``stage_cost_model``):
    under a full pipeline the slowest stage sets the node's tokens/s, and the tail carries
    lm_head + sampler on top of its blocks (an fp8 70B's bf16 lm_head alone is ~2.4 blocks).
    Ties (equal max) go to the layout with the smallest sum of squared stage times, i.e. the
    evenest one.  Exact dynamic programme over contiguous spans (L <= 128, S <= 16)."""
    L = int(num_layers or cfg.num_hidden_layers)
    S = int(num_stages)
    if S < 1 or S > L:
        raise ValueError(f"cannot split {L} layers into {S} stages")
    if S == 1:
        return []
    blk, head, tail = stage_cost_model(cfg, batch=batch, ctx=ctx, fp8=fp8)

    def cost(k: int, n: int) -> float:  # stage k holding n blocks
        return n * blk + (head if k == 0 else 0.0) + (tail if k == S - 1 else 0.0)

    INF = (float("inf"), float("inf"))
    # best[k][j]: (max, sum sq) over stages 0..k-1 covering blocks [0, j); arg[k][j]: cut before
    best = [[INF] * (L + 1) for _ in range(S + 1)]
    arg = [[-1] * (L + 1) for _ in range(S + 1)]
    best[0][0] = (0.0, 0.0)
    for k in range(1, S + 1):
        for j in range(k, L - (S - k) + 1):
            for i in range(k - 1, j):
                pm, ps = best[k - 1][i]
                if pm == float("inf"):
                    continue
                c = cost(k - 1, j - i)
                cand = (max(pm, c), ps + c * c)
                if cand[0] < best[k][j][0] - 1e-12 or (abs(cand[0] - best[k][j][0]) <= 1e-12 and
                                                       cand[1] < best[k][j][1]):
                    best[k][j], arg[k][j] = cand, i
    cuts, j = [], L
    for k in range(S, 0, -1):
        i = arg[k][j]
        cuts.append(i)
        j = i
    return sorted(c for c in cuts if c > 0)


def stage_times(cfg, cuts: Sequence[int], **kw) -> List[float]:
    """Modelled seconds per micro-batch step of every stage of ``cuts``."""
    L = cfg.num_hidden_layers
    rng = stage_ranges(cuts, L)
    blk, head, tail = stage_cost_model(cfg, **kw)
    S = len(rng)
    return [(e - s) * blk + (head if k == 0 else 0.0) + (tail if k == S - 1 else 0.0)
            for k, (s, e) in enumerate(rng)]


def resolve_splits(spec: str, cfg, **kw) -> List[int]:
    """``--splits`` value: explicit cut points, or ``auto:N`` = ``balanced_splits`` for N stages."""
    spec = str(spec).strip()
    if spec.startswith("auto"):
        _, _, n = spec.partition(":")
        if not n:
            raise ValueError("--splits auto:N needs the number of stages, e.g. auto:4")
        return balanced_splits(cfg, int(n), **kw)
    return parse_splits(spec, cfg.num_hidden_layers)


def stage_role(stage: int, num_stages: int) -> str:
    if num_stages == 1:
        return "full"
    if stage == 0:
        return "stage0"
    if stage == num_stages - 1:
        return "last"
    return "segment"


def __getattr__(name):  # lazy re-export, like the reference shim src/partition.py:1-8
    if name in ("load_stage_model", "Stage0", "StageSegment", "StageLast"):
        from . import llama_partition

        return getattr(llama_partition, name)
    raise AttributeError(name)

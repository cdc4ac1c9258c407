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

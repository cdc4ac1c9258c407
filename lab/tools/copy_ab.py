"""Timing lab (not a correctness mode): what the per-step host <-> device copies of a 64-session
decode step cost on the GPU timeline.  Runs the 1-GPU bench with

  --skip-meta   the decode graph replays without uploading its metadata blob (the previous
                step's positions / slots / contexts are reused: same kernels and shapes, wrong
                tokens) and without copying the input ids into the graph's static input;
  --skip-d2h    additionally the engine skips the pinned device -> host copy of the tokens;

and prints the bench's JSON line.  Only ms_per_step is meaningful - and only for the variants
that keep refreshing the metadata (--old-ev / --no-token-input / --no-mark / default): every
variant that skips the blob upload (--skip-meta, --skip-blob, --skip-x, --no-rec) replays the
STALE positions / contexts, so attention stops growing over the timed steps and the step looks
~55 us faster for that reason alone (profiles/r5t/README.md).

    python scripts/copy_ab.py --skip-meta -- --steps 20 --warmup 5
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    argv = sys.argv[1:]
    skip_meta, skip_d2h = "--skip-meta" in argv, "--skip-d2h" in argv
    skip_blob, skip_x = "--skip-blob" in argv, "--skip-x" in argv
    x_kernel = "--x-kernel" in argv  # the ids move by an elementwise kernel, not a runtime copy
    no_token_input = "--no-token-input" in argv  # the sampler's ids are copied into the graph input
    no_rec = "--no-rec" in argv    # replay keeps both copies but records no event after the blob copy
    no_mark = "--no-mark" in argv  # no event record after each replay (mark_replayed)
    old_ev = "--old-ev" in argv    # the round-4 replay: an event recorded right behind the blob copy
    if "--" in argv:
        argv = argv[argv.index("--") + 1:]
    import bench
    from src.parallel import engine as eng
    from src.runtime import executor as exm

    state = {"timed": False}
    if no_rec:
        orig3 = exm._DecodeGraph.replay

        def replay3(self, plan, x):
            if not state["timed"] or not getattr(self, "_warm_once", False):
                self._warm_once = True
                return orig3(self, plan, x)
            self._k ^= 1
            self.blob.copy_(self._stage[self._k], non_blocking=True)  # (stale staging: timing only)
            if x.data_ptr() != self.x.data_ptr():
                self.x[:plan.T].copy_(x.view(-1) if self.ex.is_first else x)
            self.graph.replay()
            return self.out[:plan.T]

        exm._DecodeGraph.replay = replay3
    if old_ev:
        import torch

        orig4 = exm._DecodeGraph.replay

        def replay4(self, plan, x):
            b, B = plan.T, self.B
            self._k ^= 1
            k = self._k
            if self._stage_ev[k] is not None:
                self._stage_ev[k].synchronize()
            host = self._stage[k].numpy()
            h64 = host[: 16 * B].view(np.int64).reshape(2, B)
            h32 = host[16 * B:].view(np.int32)
            h64[:, :b] = plan.h64
            h64[0, b:] = 0
            h64[1, b:] = -1
            h32[:b] = plan.h32[:b]
            h32[b:B] = 0
            h32[B:B + b] = plan.h32[b:2 * b]
            h32[B + b:2 * B] = 0
            self.blob.copy_(self._stage[k], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._stage_ev[k] = ev
            if x.data_ptr() != self.x.data_ptr():
                self.x[:b].copy_(x.view(-1) if self.ex.is_first else x)
            self.graph.replay()
            return self.out[:b]

        import numpy as np

        exm._DecodeGraph.replay = replay4
        del orig4
    if no_mark:
        orig_mark = exm._DecodeGraph.mark_replayed

        def mark(self):
            if not state["timed"]:
                return orig_mark(self)

        exm._DecodeGraph.mark_replayed = mark
    if no_token_input:
        exm.StageExecutor.token_input = lambda self, *a, **k: None
    if x_kernel:
        import torch

        orig2 = exm._DecodeGraph.replay

        def replay2(self, plan, x):
            if not state["timed"] or not getattr(self, "_warm_once", False):
                self._warm_once = True
                return orig2(self, plan, x)
            self._k ^= 1
            k = self._k
            if self._stage_ev[k] is not None:
                self._stage_ev[k].synchronize()
            self.blob.copy_(self._stage[k], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._stage_ev[k] = ev
            torch.add(x.view(-1) if self.ex.is_first else x, 0, out=self.x[:plan.T])
            self.graph.replay()
            return self.out[:plan.T]

        exm._DecodeGraph.replay = replay2
    if skip_blob or skip_x:  # one of the two pre-replay copies only
        import numpy as np  # noqa: F401

        orig1 = exm._DecodeGraph.replay

        def replay1(self, plan, x):
            if not state["timed"] or not getattr(self, "_warm_once", False):
                self._warm_once = True
                return orig1(self, plan, x)
            if not skip_blob:
                self._k ^= 1
                self.blob.copy_(self._stage[self._k], non_blocking=True)
            if not skip_x:
                self.x[:plan.T].copy_(x.view(-1) if self.ex.is_first else x)
            self.graph.replay()
            return self.out[:plan.T]

        exm._DecodeGraph.replay = replay1
    if skip_meta:
        orig = exm._DecodeGraph.replay

        def replay(self, plan, x):
            if not state["timed"] or not getattr(self, "_warm_once", False):
                self._warm_once = True
                return orig(self, plan, x)
            self.graph.replay()
            return self.out[:plan.T]

        exm._DecodeGraph.replay = replay
    if skip_d2h:
        orig_consume = eng.PipelineServingEngine._consume

        def consume(self, step):
            if not state["timed"]:
                return orig_consume(self, step)
            if step.consumed:
                return
            step.consumed = True
            if step.waiter is not None:
                step.tok_dev = step.waiter()
            step.tok_host = None  # no host copy: _book sees no tokens

        eng.PipelineServingEngine._consume = consume
    orig_rr = eng.PipelineServingEngine.run_rounds

    def run_rounds(self, n):
        # the timed call is the one with timing on (bench.py sets eng.timing before it)
        state["timed"] = bool(self.timing)
        return orig_rr(self, n)

    eng.PipelineServingEngine.run_rounds = run_rounds
    return bench.main(["--gpus", "1", *argv])


if __name__ == "__main__":
    sys.exit(main())

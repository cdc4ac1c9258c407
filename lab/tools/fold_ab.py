"""Timing lab: the 1-GPU bench with the qkv fold decision forced (``--fold on|off``) instead of
the warm-up A/B (``StageExecutor._confirm_qkv_fold``), so both variants of a build can be timed on
one box.

    python scripts/fold_ab.py --fold on [--lib other_build.so] -- --model llama3-70b --fp8 --steps 20 --warmup 3
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    argv = sys.argv[1:]
    fold = argv[argv.index("--fold") + 1] == "on"
    lib = argv[argv.index("--lib") + 1] if "--lib" in argv else None
    if "--" in argv:
        argv = argv[argv.index("--") + 1:]
    if lib:  # another build of the kernel library (same-box A/B of two builds)
        from src import ops

        ops.LIB_PATH = os.path.abspath(lib)
    import bench
    from src.runtime import executor as exm

    orig = exm.StageExecutor._confirm_qkv_fold

    def forced(self, sids, gen, reps=10):
        t = orig(self, sids, gen, reps)
        if t is None:
            return None
        Bb = self._bucket(len(sids))
        self.qkv_fold_by_bucket[Bb] = fold
        self._graphs.clear()  # re-capture with the forced variant
        return t

    exm.StageExecutor._confirm_qkv_fold = forced
    return bench.main(["--gpus", "1", *argv])


if __name__ == "__main__":
    sys.exit(main())

"""A/B of the GQA decode attention kernel on the 1-GPU bench: ``--valu`` puts decode steps on the
flash-decoding kernel (csrc/attention.hip, 4 heads of a group per workgroup) instead of the MFMA
kernel (csrc/attention_mfma.hip).  Prefill keeps the MFMA kernels either way.

    python scripts/gqa_decode_ab.py --valu -- --model llama3-70b --fp8 --steps 10 --warmup 3
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    argv = sys.argv[1:]
    valu = "--valu" in argv
    if "--" in argv:
        argv = argv[argv.index("--") + 1:]
    import bench
    from src.runtime import executor as exm

    if valu:
        init = exm.StageExecutor.__init__

        def patched(self, *a, **k):
            init(self, *a, **k)
            self.gqa_decode_mfma = False
            self._attn_min_part = 64

        exm.StageExecutor.__init__ = patched
    return bench.main(["--gpus", "1", *argv])


if __name__ == "__main__":
    sys.exit(main())

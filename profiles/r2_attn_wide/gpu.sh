set -o pipefail
# 16-wave flash-decoding workgroups for small grids (batch 1: no split-K / reduce launch)
O=gpurun_out/r2_attn_wide
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or attn or decode or rope or engine" > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > $O/b1_wide.log 2>&1 && \
MPAMD_ATTN_WIDE_WGS=0 timeout -k 10 300 python -u bench.py --batch 1 > $O/b1_nowide.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 --prompt-len 2048 > $O/b1_long_wide.log 2>&1 && \
MPAMD_ATTN_WIDE_WGS=0 timeout -k 10 300 python -u bench.py --batch 1 --prompt-len 2048 > $O/b1_long_nowide.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/b64.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python3 bench.py --batch 1 --steps 16 --warmup 4 > $O/prof1.log 2>&1

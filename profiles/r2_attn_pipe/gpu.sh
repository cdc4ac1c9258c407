set -o pipefail
# software-pipelined single-pass flash-decoding loop (MPAMD_ATTN_PIPE) A/B
O=gpurun_out/r2_attn_pipe
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or attn or decode or rope" > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/b64_pipe.log 2>&1 && \
MPAMD_ATTN_PIPE=0 timeout -k 10 300 python -u bench.py > $O/b64_nopipe.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 128 > $O/b128_pipe.log 2>&1 && \
MPAMD_ATTN_PIPE=0 timeout -k 10 300 python -u bench.py --batch 128 > $O/b128_nopipe.log 2>&1 && \
timeout -k 10 300 python -u bench.py --prompt-len 1024 --batch 32 > $O/b32_1k_pipe.log 2>&1 && \
MPAMD_ATTN_PIPE=0 timeout -k 10 300 python -u bench.py --prompt-len 1024 --batch 32 > $O/b32_1k_nopipe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run -- python3 bench.py --steps 16 --warmup 4 > $O/prof64.log 2>&1

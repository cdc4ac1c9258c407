set -o pipefail
# single-pass (online-softmax) flash-decoding attention vs the two-pass kernel
O=gpurun_out/r2_attn1pass
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or attn or decode or rope" > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/b64_1pass.log 2>&1 && \
MPAMD_ATTN_1PASS=0 timeout -k 10 300 python -u bench.py > $O/b64_2pass.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > $O/b1_1pass.log 2>&1 && \
MPAMD_ATTN_1PASS=0 timeout -k 10 300 python -u bench.py --batch 1 > $O/b1_2pass.log 2>&1 && \
MPAMD_ATTN_INLAUNCH_REDUCE=1 timeout -k 10 300 python -u bench.py --batch 1 > $O/b1_1pass_inlaunch.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 --prompt-len 2048 > $O/b1_long_1pass.log 2>&1 && \
MPAMD_ATTN_1PASS=0 timeout -k 10 300 python -u bench.py --batch 1 --prompt-len 2048 > $O/b1_long_2pass.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run -- python3 bench.py --steps 16 --warmup 4 > $O/prof64.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python3 bench.py --batch 1 --steps 16 --warmup 4 > $O/prof1.log 2>&1

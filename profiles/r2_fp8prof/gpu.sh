set -o pipefail
# 70B fp8 kernel table; batch-1 attention split A/B (MPAMD_ATTN_MIN_PART)
O=gpurun_out/r2_fp8prof
mkdir -p $O
export TMPDIR=/tmp
MPAMD_ATTN_MIN_PART=256 timeout -k 10 300 python -u bench.py --batch 1 > $O/b1_minpart256.log 2>&1 && \
MPAMD_ATTN_MIN_PART=128 timeout -k 10 300 python -u bench.py --batch 1 > $O/b1_minpart128.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > $O/b1_default.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof70 -o run -- python3 bench.py --model llama3-70b --fp8 --steps 6 --warmup 2 > $O/prof70.log 2>&1

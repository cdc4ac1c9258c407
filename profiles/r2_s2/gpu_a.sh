set -o pipefail
# round 2, session 2: re-baseline the restored tree - GPU suite, bench (64 / 1 / 128 sessions),
# 70B fp8 and a rocprofv3 kernel table of the 64-session step
O=gpurun_out/r2_s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench64.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 1 > $O/bench1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch 128 > $O/bench128.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model llama3-70b --fp8 --steps 8 --warmup 2 > $O/bench70.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run -- python3 bench.py --steps 16 --warmup 4 > $O/prof64.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python3 bench.py --batch 1 --steps 16 --warmup 4 > $O/prof1.log 2>&1

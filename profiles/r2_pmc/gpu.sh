set -o pipefail
# PMC passes over a short 64-session bench (one counter group per run)
O=gpurun_out/r2_pmc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 bench.py --steps 4 --warmup 2 > $O/fetch.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/hit -o run -- python3 bench.py --steps 4 --warmup 2 > $O/hit.log 2>&1

set -o pipefail
# host overhead of a pipeline stage's decode step at the pp8 / pp4 / pp2 stage sizes
O=gpurun_out/r2_stage_overhead
mkdir -p $O
for L in 4 8 16; do
  timeout -k 10 200 python -u scripts/stage_overhead.py --layers $L --batch 64 >> $O/overhead.jsonl 2> $O/err_$L.log || exit 1
done
timeout -k 10 200 python -u scripts/stage_overhead.py --layers 4 --batch 16 >> $O/overhead.jsonl 2> $O/err_4b16.log

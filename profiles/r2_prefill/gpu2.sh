set -o pipefail
# warm prefill throughput (scripts/prefill_bench.py) + a kernel table of the warm 2K prefill
O=gpurun_out/r2_prefill
mkdir -p $O
export TMPDIR=/tmp
for cfg in "--batch 1 --prompt-len 2048" "--batch 8 --prompt-len 2048" "--batch 64 --prompt-len 128" "--batch 1 --prompt-len 8192"; do
  timeout -k 10 300 python -u scripts/prefill_bench.py $cfg >> $O/prefill.jsonl 2>> $O/prefill_err.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_p2k -o run -- python3 scripts/prefill_bench.py --batch 1 --prompt-len 2048 --repeats 2 > $O/prof_p2k.log 2>&1

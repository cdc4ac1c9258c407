#!/bin/bash
# Round 5: CLI pipeline (device channel) vs single-process greedy generation on one GPU, small-llama.
set -o pipefail
O=gpurun_out/${1:-r5s}
mkdir -p $O
timeout -k 10 200 python3 scripts/single_gpu_check.py --model small-llama --max_new_tokens 12 --device cuda > $O/single.txt 2>&1 || exit 1
timeout -k 10 300 python3 scripts/run_all.py --model small-llama --splits 2,4 --gpus --max_new_tokens 12 --base_port 29890 --log_dir $O/pipe --extra "--kv_cache_gb 1" > $O/pipe.txt 2>&1 || exit 1
timeout -k 10 300 python3 scripts/run_all.py --model small-llama --splits 2,4 --max_new_tokens 12 --base_port 29850 --log_dir $O/cpu > $O/cpu.txt 2>&1 || exit 1
timeout -k 10 200 python3 scripts/single_gpu_check.py --model small-llama --max_new_tokens 12 --device cpu > $O/single_cpu.txt 2>&1 || exit 1
grep -h "Generated\|Top5" $O/single.txt $O/single_cpu.txt; grep -h -A1 "GENERATED" $O/pipe.txt $O/cpu.txt

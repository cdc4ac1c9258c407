set -o pipefail
# grouped MFMA prefill attention (4 query blocks per workgroup share each K/V step)
O=gpurun_out/r2_prefill_grp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_engine_gpu.py tests/test_hf_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or attn or prefill or executor or engine or superblock or query" > $O/tests.log 2>&1 && \
for cfg in "--batch 1 --prompt-len 2048" "--batch 8 --prompt-len 2048" "--batch 64 --prompt-len 128" "--batch 1 --prompt-len 8192"; do
  timeout -k 10 300 python -u scripts/prefill_bench.py $cfg >> $O/prefill_grp.jsonl 2>> $O/err.log || exit 1
  MPAMD_ATTN_GROUPED=0 timeout -k 10 300 python -u scripts/prefill_bench.py $cfg >> $O/prefill_nogrp.jsonl 2>> $O/err.log || exit 1
done
timeout -k 10 300 python -u scripts/prefill_bench.py --model llama3-8b --batch 1 --prompt-len 8192 >> $O/prefill_grp.jsonl 2>> $O/err.log && \
MPAMD_ATTN_GROUPED=0 timeout -k 10 300 python -u scripts/prefill_bench.py --model llama3-8b --batch 1 --prompt-len 8192 >> $O/prefill_nogrp.jsonl 2>> $O/err.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_p2k -o run -- python3 scripts/prefill_bench.py --batch 1 --prompt-len 2048 --repeats 2 > $O/prof_p2k.log 2>&1

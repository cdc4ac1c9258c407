set -o pipefail
O=gpurun_out/r3_fa2
mkdir -p $O
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 "$@" || { echo "STEP FAILED: $name rc=$?" >> $O/steps.log; exit 1; }; echo "ok $name" >> $O/steps.log; }
run tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_norm.py tests/test_fp8.py -m gpu -k "attention_fa or fa_blocks or rwk or producer or consumer or w8a16 or fp8_gemm or gemm" > $O/tests.log 2>&1
run attn 300 python -u scripts/attn_bench.py > $O/attn.jsonl 2>$O/attn.err
run attn_decode 200 python -u scripts/attn_decode_bench.py > $O/attn_decode.jsonl 2>$O/attn_decode.err
for cfg in "1 2048" "1 8192" "64 128"; do set -- $cfg
  run prefill_$1x$2 120 env MPAMD_FA_WAVES=8 python -u scripts/prefill_bench.py --batch $1 --prompt-len $2 >> $O/prefill_w8.jsonl 2>>$O/prefill.err
done
run b64 300 python -u bench.py > $O/b64.log 2>&1
run b256 300 python -u bench.py --batch 256 --steps 16 --warmup 4 > $O/b256.log 2>&1
run prof256 300 rocprofv3 --kernel-trace --stats -d $O/prof256 -o run -- python3 bench.py --batch 256 --steps 8 --warmup 2 > $O/prof256.log 2>&1

set -o pipefail
O=gpurun_out/r3_g
mkdir -p $O
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 "$@" || { echo "STEP FAILED: $name rc=$?" >> $O/steps.log; exit 1; }; echo "ok $name" >> $O/steps.log; }
run b256 300 python -u bench.py --batch 256 --steps 16 --warmup 4 > $O/b256.log 2>&1
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_VERBOSE=1
run b256_tune 600 env PYTORCH_TUNABLEOP_TUNING=1 python -u bench.py --batch 256 --steps 16 --warmup 4 > $O/b256_tune.log 2>&1
run b256_tuned 300 env PYTORCH_TUNABLEOP_TUNING=0 python -u bench.py --batch 256 --steps 16 --warmup 4 > $O/b256_tuned.log 2>&1
unset PYTORCH_TUNABLEOP_ENABLED
run pf8k 300 python -u scripts/prefill_bench.py --batch 1 --prompt-len 8192 > $O/pf8k.jsonl 2>$O/pf8k.err
run pf8k_tune 600 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 python -u scripts/prefill_bench.py --batch 1 --prompt-len 8192 > $O/pf8k_tune.jsonl 2>$O/pf8k_tune.err
ls -la $O > $O/ls.txt

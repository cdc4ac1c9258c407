set -u
mkdir -p gpurun_out/mb
run() { name=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/mb/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -h '"metric"' gpurun_out/mb/$name.log | tail -1 | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run b1 --batch 1 --steps 64 --warmup 8
run l3_8b --model llama3-8b
run l70_fp8 --model llama3-70b --fp8 --steps 8 --warmup 2
run b128 --batch 128 --steps 16 --warmup 4

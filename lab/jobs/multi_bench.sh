set -u
mkdir -p gpurun_out/mb
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/mb/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/mb/pytest.log
run() { name=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/mb/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; grep -h '"metric"' gpurun_out/mb/$name.log | tail -1 | cut -c150-330; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run l3_8b --model llama3-8b
run l70_fp8 --model llama3-70b --fp8 --steps 8 --warmup 2
run base

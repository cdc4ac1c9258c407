#!/bin/bash
# Round 6: fence-free stream events (runtime/hip_events.py) - GPU tests, then the 64-session and batch-1
# 7B benches A/B (MPAMD_DEVICE_EVENTS=1 vs 0, interleaved), then the step-boundary trace with them on.
set -o pipefail
O=gpurun_out/${1:-r6dev}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_events.py \
  tests/test_graph_input_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for b in 64 1; do
    for e in 1 0; do
      MPAMD_DEVICE_EVENTS=$e timeout -k 10 300 python3 bench.py --gpus 1 --batch $b --steps 40 --warmup 8 \
        > $O/b${b}_e${e}_r$r.json 2> $O/b${b}_e${e}_r$r.err || { tail -20 $O/b${b}_e${e}_r$r.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" $O/b${b}_e${e}_r$r.json
    done
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p64 -o run -- python3 bench.py --gpus 1 --batch 64 --steps 20 --warmup 5 \
  > $O/b64_prof.json 2> $O/b64_prof.err || exit 1
DB=$(find $O/p64 -name "*.db" | head -1)
python3 lab/tools/prof_gaps.py $DB --steps 20 > $O/b64_gaps.txt || exit 1
python3 lab/tools/prof_boundary.py $DB > $O/b64_boundary.txt && rm -rf $O/p64 || exit 1
head -14 $O/b64_gaps.txt

#!/bin/bash
# Round 6: W8A8-MX opt-in mode end to end (o projection, MX input from the attention epilogue) - MX tests
# (incl. the executor mode), then Llama-3-70B fp8
# 64 sessions with MPAMD_FP8_MODE=mx vs the W8A16 default, interleaved.
set -o pipefail
O=gpurun_out/${1:-r6mx70}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_mx_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for m in mx w8a16; do
    MPAMD_FP8_MODE=$m timeout -k 10 300 python3 bench.py --model llama3-70b --fp8 --steps 20 --warmup 3 > $O/b70_${m}_$r.json 2> $O/b70_${m}_$r.err || { tail -20 $O/b70_${m}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], d['value'], d['dtype'][:24])" $O/b70_${m}_$r.json
  done
done

#!/bin/bash
# Fused first-stage entry (embedding gather inside the mode-3 stage-entry kernel): GPU tests of the
# touched paths, then interleaved bench A/B (MPAMD_FUSED_ENTRY=0 / 1) at 64 sessions and batch 1.
set -o pipefail
O=gpurun_out/${1:-r6entry}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_fused_norm.py tests/test_executor_gpu.py tests/test_mx_gpu.py tests/test_graph_input_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for rep in 1 2 3; do
  for fe in 0 1; do
    for b in 64 1; do
      MPAMD_FUSED_ENTRY=$fe timeout -k 10 200 python3 bench.py --batch $b > $O/b${b}_e${fe}_$rep.json 2> $O/b${b}_e${fe}_$rep.err || exit 1
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], d['value'])" $O/b${b}_e${fe}_$rep.json
    done
  done
done

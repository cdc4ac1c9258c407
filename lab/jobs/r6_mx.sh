#!/bin/bash
# Round 6: W8A8-MX decode GEMM - the scaled-MFMA probes, the MX oracle tests, then MX vs W8A16 per
# projection shape (isolated, cold weights).
set -o pipefail
O=gpurun_out/${1:-r6mx}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 5 60 ./lab/hip/mx_probe.bin > $O/probe.txt 2>&1; tail -1 $O/probe.txt
[ "${SKIPT:-0}" = 1 ] || timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_mx_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 lab/tools/mx_ab.py > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
MPAMD_MX_NT=8 timeout -k 10 300 python3 lab/tools/mx_ab.py --ms 64 > $O/ab_nt8.jsonl 2> $O/ab_nt8.err || { tail -20 $O/ab_nt8.err; exit 1; }
echo "--- MPAMD_MX_NT=8"; cat $O/ab_nt8.jsonl

#!/bin/bash
# Round 6: host time inside hipGraphLaunch of the 7B decode graph vs HIP runtime settings.
set -o pipefail
O=gpurun_out/${1:-r6gl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name, env assignments...
  local n=$1; shift
  env "$@" timeout -k 10 240 python3 lab/tools/decode_host_probe.py --batch ${B:-64} > $O/$n.json 2> $O/$n.err \
    || { tail -5 $O/$n.err; return 1; }
  echo "$n $(cat $O/$n.json)"
}
run base || exit 1
run sig1k ROC_SIGNAL_POOL_SIZE=1024 || exit 1
run aql16k ROC_AQL_QUEUE_SIZE=16384 || exit 1
run gbatch DEBUG_HIP_GRAPH_BATCH_SIZE=1024 || exit 1
run cbatch DEBUG_CLR_MAX_BATCH_SIZE=1024 || exit 1
run pcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
run pcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
run devka HIP_FORCE_DEV_KERNARG=1 || exit 1
run cpusync DEBUG_CLR_BATCH_CPU_SYNC_SIZE=4096 || exit 1
B=1 run b1_base || exit 1
B=1 run b1_sig1k ROC_SIGNAL_POOL_SIZE=1024 || exit 1

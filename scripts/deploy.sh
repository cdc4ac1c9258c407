#!/bin/bash
# Start one swarm process (stage server or stage-0 client) on this machine, in the background.
#
# Counterpart of the reference's scripts/deploy_direct.sh + initial_install.sh, minus
# the venv / pip / hivemind-from-source steps: the only dependencies are PyTorch-ROCm and the
# in-tree HIP/C++ extensions, which this script builds once (hipcc --offload-arch=gfx950).
# A previous instance of the SAME stage started by this script is stopped through its pid file
# (never by matching command lines).
#
#   scripts/deploy.sh STAGE [MODEL] [SPLITS] [INITIAL_PEERS] [PUBLIC_IP] [-- extra src.main flags]
#
# Ports: DHT = BASE_PORT + 2*STAGE, RPC = BASE_PORT + 2*STAGE + 1 (BASE_PORT default 8000); set
# PUBLIC_DHT_PORT / PUBLIC_RPC_PORT when a NAT / port-forward maps them (docs/PORTS.md).
set -euo pipefail

STAGE=${1:?usage: deploy.sh STAGE [MODEL] [SPLITS] [INITIAL_PEERS] [PUBLIC_IP] [-- extra flags]}
MODEL=${2:-llama2-7b}
SPLITS=${3:-8,16,24}
PEERS=${4:-}
PUBLIC_IP=${5:-}
shift $(( $# < 5 ? $# : 5 ))
[ "${1:-}" = "--" ] && shift
BASE_PORT=${BASE_PORT:-8000}
DHT_PORT=${DHT_PORT:-$((BASE_PORT + 2 * STAGE))}
RPC_PORT=${RPC_PORT:-$((BASE_PORT + 2 * STAGE + 1))}
LOG_DIR=${LOG_DIR:-logs}
PROMPT=${PROMPT:-"Hello, how are you?"}
MAX_NEW_TOKENS=${MAX_NEW_TOKENS:-32}

cd "$(dirname "$0")/.."
mkdir -p "$LOG_DIR"
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}

# build the gfx950 kernels + C++ runtime in-tree if they are missing
if ! ls global_capstone_design_distributed-inference-of-llms-over-the-internet_amd/ops/_mpamd_kernels*.so >/dev/null 2>&1; then
  echo "building HIP kernels and the native runtime ..."
  python -c "import __graft_entry__ as g; g.build()"
fi

PIDFILE="$LOG_DIR/stage${STAGE}.pid"
if [ -f "$PIDFILE" ] && kill -0 "$(cat "$PIDFILE")" 2>/dev/null; then
  echo "stopping previous stage $STAGE (pid $(cat "$PIDFILE"))"
  kill -TERM "$(cat "$PIDFILE")" || true
  sleep 2
fi

ARGS=(python -m src.main --model "$MODEL" --splits "$SPLITS" --stage "$STAGE"
      --dht_port "$DHT_PORT" --rpc_port "$RPC_PORT")
[ -n "$PEERS" ] && ARGS+=(--dht_initial_peers "$PEERS")
[ -n "$PUBLIC_IP" ] && ARGS+=(--public_ip "$PUBLIC_IP")
[ -n "${PUBLIC_DHT_PORT:-}" ] && ARGS+=(--public_dht_port "$PUBLIC_DHT_PORT")
[ -n "${PUBLIC_RPC_PORT:-}" ] && ARGS+=(--public_rpc_port "$PUBLIC_RPC_PORT")
[ "$STAGE" -eq 0 ] && ARGS+=(--prompt "$PROMPT" --max_new_tokens "$MAX_NEW_TOKENS")
ARGS+=("$@")

echo "stage $STAGE: ${ARGS[*]}"
nohup "${ARGS[@]}" > "$LOG_DIR/stage${STAGE}.log" 2>&1 &
echo $! > "$PIDFILE"
echo "pid $(cat "$PIDFILE"); log: tail -f $LOG_DIR/stage${STAGE}.log; stop: kill \$(cat $PIDFILE)"
if [ "$STAGE" -ne 0 ]; then
  # servers print their registry multiaddr once the handlers are up; show it for the next hosts
  for _ in $(seq 1 120); do
    if grep -q "handlers registered" "$LOG_DIR/stage${STAGE}.log" 2>/dev/null; then
      grep -o "DHT visible multiaddrs: .*" "$LOG_DIR/stage${STAGE}.log" | head -n 1 || true
      exit 0
    fi
    kill -0 "$(cat "$PIDFILE")" 2>/dev/null || { echo "stage $STAGE exited:"; tail -n 20 "$LOG_DIR/stage${STAGE}.log"; exit 1; }
    sleep 1
  done
  echo "stage $STAGE not ready after 120 s (see the log)"
fi

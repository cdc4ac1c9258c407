#!/bin/bash
# Keep a deployed checkout up to date (reference scripts/auto_pull.sh,
# simple_auto_pull.sh): every INTERVAL seconds fetch BRANCH and fast-forward when the remote moved.
# After an update the in-tree HIP/C++ extensions are rebuilt (they are not tracked by git) and the
# optional RESTART command runs (e.g. "scripts/deploy.sh 1 llama2-7b 8,16,24 <peers>").
#
#   scripts/auto_pull.sh [REPO_DIR] [BRANCH] [INTERVAL] [RESTART_CMD]
#   ONCE=1 scripts/auto_pull.sh ...      # single check (cron)
set -uo pipefail

REPO_DIR=${1:-.}
BRANCH=${2:-main}
INTERVAL=${3:-60}
RESTART=${4:-}
cd "$REPO_DIR" || exit 1
LOG=${LOG:-auto_pull.log}

log() { echo "[$(date '+%F %T')] $*" | tee -a "$LOG"; }

check_once() {
  if ! git fetch -q origin "$BRANCH" 2>>"$LOG"; then
    log "fetch failed"; return 1
  fi
  local here there
  here=$(git rev-parse HEAD)
  there=$(git rev-parse "origin/$BRANCH")
  [ "$here" = "$there" ] && return 0
  if ! git merge-base --is-ancestor "$here" "$there"; then
    log "local branch diverged from origin/$BRANCH; not touching it"; return 1
  fi
  if git merge -q --ff-only "origin/$BRANCH" 2>>"$LOG"; then
    log "updated ${here:0:10} -> ${there:0:10}"
    python -c "import __graft_entry__ as g; g.build()" >>"$LOG" 2>&1 || log "rebuild failed"
    if [ -n "$RESTART" ]; then
      log "restart: $RESTART"
      bash -c "$RESTART" >>"$LOG" 2>&1 || log "restart command failed"
    fi
  else
    log "fast-forward failed"; return 1
  fi
}

log "watching $(pwd) branch $BRANCH every ${INTERVAL}s"
if [ -n "${ONCE:-}" ]; then
  check_once
  exit $?
fi
while true; do
  check_once || true
  sleep "$INTERVAL"
done

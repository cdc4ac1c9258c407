#!/bin/bash
# Install scripts/auto_pull.sh as a service (reference scripts/setup_auto_pull.sh).
# Prefers a systemd *user* unit (no root needed); falls back to a crontab entry (ONCE mode, every
# minute) when systemd is not available.  Prints the unit / cron line; DRY_RUN=1 only prints.
#
#   scripts/setup_auto_pull.sh [REPO_DIR] [BRANCH] [INTERVAL] [RESTART_CMD]
set -euo pipefail

REPO_DIR=$(cd "${1:-.}" && pwd)
BRANCH=${2:-main}
INTERVAL=${3:-60}
RESTART=${4:-}
SCRIPT="$REPO_DIR/scripts/auto_pull.sh"
NAME=mini-petals-auto-pull

UNIT="[Unit]
Description=Mini-Petals MI355X auto git pull ($REPO_DIR, $BRANCH)
After=network-online.target

[Service]
Type=simple
WorkingDirectory=$REPO_DIR
ExecStart=/bin/bash $SCRIPT $REPO_DIR $BRANCH $INTERVAL '$RESTART'
Restart=always
RestartSec=10

[Install]
WantedBy=default.target"

if [ -n "${DRY_RUN:-}" ]; then
  echo "$UNIT"
  exit 0
fi

if command -v systemctl >/dev/null 2>&1 && systemctl --user show-environment >/dev/null 2>&1; then
  mkdir -p "$HOME/.config/systemd/user"
  echo "$UNIT" > "$HOME/.config/systemd/user/$NAME.service"
  systemctl --user daemon-reload
  systemctl --user enable --now "$NAME.service"
  echo "installed: systemctl --user status $NAME; logs in $REPO_DIR/auto_pull.log"
else
  LINE="* * * * * cd $REPO_DIR && ONCE=1 /bin/bash $SCRIPT $REPO_DIR $BRANCH $INTERVAL '$RESTART' >/dev/null 2>&1"
  ( crontab -l 2>/dev/null | grep -v "$SCRIPT" ; echo "$LINE" ) | crontab -
  echo "installed cron entry: $LINE"
fi

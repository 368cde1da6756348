#!/usr/bin/env bash
# Stop daemons started by alluxio-start.sh using the exact PIDs it recorded.
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
LOGS="${ALLUXIO_LOGS_DIR:-${HERE}/logs}"
for f in "${LOGS}"/*.pid; do
  [ -e "$f" ] || continue
  pid="$(cat "$f")"
  kill "$pid" 2>/dev/null && echo "stopped $(basename "$f" .pid) ($pid)"
  rm -f "$f"
done

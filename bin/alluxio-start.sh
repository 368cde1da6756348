#!/usr/bin/env bash
# Start the node's daemons (reference bin/alluxio-start.sh): `master`, `workers` (one worker process
# per visible MI355X, pinned with HIP_VISIBLE_DEVICES), `proxy`, `logserver`, or `all`.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
LOGS="${ALLUXIO_LOGS_DIR:-${HERE}/logs}"
mkdir -p "${LOGS}"
what="${1:-all}"
ngpu="$(python3 -c 'import torch; print(torch.cuda.device_count())' 2>/dev/null || echo 0)"
start_master() { nohup "${HERE}/bin/alluxio" master > "${LOGS}/master.out" 2>&1 & echo $! > "${LOGS}/master.pid"; }
start_workers() {
  local n=$(( ngpu > 0 ? ngpu : 1 ))
  for ((i = 0; i < n; i++)); do
    HIP_VISIBLE_DEVICES=$i nohup "${HERE}/bin/alluxio" worker --device 0 --port $((29999 + 10 * i)) \
      > "${LOGS}/worker${i}.out" 2>&1 &
    echo $! > "${LOGS}/worker${i}.pid"
  done
}
start_proxy() { nohup "${HERE}/bin/alluxio" proxy > "${LOGS}/proxy.out" 2>&1 & echo $! > "${LOGS}/proxy.pid"; }
start_logserver() { nohup "${HERE}/bin/alluxio" logserver > "${LOGS}/logserver.out" 2>&1 & echo $! > "${LOGS}/logserver.pid"; }
case "${what}" in
  master) start_master ;;
  workers|worker) start_workers ;;
  proxy) start_proxy ;;
  logserver) start_logserver ;;
  all) start_master; sleep 2; start_workers; start_proxy ;;
  *) echo "usage: $0 [all|master|workers|proxy|logserver]"; exit 1 ;;
esac

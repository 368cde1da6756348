#!/usr/bin/env bash
# Cluster bootstrap for cloud Hadoop services (reference integration/emr/alluxio-emr.sh and
# integration/dataproc/alluxio-dataproc.sh): install the distribution tarball built by
# tools/release.py, write alluxio-site.properties for this node's role, give every MI355X GPU its
# own worker with an HBM tier (one worker per GPU, DRAM + NVMe below it), and start the processes.
#
#   alluxio-bootstrap.sh -p emr|dataproc|vagrant -t <tarball path or s3://|gs://|http(s):// URI>
#                        [-m <master hostname>] [-r master|worker|auto] [-u <root UFS URI>]
#                        [-s key=value ...] [-n] (-n: configure only, do not start)
set -euo pipefail

PLATFORM=""; TARBALL=""; MASTER=""; ROLE="auto"; ROOT_UFS=""; START=1
declare -a PROPS=()
while getopts "p:t:m:r:u:s:n" o; do
  case "$o" in
    p) PLATFORM="$OPTARG" ;; t) TARBALL="$OPTARG" ;; m) MASTER="$OPTARG" ;; r) ROLE="$OPTARG" ;;
    u) ROOT_UFS="$OPTARG" ;; s) PROPS+=("$OPTARG") ;; n) START=0 ;;
    *) echo "usage: $0 -p emr|dataproc|vagrant -t tarball [-m master] [-r role] [-u ufs] [-s k=v] [-n]" >&2; exit 2 ;;
  esac
done
[[ -n "$PLATFORM" && -n "$TARBALL" ]] || { echo "-p and -t are required" >&2; exit 2; }
PREFIX="${ALLUXIO_PREFIX:-/opt}"
HOME_DIR="${PREFIX}/alluxio-amd"

fetch() {  # fetch <uri> <dest>
  case "$1" in
    s3://*) aws s3 cp "$1" "$2" ;;
    gs://*) gsutil cp "$1" "$2" ;;
    http://*|https://*) curl -fsSL -o "$2" "$1" ;;
    *) cp "$1" "$2" ;;
  esac
}

detect_role() {  # platform metadata says whether this node is the master
  case "$PLATFORM" in
    emr) grep -q '"isMaster": *true' /mnt/var/lib/info/instance.json 2>/dev/null && echo master || echo worker ;;
    dataproc) [[ "$(/usr/share/google/get_metadata_value attributes/dataproc-role 2>/dev/null)" == "Master" ]] \
                && echo master || echo worker ;;
    *) [[ "$(hostname -s)" == "${MASTER%%.*}" ]] && echo master || echo worker ;;
  esac
}

detect_master() {
  case "$PLATFORM" in
    emr) grep -o '"masterHost": *"[^"]*"' /mnt/var/lib/info/job-flow.json 2>/dev/null | cut -d'"' -f4 || true ;;
    dataproc) /usr/share/google/get_metadata_value attributes/dataproc-master 2>/dev/null || true ;;
  esac
}

default_ufs() {
  case "$PLATFORM" in
    emr) echo "s3://$(hostname -s)-alluxio/" ;;
    dataproc) echo "gs://$(/usr/share/google/get_metadata_value attributes/dataproc-bucket 2>/dev/null)/alluxio/" ;;
    *) echo "${HOME_DIR}/underFSStorage" ;;
  esac
}

gpu_count() {  # MI355X GPUs visible on this node (0 on CPU-only nodes)
  if command -v rocm-smi >/dev/null 2>&1; then
    rocm-smi --showid 2>/dev/null | grep -c '^GPU\[' || true
  else
    ls -d /sys/class/kfd/kfd/topology/nodes/*/ 2>/dev/null | while read -r n; do
      grep -q 'gfx_target_version [1-9]' "$n/properties" 2>/dev/null && echo x; done | wc -l
  fi
}

install_dist() {
  mkdir -p "$PREFIX"
  local tmp; tmp="$(mktemp -d)"
  fetch "$TARBALL" "$tmp/dist.tar.gz"
  tar -xzf "$tmp/dist.tar.gz" -C "$PREFIX"
  local top; top="$(tar -tzf "$tmp/dist.tar.gz" | awk -F/ 'NR == 1 {print $1}')"
  rm -rf "$HOME_DIR"; ln -sfn "${PREFIX}/${top}" "$HOME_DIR"
  (cd "$HOME_DIR" && sha256sum -c --quiet MANIFEST.sha256)
  rm -rf "$tmp"
}

write_conf() {  # write_conf <role> <ngpus>
  local conf="${HOME_DIR}/conf/alluxio-site.properties"
  {
    echo "alluxio.master.hostname=${MASTER}"
    echo "alluxio.master.mount.table.root.ufs=${ROOT_UFS}"
    echo "alluxio.master.journal.type=UFS"
    echo "alluxio.master.journal.folder=${HOME_DIR}/journal"
    echo "alluxio.worker.tieredstore.levels=2"
    echo "alluxio.worker.tieredstore.level0.alias=MEM"
    echo "alluxio.worker.tieredstore.level0.dirs.path=hbm"
    echo "alluxio.worker.tieredstore.level0.dirs.quota=200GB"
    echo "alluxio.worker.tieredstore.level1.alias=SSD"
    echo "alluxio.worker.tieredstore.level1.dirs.path=$(ls -d /mnt/nvme* /local_ssd 2>/dev/null | paste -sd, - || echo /tmp)"
    echo "alluxio.worker.hbm.page.size=2MB"
    for kv in "${PROPS[@]+"${PROPS[@]}"}"; do echo "$kv"; done
  } > "$conf"
  echo "$conf"
}

start_processes() {  # start_processes <role> <ngpus>
  cd "$HOME_DIR"
  if [[ "$1" == master ]]; then
    ./bin/alluxio format -s
    ./bin/alluxio-start.sh master
    ./bin/alluxio-start.sh job_master || true
    ./bin/alluxio-start.sh proxy || true
  fi
  if [[ "$2" -gt 0 ]]; then   # one worker per GPU: HIP_VISIBLE_DEVICES pins worker i to GPU i
    for ((i = 0; i < $2; i++)); do
      HIP_VISIBLE_DEVICES="$i" ALLUXIO_WORKER_INDEX="$i" ./bin/alluxio-start.sh worker
    done
  elif [[ "$1" == worker ]]; then
    ./bin/alluxio-start.sh worker -Dalluxio.worker.tieredstore.level0.dirs.path=dram
  fi
}

main() {
  install_dist
  [[ "$ROLE" == auto ]] && ROLE="$(detect_role)"
  [[ -n "$MASTER" ]] || MASTER="$(detect_master)"
  [[ -n "$MASTER" ]] || MASTER="$(hostname -f)"
  [[ -n "$ROOT_UFS" ]] || ROOT_UFS="$(default_ufs)"
  local ngpu; ngpu="$(gpu_count)"
  write_conf "$ROLE" "$ngpu"
  echo "alluxio-amd ${PLATFORM}: role=${ROLE} master=${MASTER} gpus=${ngpu} ufs=${ROOT_UFS}"
  [[ "$START" == 1 ]] && start_processes "$ROLE" "$ngpu"
  return 0
}

main "$@"

#!/bin/bash
# One GPU session: tests, smoke, bench variants, rocprof.  Each GPU step has its own timeout and
# the script stops at the first crash-like exit (fault/abort/segv/timeout); plain test failures
# (exit 1) do not stop later measurement steps.
# usage: tools/gpu_round.sh [steps...]   steps: tests smoke bench bench20 variants prof ring pmc pmcdram
#                                         crc dl master kbench lz4t lz4 ... (every `name)` below);
#   round-5 validation: `validate` (GPU tests, smoke, bench at the driver's 20 steps) and `rehearse`;
#   round-5 write path: ctrep (CACHE_THROUGH tee vs two streams), persist, s3ct, s3ctmt;
#   round-5 bench A/B: arenaab (native vs caching-allocator arena), batchab (HIP batching knobs)
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
STEPS="${*:-tests smoke bench variants prof}"

run() {  # name timeout cmd...
  local name=$1; local t=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/round.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/round.log"
  tail -3 "$OUT/$name.log" | tee -a "$OUT/round.log"
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then
    echo "STOP: $name ended with rc=$rc (crash/timeout); no further GPU steps" | tee -a "$OUT/round.log"
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" ;;
    bench) run bench_default 400 python bench.py ;;
    bench20) run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    variants)
      run bench_buf4m 300 python bench.py --buffer-size 4m --steps 200 --warmup 20
      run bench_buf1m 300 python bench.py --buffer-size 1m
      run bench_buf64k 300 python bench.py --buffer-size 64k
      run bench_file1g 400 python bench.py --file-size 1g --steps 200
      run bench_host 400 python bench.py --dest host --steps 20 --warmup 3
      run bench_host4m 400 python bench.py --dest host --buffer-size 4m --steps 20 --warmup 3
      ;;
    prof)
      run rocprof_bench 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 bench.py --steps 50 --warmup 5
      ;;
    lz4t) run lz4_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k lz4 -x -v --timeout 120 --timeout-method thread ;;
    lz4) run lz4_bench 600 python tools/lz4_bench.py --chunks 1024,4096,16384,32768 --variants="${LZ4_VARIANTS:-2,17,19,20,21,22}" --out "$OUT/lz4_bench.jsonl" ;;
    config5)
      run ingest_config5 900 python tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 1,3 --threads 4 --out "$OUT/ufs_ingest_config5_s3native.jsonl"
      run ingest_config5_t8 600 python tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 3 --threads 8 --out "$OUT/ufs_ingest_config5_s3native.jsonl"
      run rocprof_config5 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof_config5" -o c5 --output-format csv -- python3 tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 3 --threads 4
      ;;
    mastertiming)
      # CPU-only: where one CreateFile's time goes (ALLUXIO_MASTER_OP_TIMING) and the master's CPU
      for pt in "8 8" "16 4" "32 2"; do
        set -- $pt
        ALLUXIO_MASTER_OP_TIMING="$PWD/$OUT/master_optiming_p$1.json" run master_timing_p$1 300 python tools/master_bench_mp.py --ops CreateFile,DeleteFile --procs $1 --threads $2 --duration 5s --client-prop alluxio.user.network.native.rpc.enabled=false --out "$OUT/master_bench_timing_p$1.json"
      done
      ;;
    mastergrpc2)
      [ -n "${SKIP_P8:-}" ] || run master_bench_grpc_p8 500 python tools/master_bench_mp.py --ops CreateFile,GetFileStatus,ListDir,DeleteFile,GetFileStatusNonexistent --procs 8 --threads 8 --duration 5s --client-prop alluxio.user.network.native.rpc.enabled=false --out "$OUT/master_bench_grpc_p8.json"
      run master_bench_grpc_p32 500 python tools/master_bench_mp.py --ops CreateFile,GetFileStatus,ListDir,DeleteFile,GetFileStatusNonexistent --procs 32 --threads 2 --duration 5s --client-prop alluxio.user.network.native.rpc.enabled=false --out "$OUT/master_bench_grpc_p32.json"
      run master_bench_grpc_p16 500 python tools/master_bench_mp.py --ops CreateFile,GetFileStatus,ListDir,DeleteFile,GetFileStatusNonexistent --procs 16 --threads 4 --duration 5s --client-prop alluxio.user.network.native.rpc.enabled=false --out "$OUT/master_bench_grpc_p16.json"
      ;;
    k7mixed) run pytest_k7mixed 300 python -u -m pytest tests/test_evict_alloc_gpu.py -k "magazine" -x -v --timeout 120 --timeout-method thread ;;
    c5t8) run ingest_config5_t8 600 python tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 3 --threads 8 --out "$OUT/ufs_ingest_config5_t8.jsonl" ;;
    c5ahead)
      run ingest_config5_ahead4 600 python tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 3 --threads 4 --free-ahead 512m --out "$OUT/ufs_ingest_config5_ahead.jsonl"
      run ingest_config5_ahead8 600 python tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 3 --threads 8 --free-ahead 512m --out "$OUT/ufs_ingest_config5_ahead.jsonl"
      ;;
    hdfsgw)
      run hdfs_gateway_bench 600 python tools/hdfs_gateway_bench.py --file-size 2g --threads 1,4,8 --write-threads 1,4,8 --out "$OUT/hdfs_gateway.jsonl"
      ;;
    s3ingest)
      run ingest_s3native 600 python tools/ufs_ingest_bench.py --ufs s3native --hbm 2g --dram 6g --factor 2 --depths 1,3 --out "$OUT/ufs_ingest_s3native.jsonl"
      run ingest_s3requests 600 python tools/ufs_ingest_bench.py --ufs s3native --native-reader false --hbm 2g --dram 6g --factor 2 --depths 3 --out "$OUT/ufs_ingest_s3native.jsonl"
      ;;
    lz4pmc)
      for v in ${LZ4_PMC_VARIANTS:-20}; do
        run lz4pmc_a_v$v 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d "$OUT/lz4pmc_a_v$v" -o pmc --output-format csv -- python3 tools/lz4_one.py --variant $v --data text --chunks 4096
        run lz4pmc_b_v$v 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-trace -d "$OUT/lz4pmc_b_v$v" -o pmc --output-format csv -- python3 tools/lz4_one.py --variant $v --data text --chunks 4096
      done
      ;;
    crc) run crc_bench 300 python tools/crc_bench.py --gb 4 --out "$OUT/crc_bench.jsonl" ;;
    dl) run dl_bench_100k 400 python tools/dl_bench.py --files 100000 --out "$OUT/dl_bench_100k.jsonl" ;;
    dl1m) run dl_bench_1m 900 python tools/dl_bench.py --ufs synthetic --files 1000000 --threads 32 --out "$OUT/dl_bench_1m.jsonl" ;;
    master)
      # CPU-only: the master metadata bench on the box's CPU share (no GPU used)
      run master_bench 500 python tools/master_bench_mp.py --ops CreateFile,GetFileStatus,ListDir,DeleteFile,GetFileStatusNonexistent --procs 4 --threads 8 --duration 5s --out "$OUT/master_bench.json"
      ;;
    mastergrpc)
      run master_bench_native 500 python tools/master_bench_mp.py --ops CreateFile,GetFileStatus,ListDir,DeleteFile,GetFileStatusNonexistent --procs 4 --threads 8 --duration 5s --out "$OUT/master_bench_native.json"
      # CPU-only: stock gRPC (grpcio) clients against the master port, which the native front end
      # serves (alluxio.master.rpc.native.grpc.enabled, default on), and against the grpcio server
      run master_bench_grpc_native 500 python tools/master_bench_mp.py --ops CreateFile,GetFileStatus,ListDir,DeleteFile,GetFileStatusNonexistent --procs 4 --threads 8 --duration 5s --client-prop alluxio.user.network.native.rpc.enabled=false --out "$OUT/master_bench_grpc_native.json"
      run master_bench_grpcio 500 python tools/master_bench_mp.py --ops CreateFile,GetFileStatus,ListDir,DeleteFile,GetFileStatusNonexistent --procs 4 --threads 8 --duration 5s --client-prop alluxio.user.network.native.rpc.enabled=false --master-prop alluxio.master.rpc.native.grpc.enabled=false --out "$OUT/master_bench_grpcio.json"
      ;;
    ring)
      run bench_ring4k 300 python bench.py --buffer-size 4k --steps 200 --warmup 20
      run bench_ring4k_d64 300 python bench.py --buffer-size 4k --depth 64 --steps 200 --warmup 20
      run bench_ring4k_d1024 300 python bench.py --buffer-size 4k --depth 1024 --steps 100 --warmup 10
      run bench_ring64k 300 python bench.py --buffer-size 64k --steps 200 --warmup 20
      run bench_ring4k_f1g 300 python bench.py --buffer-size 4k --file-size 1g --steps 200 --warmup 20
      run rocprof_ring 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_ring" -o ring --output-format csv -- python3 bench.py --buffer-size 4k --steps 50 --warmup 5
      ;;
    pmc)
      # one small counter group per pass (a big derived set aborts with "exceeds the capabilities")
      run rocprof_pmc_rd 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --stats -d "$OUT/pmc_rd" -o pmc --output-format csv -- python3 bench.py --steps 10 --warmup 1
      run rocprof_pmc_wr 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace --stats -d "$OUT/pmc_wr" -o pmc --output-format csv -- python3 bench.py --steps 10 --warmup 1
      run rocprof_pmc_dram 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --kernel-trace --stats -d "$OUT/pmc_dram" -o pmc --output-format csv -- python3 bench.py --steps 10 --warmup 1
      ;;
    pmcdram)
      # HBM bytes behind the lockstep (local) and staggered readers, one counter pass each
      run pmc_dram_local 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --kernel-trace --stats -d "$OUT/pmc_dram_local" -o pmc --output-format csv -- python3 bench.py --steps 20 --warmup 2 --phases local
      run pmc_dram_stagger 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --kernel-trace --stats -d "$OUT/pmc_dram_stagger" -o pmc --output-format csv -- python3 bench.py --steps 20 --warmup 2 --phases local,stagger
      ;;
    large)
      # the HBM-resident read rate: 16 GiB file, staggered streams (DRAM read bytes ~= delivered)
      run bench_large 400 python bench.py --steps 20 --warmup 5 --phases local,stagger,large
      run pmc_dram_large 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --kernel-trace --stats -d "$OUT/pmc_dram_large" -o pmc --output-format csv -- python3 bench.py --steps 20 --warmup 2 --phases local,large
      ;;
    k9put)
      run pytest_pc 300 python -u -m pytest tests/test_page_cache_native.py -x -v --timeout 120 --timeout-method thread
      run page_cache_put 400 python tools/page_cache_bench.py --page-sizes 4k,64k,2m --out "$OUT/page_cache_put.jsonl"
      run rocprof_pc_put 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_pc_put" -o pcput --output-format csv -- python3 tools/page_cache_bench.py --page-sizes 4k --iters 5
      ;;
    hostipc)
      run worker_bench_ipc 300 python tools/worker_bench_host.py --threads 16 --transports ipc --duration 4s --warmup 1s --out "$OUT/worker_bench_ipc.jsonl"
      ;;
    datapath)
      run pytest_datapath 400 python -u -m pytest tests/test_ipc_gpu.py tests/test_data_server.py -x -v --timeout 120 --timeout-method thread
      run wb_host_4k 900 python tools/worker_bench_host.py --threads 16,64,256 --transports grpc,ipc --duration 8s --warmup 2s --out "$OUT/worker_bench_host_native.jsonl"
      run wb_host_1m 600 python tools/worker_bench_host.py --threads 16,64 --buffer-size 1m --transports grpc,ipc --duration 8s --warmup 2s --reader-buffer 4MB --out "$OUT/worker_bench_host_native_1m.jsonl"
      run wb_host_grpcio 300 python tools/worker_bench_host.py --threads 16 --transports grpcio --duration 8s --warmup 2s --out "$OUT/worker_bench_host_native.jsonl"
      ;;
    datapath2)
      run pytest_datapath 400 python -u -m pytest tests/test_ipc_gpu.py tests/test_data_server.py -x -v --timeout 120 --timeout-method thread
      run wb_host_4k_pf 900 python tools/worker_bench_host.py --threads 16,64,256 --transports grpc,ipc --duration 8s --warmup 2s --out "$OUT/worker_bench_host_prefetch.jsonl"
      run wb_host_4k_pf2m 900 python tools/worker_bench_host.py --threads 16,256 --transports grpc,ipc --duration 8s --warmup 2s --reader-buffer 2MB --out "$OUT/worker_bench_host_prefetch.jsonl"
      run wb_host_1m_pf 600 python tools/worker_bench_host.py --threads 16,64 --buffer-size 1m --transports grpc,ipc --duration 8s --warmup 2s --reader-buffer 4MB --out "$OUT/worker_bench_host_prefetch_1m.jsonl"
      ;;
    prefetchab)
      for pf in true false; do
        run wb_host_ab_$pf 900 python tools/worker_bench_host.py --threads 16,256 --transports grpc,ipc --duration 8s --warmup 2s --client-prop alluxio.user.native.reader.prefetch.enabled=$pf --out "$OUT/worker_bench_host_prefetch_ab.jsonl"
      done
      ;;
    writes)
      run pytest_dataserver 300 python -u -m pytest tests/test_data_server.py tests/test_ipc_gpu.py -x -v --timeout 120 --timeout-method thread
      run worker_write_bench 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --transports grpc,ipc --out "$OUT/worker_write_bench.jsonl"
      run wb_host_after_writes 600 python tools/worker_bench_host.py --threads 16,256 --transports grpc,ipc --duration 6s --warmup 2s --out "$OUT/worker_bench_host_r4b.jsonl"
      ;;
    through)
      run ww_through 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type THROUGH --out "$OUT/worker_write_through.jsonl"
      run ww_cache_through 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/worker_write_through.jsonl"
      run ww_through_python 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type THROUGH --client-prop alluxio.user.native.writer.enabled=false --worker-prop alluxio.worker.data.server.native.ufs.write.enabled=false --out "$OUT/worker_write_through.jsonl"
      ;;
    cthrough)
      run ww_cache_through2 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/worker_write_through.jsonl"
      ;;
    cthroughab)
      run ww_ct_overlap 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/worker_write_cache_through_ab.jsonl"
      run ww_ct_serial 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type CACHE_THROUGH --client-prop alluxio.user.file.cache.through.overlap.min=1GB --out "$OUT/worker_write_cache_through_ab.jsonl"
      run ww_ct_overlap2 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/worker_write_cache_through_ab.jsonl"
      ;;
    writebase)
      run worker_write_bench_grpcio 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --transports grpc --client-prop alluxio.user.native.writer.enabled=false --out "$OUT/worker_write_bench_grpcio.jsonl"
      ;;
    rehearse)
      run bench_rehearse_2rank 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --one-device --steps 10 --warmup 3
      run bench_rehearse_4rank 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --one-device --steps 10 --warmup 3
      ;;
    lz4encprof)
      run rocprof_lz4enc 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_lz4enc" -o lz4enc --output-format csv -- python3 tools/lz4_bench.py --chunks 1024 --variants=-1
      ;;
    hostprocs)
      run wb_host_procs4 600 python tools/worker_bench_host.py --threads 16,64,256 --transports grpc,ipc --duration 6s --warmup 2s --client-procs 4 --out "$OUT/worker_bench_host_procs.jsonl"
      run wb_host_procs8 600 python tools/worker_bench_host.py --threads 256 --transports grpc,ipc --duration 6s --warmup 2s --client-procs 8 --out "$OUT/worker_bench_host_procs.jsonl"
      ;;
    zerocopy)
      for d in host cuda; do
        run remote_${d}_p1 300 python tools/remote_device_read_bench.py --dest $d --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=1 --out "$OUT/remote_read_zero_copy.jsonl"
        run remote_${d}_p4 300 python tools/remote_device_read_bench.py --dest $d --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=4 --out "$OUT/remote_read_zero_copy.jsonl"
      done
      rm -f "$OUT/read_trace.jsonl"
      ALLUXIO_READ_TRACE="$PWD/$OUT/read_trace.jsonl" run remote_host_trace 300 python tools/remote_device_read_bench.py --dest host --file-size 512m --read-size 512m --reps 1 --native-only --client-prop alluxio.user.device.read.parallelism=1 --out "$OUT/remote_read_traced.jsonl"
      ;;
    windowab)
      for d in host cuda; do
        run wab_${d}_base 300 python tools/remote_device_read_bench.py --dest $d --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=1 --out "$OUT/remote_read_window_ab.jsonl"
        run wab_${d}_w16 300 python tools/remote_device_read_bench.py --dest $d --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=1 --worker-prop alluxio.worker.network.reader.buffer.size=16MB --out "$OUT/remote_read_window_ab.jsonl"
        run wab_${d}_w16c2 300 python tools/remote_device_read_bench.py --dest $d --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=1 --client-prop alluxio.user.network.reader.chunk.size.bytes=2MB --worker-prop alluxio.worker.network.reader.buffer.size=16MB --out "$OUT/remote_read_window_ab.jsonl"
      done
      ;;
    writescale)
      run ww_ct_r5 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/r5_worker_write_cache_through.jsonl"
      run ingest_c5_t4 600 python tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 3 --threads 4 --out "$OUT/r5_ufs_ingest_config5.jsonl"
      run ingest_c5_t8 600 python tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 3 --threads 8 --out "$OUT/r5_ufs_ingest_config5.jsonl"
      ALLUXIO_MOVE_COPY_KERNEL=0 run ingest_c5_t8_runtimecopy 600 python tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 3 --threads 8 --out "$OUT/r5_ufs_ingest_config5_runtime_copy.jsonl"
      run rocprof_c5_t8 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof_c5_r5" -o c5 --output-format csv -- python3 tools/ufs_ingest_bench.py --ufs s3native --hbm 4g --dram 8g --factor 2 --depths 3 --threads 8
      ;;
    ctpair)
      run ww_ct_pair 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/r5_worker_write_cache_through.jsonl"
      ;;
    wdiag)
      run ww_diag_ct 600 python tools/worker_write_bench.py --threads 1,4,8,16 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/r5_worker_write_diag.jsonl"
      run ww_diag_mc 600 python tools/worker_write_bench.py --threads 4,16 --file-size 256m --write-type MUST_CACHE --out "$OUT/r5_worker_write_diag.jsonl"
      run ww_diag_th 600 python tools/worker_write_bench.py --threads 4,16 --file-size 256m --write-type THROUGH --out "$OUT/r5_worker_write_diag.jsonl"
      ;;
    ctio)
      run ww_ct_async 600 python tools/worker_write_bench.py --threads 1,4,8,16 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/r5_worker_write_cache_through.jsonl"
      run ww_ct_io16 600 python tools/worker_write_bench.py --threads 4,8,16 --file-size 256m --write-type CACHE_THROUGH --worker-prop alluxio.worker.data.server.native.io.threads=16 --out "$OUT/r5_worker_write_cache_through_io16.jsonl"
      run ww_mc_async 600 python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --write-type MUST_CACHE --out "$OUT/r5_worker_write_must_cache.jsonl"
      ;;
    ctnuma)
      run ww_ct_bound 600 python tools/worker_write_bench.py --threads 1,4,8,16 --file-size 256m --write-type CACHE_THROUGH --bind-gpu-node --out "$OUT/r5_worker_write_cache_through_bound.jsonl"
      run ww_ct_bound_io16 600 python tools/worker_write_bench.py --threads 1,4,8,16 --file-size 256m --write-type CACHE_THROUGH --bind-gpu-node --worker-prop alluxio.worker.data.server.native.io.threads=16 --out "$OUT/r5_worker_write_cache_through_bound.jsonl"
      run numa_bound_1m_b 600 python tools/worker_bench_host.py --threads 64 --transports ipc --duration 6s --warmup 2s --client-procs 4 --d2h-roof --bind-gpu-node --out "$OUT/r5_host_read_numa_bound2.jsonl"
      run numa_bound_4m_b 600 python tools/worker_bench_host.py --threads 64 --transports ipc --duration 6s --warmup 2s --client-procs 4 --d2h-roof --bind-gpu-node --reader-buffer 4MB --out "$OUT/r5_host_read_numa_bound2.jsonl"
      ;;
    ctshm)
      run ww_ct_shm 600 python tools/worker_write_bench.py --threads 1,4,8,16 --file-size 256m --write-type CACHE_THROUGH --bind-gpu-node --work-dir /dev/shm --out "$OUT/r5_worker_write_cache_through_shm.jsonl"
      run ww_th_shm 600 python tools/worker_write_bench.py --threads 1,4,8,16 --file-size 256m --write-type THROUGH --bind-gpu-node --work-dir /dev/shm --out "$OUT/r5_worker_write_cache_through_shm.jsonl"
      ;;
    cttiming)
      run ww_ct_timing 600 python tools/worker_write_bench.py --threads 4,8,16 --file-size 256m --write-type CACHE_THROUGH --bind-gpu-node --client-timing "$PWD/$OUT/ct_timing" --out "$OUT/r5_worker_write_ct_timing.jsonl"
      run ww_mc_timing 600 python tools/worker_write_bench.py --threads 4,8,16 --file-size 256m --write-type MUST_CACHE --bind-gpu-node --client-timing "$PWD/$OUT/ct_timing" --out "$OUT/r5_worker_write_ct_timing.jsonl"
      ;;
    ctfinal)
      run ww_ct_final 600 python tools/worker_write_bench.py --threads 1,4,8,16 --file-size 256m --write-type CACHE_THROUGH --client-timing "$PWD/$OUT/ct_timing" --out "$OUT/r5_worker_write_cache_through_final.jsonl"
      run ww_mc_final 600 python tools/worker_write_bench.py --threads 1,4,8,16 --file-size 256m --write-type MUST_CACHE --out "$OUT/r5_worker_write_cache_through_final.jsonl"
      ;;
    arenaab)
      run bench_arena_native_a 400 python bench.py
      export ALLUXIO_HBM_ARENA_TORCH=1
      run bench_arena_torch_a 400 python bench.py
      run rocprof_arena_torch 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_arena_torch" -o bench --output-format csv -- python3 bench.py --steps 50 --warmup 5
      unset ALLUXIO_HBM_ARENA_TORCH
      run rocprof_arena_native 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_arena_native" -o bench --output-format csv -- python3 bench.py --steps 50 --warmup 5
      run bench_arena_native_b 400 python bench.py
      export ALLUXIO_HBM_ARENA_TORCH=1
      run bench_arena_torch_b 400 python bench.py
      unset ALLUXIO_HBM_ARENA_TORCH
      ;;
    batchab)
      run bench_batch_default 400 python bench.py --phases local,duration
      export DEBUG_CLR_MAX_BATCH_SIZE=4096
      run bench_batch_4096 400 python bench.py --phases local,duration
      run rocprof_batch_4096 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_batch_4096" -o bench --output-format csv -- python3 bench.py --phases local,duration --duration 1
      unset DEBUG_CLR_MAX_BATCH_SIZE
      export DEBUG_CLR_BATCH_CPU_SYNC_SIZE=4096
      run bench_cpusync_4096 400 python bench.py --phases local,duration
      unset DEBUG_CLR_BATCH_CPU_SYNC_SIZE
      ;;
    ctrep)
      run ww_ct_rep 900 python tools/worker_write_bench.py --threads 1,4,8,16 --files 4 --repeat 3 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/r5_worker_write_cache_through_tee.jsonl"
      run ww_ct_rep_bound 900 python tools/worker_write_bench.py --threads 4,8,16 --files 4 --repeat 3 --file-size 256m --write-type CACHE_THROUGH --bind-gpu-node --work-dir /dev/shm --out "$OUT/r5_worker_write_cache_through_tee.jsonl"
      run ww_ct_rep_notee 900 python tools/worker_write_bench.py --threads 4,8,16 --files 4 --repeat 2 --file-size 256m --write-type CACHE_THROUGH --client-prop alluxio.user.file.cache.through.tee.enabled=false --out "$OUT/r5_worker_write_cache_through_tee.jsonl"
      ;;
    persist)
      run persist_bench 600 python tools/persist_bench.py --threads 1,4,8 --files 4 --file-size 512m --out "$OUT/r5_persist_bench.jsonl"
      run persist_bench_s3 600 python tools/persist_bench.py --ufs s3 --threads 1,4,8 --files 2 --file-size 512m --out "$OUT/r5_persist_bench.jsonl"
      ;;
    s3ct)
      run s3_ct_tee 600 python tools/s3_write_bench.py --size 4g --paths through --write-type CACHE_THROUGH --tier hbm:0 --out "$OUT/r5_s3_cache_through.jsonl"
      run s3_ct_notee 600 python tools/s3_write_bench.py --size 4g --paths through --write-type CACHE_THROUGH --tier hbm:0 --client-prop alluxio.user.file.cache.through.tee.enabled=false --out "$OUT/r5_s3_cache_through.jsonl"
      run s3_through 600 python tools/s3_write_bench.py --size 4g --paths through --tier hbm:0 --out "$OUT/r5_s3_cache_through.jsonl"
      ;;
    s3ctmt)
      run ww_s3_ct_tee 600 python tools/worker_write_bench.py --s3 --threads 1,4,16 --files 2 --file-size 256m --write-type CACHE_THROUGH --client-prop alluxio.user.file.cache.through.tee.object.store.enabled=true --out "$OUT/r5_s3_cache_through_threads.jsonl"
      run ww_s3_ct_two 600 python tools/worker_write_bench.py --s3 --threads 1,4,16 --files 2 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/r5_s3_cache_through_threads.jsonl"
      ;;
    r6uds)
      # round 6: one ReadBlock stream (and four) over the worker's Unix domain socket vs loopback TCP
      for d in host cuda; do
        for par in 1 4; do
          run uds_${d}_p$par 300 python tools/remote_device_read_bench.py --uds --dest $d --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/r6_remote_read_uds.jsonl"
          run tcp_${d}_p$par 300 python tools/remote_device_read_bench.py --dest $d --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/r6_remote_read_uds.jsonl"
        done
      done
      ;;
    r6large)
      run bench_large_r6 400 python bench.py --steps 20 --warmup 5 --phases local,stagger,large
      run copy_roof_r6 300 python tools/copy_roof.py --gib 4 --out "$OUT/r6_copy_roof.json"
      run pmc_dram_large_r6 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --kernel-trace --stats -d "$OUT/pmc_dram_large_r6" -o pmc --output-format csv -- python3 bench.py --steps 20 --warmup 2 --phases local,large
      ;;
    r6w8s)
      # sustained 8 s writes, 64 MiB blocks (the round-6 commit target rows)
      run ww8_mc 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --out "$OUT/r6_worker_write_8s.jsonl"
      run ww8_ct 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/r6_worker_write_8s.jsonl"
      ;;
    r6commit)
      # native block commit: sustained 8 s writes, 64 MiB blocks, loopback TCP and the (now default) domain socket
      run ww8nc_mc_tcp 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_worker_write_8s_native_commit.jsonl"
      run ww8nc_ct_tcp 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_worker_write_8s_native_commit.jsonl"
      run ww8nc_mc_uds 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --out "$OUT/r6_worker_write_8s_native_commit.jsonl"
      run ww8nc_ct_uds 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/r6_worker_write_8s_native_commit.jsonl"
      ;;
    r6stress)
      # native StressWorkerBench client: T C++ reader threads in ONE client process, 4 KiB read(buf)
      run wb_native_4k 900 python tools/worker_bench_host.py --mode native-threads --threads 16,64,256 --transports grpc,ipc --duration 6s --warmup 2s --d2h-roof --out "$OUT/r6_worker_bench_native_threads.jsonl"
      ;;
    r6wprof)
      # where the bench process's Python CPU goes during sustained 16-thread writes
      run ww8_prof_mc 600 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --py-sample --out "$OUT/r6_worker_write_pyprof.jsonl"
      run ww8_prof_ct 600 python tools/worker_write_bench.py --threads 1,16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --py-sample --out "$OUT/r6_worker_write_pyprof.jsonl"
      ;;
    r6ct)
      # CACHE_THROUGH only, after the tee pieces went back to whole blocks
      run ww8ct_tcp 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_worker_write_ct.jsonl"
      run ww8ct_uds 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --out "$OUT/r6_worker_write_ct.jsonl"
      ;;
    r6cttime)
      # where one CACHE_THROUGH file's time goes at 1 and 16 writers (client phases + master/worker handlers)
      run ww_ct_time1 300 python tools/worker_write_bench.py --threads 1 --files 4 --min-seconds 6 --file-size 256m --write-type CACHE_THROUGH --client-timing "$OUT/r6_ct_timing" --out "$OUT/r6_ct_timing.jsonl"
      run ww_mc_time1 300 python tools/worker_write_bench.py --threads 1 --files 4 --min-seconds 6 --file-size 256m --write-type MUST_CACHE --client-timing "$OUT/r6_mc_timing" --out "$OUT/r6_ct_timing.jsonl"
      run ww_th_time1 300 python tools/worker_write_bench.py --threads 1 --files 4 --min-seconds 6 --file-size 256m --write-type THROUGH --client-timing "$OUT/r6_th_timing" --out "$OUT/r6_ct_timing.jsonl"
      ;;
    r6coldab)
      # cold single stream: UFS slot size / depth A/B (default 8 MiB x 3)
      for sd in "2MB 8" "4MB 4" "8MB 3"; do
        set -- $sd
        run cold_s$1 300 python tools/remote_device_read_bench.py --uds --cold --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=1 --worker-prop alluxio.worker.ufs.ingest.chunk.size=$1 --worker-prop alluxio.worker.ufs.ingest.depth=$2 --out "$OUT/r6_cold_slot_ab.jsonl"
      done
      run cached_s 300 python tools/remote_device_read_bench.py --uds --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=1 --out "$OUT/r6_cold_slot_ab.jsonl"
      ;;
    r6io)
      # 16 writers with more data-server I/O threads (one connection per thread instead of two)
      for io in 16 24; do
        run ww_mc_io$io 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.native.io.threads=$io --out "$OUT/r6_worker_write_io.jsonl"
        run ww_ct_io$io 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --worker-prop alluxio.worker.data.server.native.io.threads=$io --out "$OUT/r6_worker_write_io.jsonl"
      done
      ;;
    r6wkern)
      # kernel trace of sustained native writes: the per-page CRC32C kernel runs on the write streams,
      # once per committed HBM block, next to the H2D copies
      run rocprof_writes 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof_writes" -o w --output-format csv -- python3 tools/worker_write_bench.py --threads 4 --files 4 --min-seconds 4 --file-size 256m --write-type MUST_CACHE --out "$OUT/r6_write_kernels.jsonl"
      ;;
    r6crc)
      # one CRC launch pair per committed block (paged kernel): correctness, write sweep, kernel counts
      run pytest_crc 300 python -u -m pytest tests/test_native_commit.py tests/test_kernels_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread
      run ww_crc_mc 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_writes_paged_crc.jsonl"
      run rocprof_writes_paged 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_writes_paged" -o w --output-format csv -- python3 tools/worker_write_bench.py --threads 4 --files 4 --min-seconds 4 --file-size 256m --write-type MUST_CACHE --out "$OUT/r6_write_kernels_paged.jsonl"
      ;;
    r6freeahead)
      # creates that must evict: one radix-select per create vs freeing 1 GiB ahead
      run ww_fa0 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_free_ahead.jsonl"
      run ww_fa1g 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --worker-prop alluxio.worker.tieredstore.free.ahead.bytes=1GB --out "$OUT/r6_free_ahead.jsonl"
      run ww_fa1g_ct 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --worker-prop alluxio.worker.tieredstore.free.ahead.bytes=1GB --out "$OUT/r6_free_ahead.jsonl"
      ;;
    r6freeahead2)
      for fa in 0 256MB 1GB; do
        run ww_ct_fa_$fa 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --worker-prop alluxio.worker.tieredstore.free.ahead.bytes=$fa --out "$OUT/r6_free_ahead2.jsonl"
        run ww_mc_fa_$fa 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --worker-prop alluxio.worker.tieredstore.free.ahead.bytes=$fa --out "$OUT/r6_free_ahead2.jsonl"
      done
      ;;
    r6wdefault)
      # sustained writes with the defaults (HBM eviction batches on)
      run ww_def_mc 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_writes_evict_batch.jsonl"
      run ww_def_ct 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_writes_evict_batch.jsonl"
      ;;
    r6startab)
      # next-block stream start on / off, cold and cached single stream, same box
      for ns in true false; do
        run cold_ns_$ns 300 python tools/remote_device_read_bench.py --uds --cold --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=1 --client-prop alluxio.user.native.reader.next.block.start.enabled=$ns --out "$OUT/r6_next_block_start_ab.jsonl"
        run cached_ns_$ns 300 python tools/remote_device_read_bench.py --uds --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=1 --client-prop alluxio.user.native.reader.next.block.start.enabled=$ns --out "$OUT/r6_next_block_start_ab.jsonl"
      done
      ;;
    r6wsize)
      # is the 16-writer ceiling the client's per-call cost? the same writes with larger write() calls
      for ws in 1m 4m 16m; do
        run ww_ws_$ws 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --write-size $ws --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_write_size.jsonl"
      done
      ;;
    r6wcall)
      # 16 writers x 1 MiB: one write() call's time against the native sink call inside it
      run ww_call 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 6 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --client-timing "$OUT/r6_wcall" --out "$OUT/r6_wcall.jsonl"
      ;;
    r6wwin)
      # 16 writers x 1 MiB with larger HTTP/2 stream windows on the data server
      for win in 4MB 16MB 32MB; do
        run ww_win_$win 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --worker-prop alluxio.worker.data.server.native.write.window=$win --out "$OUT/r6_write_window.jsonl"
      done
      run ww_win_uds16 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.native.write.window=16MB --out "$OUT/r6_write_window.jsonl"
      ;;
    r6wwin2)
      for rep in 1 2; do
        for win in 4MB 32MB 64MB; do
          run ww_win2_${win}_$rep 300 python tools/worker_write_bench.py --threads 16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --worker-prop alluxio.worker.data.server.native.write.window=$win --out "$OUT/r6_write_window2.jsonl"
        done
      done
      ;;
    r6final)
      # the round's closing numbers on one box: tests, smoke, driver-shape bench, writes, stress, cold, fan-out
      run pytest_gpu_final6 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
      run smoke_final6 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()"
      run bench_final6 300 python bench.py --gpus 1 --steps 20 --warmup 5
      run ww_final_mc 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type MUST_CACHE --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_final_writes.jsonl"
      run ww_final_ct 600 python tools/worker_write_bench.py --threads 1,4,16 --files 4 --min-seconds 8 --file-size 256m --write-type CACHE_THROUGH --worker-prop alluxio.worker.data.server.domain.socket.default.enabled=false --out "$OUT/r6_final_writes.jsonl"
      run wb_final 900 python tools/worker_bench_host.py --mode native-threads --threads 16,64,256 --transports grpc,ipc --duration 6s --warmup 2s --d2h-roof --out "$OUT/r6_final_stress.jsonl"
      for par in 1 4; do
        run cold_final_p$par 300 python tools/remote_device_read_bench.py --uds --cold --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/r6_final_cold.jsonl"
        run cached_final_p$par 300 python tools/remote_device_read_bench.py --uds --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/r6_final_cold.jsonl"
      done
      run fanout_final 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 8 --one-device --steps 10 --warmup 3 --phases local,replicate --profile-json "$OUT/r6_final_fanout.json"
      ;;
    r6fanout)
      # replica fan-out breakdown: 8 ranks (8 workers) on the one GPU, 3 replicas per block
      run bench_rehearse_8rank_r6 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 8 --one-device --steps 10 --warmup 3 --phases local,replicate --profile-json "$OUT/r6_rehearse_8rank.json"
      ;;
    r6create)
      # temp block created after 2 reads (old) vs after every slot filled once (0), A/B/A/B, same box
      CA=alluxio.worker.data.server.native.ufs.create.after.reads
      for rep in 1 2; do
        for ca in 0 2; do
          for par in 1 4; do
            run cold_ca${ca}_p${par}_$rep 300 python tools/remote_device_read_bench.py --uds --cold --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --worker-prop $CA=$ca --out "$OUT/r6_cold_create_ab.jsonl"
          done
        done
      done
      for par in 1 4; do
        run cached_p$par 300 python tools/remote_device_read_bench.py --uds --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/r6_cold_create_ab.jsonl"
      done
      ;;
    r6cold4)
      # four cold streams with the reader's finer timing (device setup, slot alloc, first read), and the cached pair
      for par in 4 1; do
        run cold4_p$par 300 python tools/remote_device_read_bench.py --uds --cold --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/r6_cold_timing.jsonl"
      done
      run cached4_p4 300 python tools/remote_device_read_bench.py --uds --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=4 --out "$OUT/r6_cold_timing.jsonl"
      ;;
    r6ra)
      # next-block read-ahead A/B/A/B (cold, one stream and four) plus the cached rows, same box
      RA=alluxio.worker.data.server.native.ufs.readahead.enabled
      for rep in 1 2; do
        for ra in true false; do
          for par in 1 4; do
            run cold_ra${ra}_p${par}_$rep 300 python tools/remote_device_read_bench.py --uds --cold --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --worker-prop $RA=$ra --out "$OUT/r6_cold_readahead_ab.jsonl"
          done
        done
      done
      for par in 1 4; do
        run cached_p$par 300 python tools/remote_device_read_bench.py --uds --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/r6_cold_readahead_ab.jsonl"
      done
      ;;
    r6cold)
      # cold read-through vs cached, one ReadBlock stream at a time and four, host destination (UDS default)
      for par in 1 4; do
        run cold_p$par 300 python tools/remote_device_read_bench.py --uds --cold --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/r6_cold_vs_cached.jsonl"
        run cached_p$par 300 python tools/remote_device_read_bench.py --uds --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/r6_cold_vs_cached.jsonl"
      done
      ;;
    r6tests)
      run pytest_gpu_r6 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
      ;;
    validate)
      run pytest_gpu_validate 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
      run smoke_validate 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()"
      run bench_validate_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5
      ;;
    final)
      run pytest_gpu_final 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
      run smoke_final 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()"
      run bench_final 400 python bench.py
      run wb_host_sweep_final 900 python tools/worker_bench_host.py --threads 16,64,256 --transports grpc,ipc --duration 6s --warmup 2s --out "$OUT/r5_worker_bench_host_sweep.jsonl"
      ;;
    roof)
      run copy_roof 300 python tools/copy_roof.py --gib 4 --out "$OUT/r5_copy_roof.json"
      ;;
    master16)
      run master_p16 300 python tools/master_bench_mp.py --ops CreateFile,DeleteFile --procs 16 --threads 4 --duration 5s --client-prop alluxio.user.network.native.rpc.enabled=false --out "$OUT/master_bench_p16_r5b.json"
      ;;
    numa)
      run wb_host_procs4_roof 600 python tools/worker_bench_host.py --threads 16,64 --transports ipc --duration 6s --warmup 2s --client-procs 4 --d2h-roof --out "$OUT/worker_bench_host_procs_roof.jsonl"
      run wb_host_procs1_roof 400 python tools/worker_bench_host.py --threads 16 --transports ipc,grpc --duration 6s --warmup 2s --client-procs 1 --d2h-roof --out "$OUT/worker_bench_host_procs_roof.jsonl"
      ;;
    numa2)
      run numa_bound_1m 600 python tools/worker_bench_host.py --threads 64 --transports ipc --duration 6s --warmup 2s --client-procs 4 --d2h-roof --bind-gpu-node --out "$OUT/r5_host_read_numa_bound.jsonl"
      run numa_bound_4m 600 python tools/worker_bench_host.py --threads 64 --transports ipc --duration 6s --warmup 2s --client-procs 4 --d2h-roof --bind-gpu-node --reader-buffer 4MB --out "$OUT/r5_host_read_numa_bound.jsonl"
      run numa_free_4m 600 python tools/worker_bench_host.py --threads 64 --transports ipc --duration 6s --warmup 2s --client-procs 4 --d2h-roof --reader-buffer 4MB --out "$OUT/r5_host_read_numa_bound.jsonl"
      ;;
    hostprocs2)
      ALLUXIO_READER_STREAMS=1 run wb_host_procs8_s1 600 python tools/worker_bench_host.py --threads 256 --transports ipc --duration 6s --warmup 2s --client-procs 8 --out "$OUT/worker_bench_host_procs_streams.jsonl"
      ALLUXIO_READER_STREAMS=8 run wb_host_procs8_s8 600 python tools/worker_bench_host.py --threads 256 --transports ipc --duration 6s --warmup 2s --client-procs 8 --out "$OUT/worker_bench_host_procs_streams.jsonl"
      ALLUXIO_READER_STREAMS=1 run wb_host_procs4_s1 600 python tools/worker_bench_host.py --threads 16,64,256 --transports ipc --duration 6s --warmup 2s --client-procs 4 --out "$OUT/worker_bench_host_procs_streams.jsonl"
      ;;
    hostprocs3)
      HSA_ENABLE_SDMA=0 run wb_host_procs4_nosdma 600 python tools/worker_bench_host.py --threads 16,64,256 --transports ipc --duration 6s --warmup 2s --client-procs 4 --out "$OUT/worker_bench_host_procs_sdma.jsonl"
      run wb_host_procs4_sdma 600 python tools/worker_bench_host.py --threads 16,64,256 --transports ipc --duration 6s --warmup 2s --client-procs 4 --out "$OUT/worker_bench_host_procs_sdma.jsonl"
      ;;
    remotedev) run remote_device_read 600 python tools/remote_device_read_bench.py --file-size 1g --out "$OUT/remote_device_read.jsonl" ;;
    remotehost)
      for par in 1 4; do
        run remote_host_read_p$par 300 python tools/remote_device_read_bench.py --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/remote_host_read.jsonl"
      done
      ;;
    remotecold)
      run remote_cold_host 300 python tools/remote_device_read_bench.py --cold --dest host --file-size 2g --read-size 2g --native-only --out "$OUT/remote_cold_read.jsonl"
      run remote_cold_host_p1 300 python tools/remote_device_read_bench.py --cold --dest host --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=1 --out "$OUT/remote_cold_read.jsonl"
      run remote_cold_dev 300 python tools/remote_device_read_bench.py --cold --file-size 2g --read-size 2g --native-only --out "$OUT/remote_cold_read.jsonl"
      ;;
    s3write)
      run s3_write_8g 600 python tools/s3_write_bench.py --size 8g --paths ufs,through --out "$OUT/s3_write.jsonl"
      run s3_write_8g_spool 400 python tools/s3_write_bench.py --size 8g --paths ufs --spool --out "$OUT/s3_write.jsonl"
      run s3_write_8g_p32 400 python tools/s3_write_bench.py --size 8g --paths ufs,through --part 32MB --out "$OUT/s3_write.jsonl"
      run s3_write_8g_p16 400 python tools/s3_write_bench.py --size 8g --paths ufs,through --part 16MB --out "$OUT/s3_write.jsonl"
      ;;
    arena)
      run pytest_arena 400 python -u -m pytest tests/test_ipc_gpu.py -k "arena or read_from_other" -v --timeout 200 --timeout-method thread
      ;;
    remoteprof)
      run rocprof_remote_host 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof_remote_host" -o rh --output-format csv -- python3 tools/remote_device_read_bench.py --dest host --file-size 1g --read-size 1g --native-only --client-prop alluxio.user.device.read.parallelism=1
      ;;
    bigwrite)
      for par in 1 4; do
        run big_write_p$par 170 python tools/worker_write_bench.py --threads 1 --files 2 --file-size 1g --write-size 1g --transports grpc,ipc --client-prop alluxio.user.device.read.parallelism=$par --worker-prop alluxio.worker.tieredstore.level0.dirs.quota=${BIGW_QUOTA:-8GB} --out "$OUT/worker_big_write.jsonl"
      done
      ;;
    remotedevab)
      for par in 2 4 8 16; do
        run remote_device_read_p$par 300 python tools/remote_device_read_bench.py --file-size 2g --read-size 2g --native-only --client-prop alluxio.user.device.read.parallelism=$par --out "$OUT/remote_device_read_par.jsonl"
      done
      ;;
    remotedevpar)
      run ipc_gpu_tests 300 python -u -m pytest tests/test_ipc_gpu.py -x -v --timeout 120 --timeout-method thread
      run remote_device_read_256m 600 python tools/remote_device_read_bench.py --file-size 1g --read-size 256m --out "$OUT/remote_device_read.jsonl"
      run remote_device_read_1g 600 python tools/remote_device_read_bench.py --file-size 1g --read-size 1g --out "$OUT/remote_device_read.jsonl"
      ;;
    hostsweep)
      for rb in 256KB 512KB 1MB; do
        for pf in false true; do
          run wb_sweep_${rb}_$pf 600 python tools/worker_bench_host.py --threads 16,256 --transports grpc,ipc --duration 6s --warmup 2s --reader-buffer $rb --client-prop alluxio.user.native.reader.prefetch.enabled=$pf --out "$OUT/worker_bench_host_sweep.jsonl"
        done
      done
      ;;
    replicate)
      run replicate_bench 600 python tools/replicate_bench.py --ranks 2 --blocks 16 --block-size 64m --batches 64m,256m,1g --out "$OUT/replicate_bench.jsonl"
      run replicate_bench3 600 python tools/replicate_bench.py --ranks 3 --blocks 8 --block-size 64m --batches 64m,512m --methods ring --out "$OUT/replicate_bench.jsonl"
      run rocprof_replicate 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_replicate" -o repl --output-format csv -- python3 tools/replicate_bench.py --ranks 3 --blocks 8 --block-size 64m --batches 64m --methods ring --reps 1
      ;;
    hostread)
      run worker_bench_host 900 python tools/worker_bench_host.py --threads 16,64,256 --duration 8s --warmup 2s --out "$OUT/worker_bench_host.jsonl"
      ;;
    masterufs)
      # CPU-only: CreateDir THROUGH against a root UFS whose every call sleeps 5 ms
      for t in 1 8 32; do
        p=$(( t < 4 ? 1 : 4 )); th=$(( t / p ))
        run master_ufs_sleep_t$t 300 python tools/master_bench_mp.py --ops CreateDir --procs $p --threads $th --duration 5s --write-type THROUGH --ufs-sleep-ms 5 --out "$OUT/master_ufs_sleep_t$t.json"
      done
      ;;
    largetune)
      run ring_tune_large 500 python tools/ring_tune.py --file-size 16g --stagger --depths 256 --variants 0,1,2,3 --caps 4096,8192,16384 --rounds 3 --steps 32 --out "$OUT/ring_tune_large.json"
      ;;
    kprof) run rocprof_kbench 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_k" -o kb --output-format csv -- python3 tools/kernel_bench.py --out "$OUT/kb_prof.json" ;;
    evictb) run evict_bench 300 python tools/evict_bench.py --counts 10000,150000 --out "$OUT/evict_bench.jsonl" ;;
    evict)
      run pytest_evict 300 python -u -m pytest tests/test_evict_alloc_gpu.py tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread
      run evict_bench 300 python tools/evict_bench.py --counts 10000,150000 --out "$OUT/evict_bench.jsonl"
      run evict_bench_lrfu 300 python tools/evict_bench.py --counts 150000 --policy 1 --out "$OUT/evict_bench.jsonl"
      run rocprof_evict 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_evict" -o ev --output-format csv -- python3 tools/evict_bench.py --counts 150000 --iters 10
      ;;
    ingest)
      run ufs_ingest_local 600 python tools/ufs_ingest_bench.py --ufs local --hbm 2g --dram 6g --factor 2 --file-size 256m --out "$OUT/ufs_ingest.jsonl"
      run ufs_ingest_s3 600 python tools/ufs_ingest_bench.py --ufs s3 --hbm 256m --dram 1g --factor 2 --file-size 64m --out "$OUT/ufs_ingest.jsonl"
      ;;
    kbench) run kernel_bench 300 python tools/kernel_bench.py --out "$OUT/kernel_bench.json" ;;
    pcsweep) run page_cache_sweep 400 python tools/page_cache_bench.py --variants both --passes 2 --page-sizes 4k,8k,16k,32k,64k,256k --out "$OUT/page_cache_sweep.jsonl" ;;
    pcwave) run page_cache_wave 400 python tools/page_cache_bench.py --variants both --passes 2 --wave-variants 0,1,2,3 --page-sizes 4k,16k --iters 30 --out "$OUT/page_cache_wave.jsonl" ;;
    pc)
      run page_cache_bench 300 python tools/page_cache_bench.py --out "$OUT/page_cache_bench.jsonl"
      run rocprof_pc 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_pc" -o pc --output-format csv -- python3 tools/page_cache_bench.py --page-sizes 4k,64k,2m --iters 5
      ;;
    ringtune) run ring_tune 600 python tools/ring_tune.py --out "$OUT/ring_tune.json" $RINGTUNE_ARGS ;;
    tune) run copy_tune 600 python tools/copy_tune.py --out "$OUT/copy_tune.json" ;;
  esac
done
echo "=== done" | tee -a "$OUT/round.log"

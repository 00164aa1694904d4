#!/bin/bash
# One gpurun session: GPU parity tests, smoke, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; the script stops at the first crash
# (abort/segfault/timeout) and never retries a GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# any failing step ends the session: a Python exception may hide a GPU memory
# fault (hipErrorIllegalAddress), after which nothing more may run on the GPU
crashed() { [ "$1" != 0 ]; }
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if crashed $rc; then echo "FAILED: $name (rc=$rc); stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"pytest smoke bench prof"}
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    soak)   RSGPU_SOAK_SECONDS=${SOAK_SECONDS:-240} RSGPU_SOAK_SEED=${SOAK_SEED:-20261016} run soak $(( ${SOAK_SECONDS:-240} + 240 )) python -u -m pytest tests/test_gpu_soak.py -m gpu -x -s --timeout $(( ${SOAK_SECONDS:-240} + 200 )) --timeout-method thread ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py ;;
    bench_all)
            run bench_enc 300 python bench.py --workload enc --no-cpu
            run bench_dec4 300 python bench.py --workload dec4 --no-cpu
            run bench_mixed 300 python bench.py --workload encdec_mixed --no-cpu ;;
    allwl)  # every device-resident workload once (value, frac, per-op kernel ms, decode check)
            for wl in ${ALL_WLS:-enc dec4 encdec_mixed encdec_upstream small small_mixed small1k small1k_sm small1k_sm_mixed_a128 wide}; do
              run wl_$wl 300 python bench.py --workload $wl --no-cpu --no-pmc
            done
            run wl_trace 600 python bench.py --workload trace --steps 3 --warmup 1 --no-cpu
            python - > gpurun_out/all_workloads.txt <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/wl_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); r = d.get("roofline") or {}
            print(f[len("gpurun_out/wl_"):-4], d["value"], r.get("frac"), r.get("kernel_ms_alone"), d.get("decode_check"))
PY
            cat gpurun_out/all_workloads.txt ;;
    shardmajor) run pytest_shardmajor 600 python -u -m pytest tests/test_gpu_shardmajor.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    masks)  run pytest_masks 600 python -u -m pytest tests/test_gpu_masks.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    mixed)  for wl in small_mixed encdec_mixed small; do
              run bench_$wl 300 python bench.py --workload $wl --no-cpu
            done ;;
    prof_mixed) for wl in small_mixed encdec_mixed; do
              run prof_$wl 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$wl -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --workload $wl
            done ;;
    small1k) for wl in ${SMALL_WLS:-small1k small1k_p4 small1k_p1}; do
              run bench_$wl 300 python bench.py --workload $wl --no-cpu
              run prof_$wl 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$wl -o run --output-format csv -- python3 bench.py --no-cpu --steps 10 --workload $wl
              run pmc_fetch_$wl 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$wl -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --workload $wl
              run pmc_write_$wl 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$wl -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --workload $wl
            done ;;
    worker) run pytest_worker 600 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_worker_concurrency.py -m gpu -x -v -s --timeout 150 --timeout-method thread ;;
    lat_sizes) for b in ${LAT_SIZES:-1024 4096 16384 40960}; do
              LAT_WORKER=16 LAT_BYTES=$b run lat_worker_vram_$b 120 ./tools/lat_bench 200 1
              RSGPU_WORKER_TRANSPORT=host LAT_WORKER=16 LAT_BYTES=$b run lat_worker_host_$b 120 ./tools/lat_bench 200 1
            done ;;
    lat_alloc) # host image allocation kinds, interleaved: Mapped|Coherent (default since r05) vs hipHostMallocDefault
            for rep in 1 2; do
              LAT_BYTES=1048576 run lat_1m_coherent_$rep 120 ./tools/lat_bench 300 1
              RSGPU_HOST_ALLOC=default LAT_BYTES=1048576 run lat_1m_default_$rep 120 ./tools/lat_bench 300 1
              LAT_WORKER=16 LAT_BYTES=1024 run lat_1k_coherent_$rep 120 ./tools/lat_bench 300 1
              RSGPU_HOST_ALLOC=default LAT_WORKER=16 LAT_BYTES=1024 run lat_1k_default_$rep 120 ./tools/lat_bench 300 1
            done ;;
    trace_alloc) run trace_coherent 900 python bench.py --workload trace --steps 3 --warmup 1
            RSGPU_HOST_ALLOC=default run trace_default 900 python bench.py --workload trace --steps 3 --warmup 1 --no-cpu ;;
    dma_split) # the copy engine beside the zero-copy pass (RSGPU_DMA_SPLIT=<percent of columns>), 1 MiB per object
            RSGPU_DMA_SPLIT=40 run pytest_dma_split 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_c_abi.py -m gpu -x -q --timeout 150 --timeout-method thread
            for rep in 1 2; do
              for pct in ${DMA_PCTS:-0 20 30 40 50}; do
                RSGPU_DMA_SPLIT=$pct LAT_BYTES=${DMA_BYTES:-1048576} run lat_dma_${pct}_$rep 120 ./tools/lat_bench 300
              done
            done ;;
    wslice) # large pinned objects as column slices over many mailboxes (worker) vs the stream path
            for b in ${WS_BYTES:-262144 1048576 4194304}; do
              LAT_BYTES=$b run ws_stream_$b 120 ./tools/lat_bench 300
              for ns in ${WS_SLOTS:-16 64}; do
                RSGPU_WORKER_SPLIT_MAX=4194304 LAT_WORKER=$ns LAT_MAX_SHARD=4096 LAT_BYTES=$b run ws_w${ns}_$b 120 ./tools/lat_bench 300
              done
            done ;;
    pylat)  # per-object latency from Python: C marshalling (default) vs ctypes, 1 KiB via the worker and 1 MiB
            for rep in 1 2; do
              run pylat_1k_c_$rep 300 python bench.py --workload latency --steps 300 --warmup 20 --obj-bytes 1024 --worker 16
              INFINICACHE_PY_MARSHAL=ctypes run pylat_1k_ctypes_$rep 300 python bench.py --workload latency --steps 300 --warmup 20 --obj-bytes 1024 --worker 16
              run pylat_1m_c_$rep 300 python bench.py --workload latency --steps 200 --warmup 10
              INFINICACHE_PY_MARSHAL=ctypes run pylat_1m_ctypes_$rep 300 python bench.py --workload latency --steps 200 --warmup 10
            done ;;
    trace_group) # config 5 with adjacent small objects sharing one H2D (RSGPU_PIPE_GROUP bytes), interleaved
            for rep in 1 2; do
              for g in ${GROUPS_B:-0 16777216 67108864}; do
                RSGPU_PIPE_GROUP=$g run trace_group_${g}_$rep 600 python bench.py --workload trace --steps 3 --warmup 1 --no-cpu
              done
            done ;;
    trace_marshal) # config 5 with the batch marshalling in C (default) vs ctypes, interleaved
            for rep in 1 2; do
              run trace_c_$rep 600 python bench.py --workload trace --steps 3 --warmup 1 --no-cpu
              INFINICACHE_PY_MARSHAL=ctypes run trace_ctypes_$rep 600 python bench.py --workload trace --steps 3 --warmup 1 --no-cpu
            done ;;
    tests)  # a chosen set of GPU test files (TESTS), one pytest process
            run pytest_sel 900 python -u -m pytest ${TESTS} -m gpu -x -v -s --timeout 150 --timeout-method thread ;;
    rccl1)  # BASELINE config 4's collectives over RCCL with one rank (the -m gpu test writes the line)
            BENCH_RCCL_JSON=gpurun_out/r05_bench_rccl_1rank.json run pytest_rccl1 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v -s --timeout 240 --timeout-method thread ;;
    avail)  run avail 120 rocprofv3 --list-avail ;;
    dec4get) # BASELINE config 3 as Client.decode runs it: fused and unfused Get lines + kernel stats
            for wl in dec4_get dec4_upstream; do
              run bench_$wl 600 python bench.py --workload $wl
              run prof_$wl 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$wl -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 20 --workload $wl
            done ;;
    sq)     # issue / wait / clock counters per kernel (one pass per workload; 8 SQ + 2 GRBM slots)
            for wl in ${SQ_WLS:-dec4_get encdec}; do
              run sq_$wl 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/sq_$wl -o run --output-format csv -- python3 bench.py --no-cpu --no-pmc --steps 5 --warmup 50 --workload $wl
            done ;;
    tri)    # input-triples kernel vs single inputs (kbench, cold), then the library default through the bench
            for sh in ${TRI_SHAPES:-decx10_4 decx10_4@1 enc10_4 ver10_4}; do
              KB_SET=tri KB_ROT=${TRI_ROT:-3} run kbench_tri_${sh/@/_at} 300 ./tools/kbench $sh ${TRI_ROUNDS:-10}
            done ;;
    wsweep) # occupancy cap (RSGPU_MIXED_W workgroups per CU) of the fused RS(10+4) Get, 4 MiB, cold, two passes
            for rep in 1 2; do
              for w in ${WS:-3 4 5 6 8}; do
                RSGPU_MIXED_W=$w KB_LOST=0,5 run wsweep_w${w}_$rep 120 ./tools/kbench lib:dec10_4@4 10
              done
            done
            grep -h "^lib" gpurun_out/wsweep_w*.log > gpurun_out/wsweep_summary.txt || true ;;
    rehearse8) # the N = 8 scaling harness on the one-GPU box (8 gloo ranks sharing cuda:0), full batch
            BENCH_DIST_BACKEND=gloo BENCH_SHARE_GPU=1 run rehearse8 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 8 ;;
    pcie)   run pcie 300 ./tools/pcie_bench ;;
    example) run example 300 python examples/client_example.py --loopback --addr 127.0.0.1:16378 ;;
    rehearse2) BENCH_DIST_BACKEND=gloo BENCH_SHARE_GPU=1 run rehearse2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --no-cpu --copies 2 ;;
    trace_dev) run bench_trace_dev 900 python bench.py --workload trace --steps 3 --warmup 1 --devices ${TRACE_DEVICES:-1} ;;
    torchrun1) run torchrun1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --no-cpu ;;
    latency) run bench_latency 600 python bench.py --workload latency --steps 200 --warmup 10 ;;
    trace)  run bench_trace 900 python bench.py --workload trace --steps 3 --warmup 1 ;;
    kbench) for sh in ${KSHAPES:-enc10_2 dec10_2 enc10_4 rdata10_4 decx10_4 ver10_2 ver10_4}; do
              run kbench_$sh 300 ./tools/kbench $sh 15
            done ;;
    lat)    run lat_bench 300 ./tools/lat_bench 300 2 ;;
    kgen)   for sh in ${KGEN:-enc20_4 dec20_4 enc20_8 enc32_8 dec32_8 enc64_16}; do
              run kgen_$sh 300 ./tools/kbench lib:$sh 15
            done ;;
    cpuinfo) (nproc; grep -m1 "model name" /proc/cpuinfo; grep -o -w -e avx512bw -e avx2 -e gfni /proc/cpuinfo | sort | uniq -c; cat /sys/fs/cgroup/cpu.max) > gpurun_out/cpuinfo.log 2>&1 ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 ;;
    pmc_all) for wl in enc dec4; do
              run prof_$wl 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$wl -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --workload $wl
              run pmc_fetch_$wl 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$wl -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --workload $wl
              run pmc_write_$wl 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$wl -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --workload $wl
            done ;;
    pmc)    run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu --steps 5
            run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 ;;
  esac
done
echo "ALL DONE"

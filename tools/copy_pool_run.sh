# host copy pool: parity suites, then pageable per-object latency with and without the pool
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_c_abi.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/parity.log 2>&1
rc=$?; tail -3 gpurun_out/parity.log; [ $rc = 0 ] || exit $rc
for b in ${LAT_SIZES:-1048576 4194304 16777216}; do
  for t in ${COPY_THREADS:-0 8}; do
    RSGPU_COPY_THREADS=$t LAT_BYTES=$b timeout -k 10 120 ./tools/lat_bench 100 > gpurun_out/lat_copy${t}_$b.txt 2>&1 || exit 3
  done
done
for f in gpurun_out/lat_copy*.txt; do echo "== $f"; grep pageable $f; done

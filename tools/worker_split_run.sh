cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
RSGPU_WORKER_SPLIT_MAX= timeout -k 10 400 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_worker_concurrency.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/worker.log 2>&1
rc=$?; tail -5 gpurun_out/worker.log; [ $rc = 0 ] || exit $rc
for b in ${LAT_SIZES:-65536 262144 1048576 4194304}; do
  LAT_BYTES=$b LAT_WORKER=16 LAT_MAX_SHARD=4096 timeout -k 10 120 ./tools/lat_bench 300 1 > gpurun_out/latw_$b.txt 2>&1 || exit 3
  LAT_BYTES=$b timeout -k 10 120 ./tools/lat_bench 300 1 > gpurun_out/lats_$b.txt 2>&1 || exit 4
done
tail -n +1 gpurun_out/lat*.txt

cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_masks.py tests/test_gpu_shardmajor.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mask or multi or shardmajor or mixed" > gpurun_out/masks.log 2>&1
rc=$?; tail -3 gpurun_out/masks.log; [ $rc = 0 ] || exit $rc
for wl in encdec_mixed encdec_mixed small_mixed; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu --no-pmc 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$wl', d['value'], r['frac'], r['kernel_ms_alone'], d.get('decode_check'))" || exit 4
done

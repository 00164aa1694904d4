#!/bin/bash
# Long concurrent stress of every per-object route (tests/c_abi_stress.c) on
# the product library and under ASan/UBSan and TSan builds; one step at a
# time, each under its own limit, stopping at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/stress_long.txt
: > $out
for spec in "plain 16 120 11" "asan 8 60 12" "tsan 8 60 13"; do
  set -- $spec
  echo "== $1 threads=$2 seconds=$3 seed=$4" | tee -a $out
  timeout -k 10 $(( $3 + 600 )) python -u -c "
import sys; sys.path.insert(0, 'tests')
import test_sanitize as t
print(t._stress('$1', $2, $3, $4))" >> $out 2>&1 || { echo "FAILED: $1"; tail -20 $out; exit 1; }
  tail -2 $out
done
echo "ALL DONE"

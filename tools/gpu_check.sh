#!/bin/bash
# GPU validation pass: kernel numerics tests, smoke, short native bench.
# Stops at the first step that faults / aborts / times out (rc not in {0,1}).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:randomly > gpurun_out/kt.log 2>&1; rc=$?
echo "kernel tests rc=$rc"; tail -30 gpurun_out/kt.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
for b in ${BENCH_BATCHES:-16 64}; do
  timeout -k 10 400 python bench.py --batch $b --steps 10 --warmup 3 >> gpurun_out/native.jsonl 2>> gpurun_out/native.err; rc=$?
  echo "bench b=$b rc=$rc"; tail -1 gpurun_out/native.jsonl
  [ $rc -eq 0 ] || exit $rc
done

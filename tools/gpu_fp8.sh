#!/bin/bash
# fp8 conv path: numerics tests, then a bf16 vs fp8 bench pair.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fp8t.log 2>&1; rc=$?
echo "fp8 tests rc=$rc: $(tail -1 gpurun_out/fp8t.log)"; grep -E "FAILED|Error|assert" gpurun_out/fp8t.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for prec in ${PRECS:-fp8 bf16}; do
  timeout -k 10 400 python bench.py --batch ${B:-128} --steps 10 --warmup 3 --precision $prec >> gpurun_out/fp8bench.jsonl 2>> gpurun_out/fp8bench.err || exit $?
  tail -1 gpurun_out/fp8bench.jsonl | cut -c1-260
done
if [ -n "$PROF" ]; then
  B=64 BENCH_ARGS="--precision fp8" bash tools/gpu_prof_native.sh || exit $?
  head -40 gpurun_out/native_prof_b64/summary.txt
fi

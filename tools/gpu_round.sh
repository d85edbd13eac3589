#!/bin/bash
# Full GPU pass: numerics tests, smoke, bench at B=64/128, per-layer conv bench (v1 vs auto),
# rocprof kernel trace of the bench.  Stops at the first fault/abort/timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/kt.log 2>&1; rc=$?
echo "gpu tests rc=$rc: $(tail -1 gpurun_out/kt.log)"; grep FAILED gpurun_out/kt.log | head
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
for b in ${BENCH_BATCHES:-64 128}; do
  timeout -k 10 400 python bench.py --batch $b --steps 10 --warmup 3 >> gpurun_out/native.jsonl 2>> gpurun_out/native.err || exit $?
  tail -1 gpurun_out/native.jsonl | cut -c1-200
done
if [ -n "$CONV_BENCH" ]; then
  timeout -k 10 600 python tools/conv_bench.py --batch 64 --iters 10 --variants $CONV_BENCH > gpurun_out/convbench.jsonl 2>&1 || exit $?
fi
B=${PROF_B:-64} bash tools/gpu_prof_native.sh || exit $?
head -25 gpurun_out/native_prof_b${PROF_B:-64}/summary.txt

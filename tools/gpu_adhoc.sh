#!/bin/bash
# full GPU test suite + bench + kernel profile (halo kernels)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && rm -f gpurun_out/bounds.jsonl
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/kt.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/kt.log)"; grep -E "^FAILED|^E  " gpurun_out/kt.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_b256.jsonl 2> gpurun_out/bench.err || exit $?
cut -c1-260 gpurun_out/bench_b256.jsonl
B=256 bash tools/gpu_prof_native.sh || exit $?
head -45 gpurun_out/native_prof_b256/summary.txt

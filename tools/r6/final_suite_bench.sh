#!/bin/bash
# final build: the GPU suite, then the bench set (tools/r6/final_bench.sh)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_suite.log 2>&1; rc=$?
grep -E "passed|failed" $O/gpu_suite.log | tail -2
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r6final} bash tools/r6/final_bench.sh

#!/bin/bash
# the wgrad side-stream graph test crashed (segfault in replay): pairing off vs on, isolated
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5y
mkdir -p $O
P2P_GRAD_PAIR=0 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_wgrad_stream_gpu.py > $O/pair0.log 2>&1
rc=$?
echo "pair off: rc $rc $(grep -E 'passed|failed' $O/pair0.log | tail -1)"
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_wgrad_stream_gpu.py > $O/pair1.log 2>&1
echo "pair on: rc $? $(grep -E 'passed|failed|Segmentation' $O/pair1.log | tail -2)"
exit 0

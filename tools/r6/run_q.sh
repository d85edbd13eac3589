#!/bin/bash
# fp8 routing A/B at B=2048: Cout 65-128 input gradients bf16 (default) vs fp8; s2t fp8 dgrad
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp8_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6t1 ROUNDS=2 BARGS="--precision fp8" bash tools/r6/ab_env.sh "X=1" "P2P_FP8_DGRAD_BF16=0" "P2P_S2T_F8=3" || exit $?
echo done

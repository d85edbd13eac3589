#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_determinism_gpu.py tests/test_fp8_gpu.py -k "determin or wgrad or step" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6j1 ROUNDS=2 BARGS="--precision fp8" bash tools/r6/ab_env.sh "P2P_WGRAD_XCD=0" "P2P_WGRAD_XCD=1" || exit $?
TAG=r6j2 ROUNDS=2 BARGS="--family ref --batch 64" bash tools/r6/ab_env.sh "P2P_WGRAD_XCD=0" "P2P_WGRAD_XCD=1" || exit $?
TAG=r6j3 ROUNDS=1 bash tools/r6/ab_env.sh "P2P_WGRAD_XCD=0" "P2P_WGRAD_XCD=1" || exit $?

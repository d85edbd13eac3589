#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests/ -m gpu > $O/suite.log 2>&1; rc=$?
tail -3 $O/suite.log; grep -E "FAILED|ERROR" $O/suite.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TAG=r6j1 ROUNDS=2 BARGS="--precision fp8" bash tools/r6/ab_env.sh "P2P_WGRAD_XCD=0" "P2P_WGRAD_XCD=1" || exit $?
TAG=r6j2 ROUNDS=2 BARGS="--family ref --batch 64" bash tools/r6/ab_env.sh "P2P_WGRAD_XCD=0" "P2P_WGRAD_XCD=1" || exit $?

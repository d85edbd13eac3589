#!/bin/bash
# full GPU suite on the 512-row build; family R with the 512-row tile pinned vs 256
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s tests/ > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6r1 ROUNDS=2 BARGS="--family ref --batch 64" bash tools/r6/ab_env.sh "P2P_M32_BM=256" "P2P_M32_BM=512" || exit $?
echo done

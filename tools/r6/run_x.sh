#!/bin/bash
# 512 x 64 m32 tile: tests, A/B on family R (B = 64) and the headline
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6af; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_m32_gpu.py tests/test_family_r_gpu.py tests/test_pix2pix_step_gpu.py tests/test_determinism_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6af1 ROUNDS=2 BARGS="--family ref --batch 64" bash tools/r6/ab_env.sh "X=1" "P2P_M32_C64=0" || exit $?
TAG=r6af2 ROUNDS=1 bash tools/r6/ab_env.sh "X=1" "P2P_M32_C64=0" || exit $?
echo done

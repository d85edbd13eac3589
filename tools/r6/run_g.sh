#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fp8_gpu.py tests/test_conv_m32_gpu.py tests/test_graph_family_r_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
TAG=r6g1 ROUNDS=2 BARGS="--precision fp8" bash tools/r6/ab_env.sh "P2P_M32_F8=0" "P2P_M32_F8=1" "P2P_M32_F8=1 P2P_S2T_F8=3" || exit $?
TAG=r6g2 ROUNDS=2 bash tools/r6/ab_env.sh "P2P_WM32_R128=0" "P2P_WM32_R128=1" || exit $?
TAG=r6g3 ROUNDS=2 BARGS="--family ref --batch 64" bash tools/r6/ab_env.sh "P2P_WM32_R128=0" "P2P_WM32_R128=1" "P2P_LIB=alt/libp2p_nolaunder.so" || exit $?

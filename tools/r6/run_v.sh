#!/bin/bash
# EXT epilogue half-group pipelining: tests, A/B (bf16, fp8, family R) vs the serial groups build
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6ac; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_m32_gpu.py tests/test_nb_fuse_gpu.py tests/test_determinism_gpu.py tests/test_kernels_gpu.py -k "not wgrad_split" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6ac1 ROUNDS=2 bash tools/r6/ab_env.sh "X=1" "P2P_LIB=alt/libp2p_extserial.so" || exit $?
TAG=r6ac2 ROUNDS=1 BARGS="--precision fp8" bash tools/r6/ab_env.sh "X=1" "P2P_LIB=alt/libp2p_extserial.so" || exit $?
TAG=r6ac3 ROUNDS=1 BARGS="--family ref --batch 64" bash tools/r6/ab_env.sh "X=1" "P2P_LIB=alt/libp2p_extserial.so" || exit $?
echo done

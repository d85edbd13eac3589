#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_family_r_gpu.py -k "wgrad or determin or family" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6l1 ROUNDS=2 bash tools/r6/ab_env.sh "P2P_WGRAD_BLOCKS=512" "P2P_WGRAD_BLOCKS=256" || exit $?
TAG=r6l2 ROUNDS=1 BARGS="--precision fp8" bash tools/r6/ab_env.sh "P2P_WGRAD_BLOCKS=512" "P2P_WGRAD_BLOCKS=256" || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 5 --warmup 2 > $O/tr.log 2>&1 || exit $?
python tools/prof_summary.py $O/tr/run_kernel_trace.csv --steps 5 --top 60 --width 160 > $O/summary_b2048.txt
grep -E "wall|reduce|presum" $O/summary_b2048.txt | head

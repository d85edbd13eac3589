#!/bin/bash
# halo_pk8 gate loads hoisted before the K loop: tests, A/B vs the previous build, trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_image_path_gpu.py tests/test_pix2pix_step_gpu.py tests/test_determinism_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6ab1 ROUNDS=2 bash tools/r6/ab_env.sh "X=1" "P2P_LIB=alt/libp2p_oldunion.so" || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 5 --warmup 2 > $O/tr.log 2>&1 || { echo "trace failed"; tail -5 $O/tr.log; exit 1; }
python tools/prof_summary.py $O/tr/run_kernel_trace.csv --steps 5 --top 300 --width 160 > $O/summary_b2048.txt
grep -E "steady|halo_union|halo_pk8" $O/summary_b2048.txt
echo done

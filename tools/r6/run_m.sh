#!/bin/bash
# 512 x 128 m32 tile: tests, step A/B against the 256-row tile, B=2048 kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_m32_gpu.py -k 512 > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
TAG=r6n1 ROUNDS=2 bash tools/r6/ab_env.sh "P2P_M32_BM=256" "P2P_M32_BM=0" || exit $?
TAG=r6n2 ROUNDS=1 BARGS="--family ref --batch 64" bash tools/r6/ab_env.sh "P2P_M32_BM=256" "P2P_M32_BM=0" || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 5 --warmup 2 > $O/tr.log 2>&1 || { echo "trace failed"; tail -5 $O/tr.log; exit 1; }
python tools/prof_summary.py $O/tr/run_kernel_trace.csv --steps 5 --top 70 --width 160 > $O/summary_b2048.txt
head -24 $O/summary_b2048.txt
echo done

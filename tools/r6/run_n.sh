#!/bin/bash
# 512-row tile: per-row origins (default) vs derived rows (alt build) vs the 256-row tile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_m32_gpu.py -k 512 > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6o1 ROUNDS=2 bash tools/r6/ab_env.sh "X=1" "P2P_LIB=alt/libp2p_derive.so" "P2P_M32_BM=256" || exit $?
for v in main alt; do
  if [ $v = alt ]; then L="P2P_LIB=alt/libp2p_derive.so"; else L="X=1"; fi
  timeout -k 10 500 env $L rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- python bench.py --steps 5 --warmup 2 > $O/tr_$v.log 2>&1 || { echo "trace failed"; tail -5 $O/tr_$v.log; exit 1; }
  python tools/prof_summary.py $O/tr_$v/run_kernel_trace.csv --steps 5 --top 70 --width 160 > $O/summary_$v.txt
  grep -E "steady|m32_kernel<128" $O/summary_$v.txt
done
echo done

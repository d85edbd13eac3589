#!/bin/bash
# reduce with all slab loads in flight; family R split cap A/B; traces
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6u; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_family_r_gpu.py tests/test_wgrad_stream_gpu.py -k "wgrad or determin or family" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6u1 ROUNDS=2 BARGS="--family ref --batch 64" bash tools/r6/ab_env.sh "X=1" "P2P_WGRAD_MAXSPLITS=64" "P2P_WGRAD_MAXSPLITS=32" || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 5 --warmup 2 > $O/tr.log 2>&1 || { echo "trace failed"; tail -5 $O/tr.log; exit 1; }
python tools/prof_summary.py $O/tr/run_kernel_trace.csv --steps 5 --top 300 --width 160 > $O/summary_b2048.txt
grep -E "steady|reduce|presum" $O/summary_b2048.txt
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/trf -o run -- python bench.py --family ref --batch 64 --steps 5 --warmup 2 > $O/trf.log 2>&1 || { echo "trace failed"; tail -5 $O/trf.log; exit 1; }
python tools/prof_summary.py $O/trf/run_kernel_trace.csv --steps 5 --top 300 --width 160 > $O/summary_famr.txt
grep -E "steady|reduce|presum" $O/summary_famr.txt
echo done

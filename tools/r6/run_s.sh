#!/bin/bash
# logits-conv input gradient kernel: tests, A/B, family R
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_family_r_gpu.py tests/test_pix2pix_step_gpu.py tests/test_determinism_gpu.py tests/test_graph_gpu.py -k "logits_conv or family or step or unet" > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6z1 ROUNDS=2 bash tools/r6/ab_env.sh "X=1" "P2P_C1_DGRAD=0" || exit $?

timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 5 --warmup 2 > $O/tr.log 2>&1 || { echo "trace failed"; tail -5 $O/tr.log; exit 1; }
python tools/prof_summary.py $O/tr/run_kernel_trace.csv --steps 5 --top 300 --width 160 > $O/summary_b2048.txt
grep -E "steady|dgrad_c1|glds_kernel<128, 128, 2, 2, 1" $O/summary_b2048.txt
echo done

#!/bin/bash
# wgrad reduce with a pre-sum pass for many splits: numerics, the step, the B=1024 trace

set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_conv_m32_gpu.py tests/test_family_r_gpu.py tests/test_graph_gpu.py tests/test_ddp_gpu.py \
  tests/test_production_shapes_gpu.py tests/test_pix2pix_step_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -1 $O/bench.jsonl | cut -c1-150
done
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --batch 1024 --steps 5 --warmup 2 > $O/prof_log.txt 2>&1 || { tail $O/prof_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 90 --width 120 > $O/b1024_kernels.txt
head -3 $O/b1024_kernels.txt
grep "wgrad_reduce\|wgrad_presum" $O/b1024_kernels.txt
rm -rf $O/prof
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --family ref --batch 64 --steps 5 --warmup 2 > $O/famr_log.txt 2>&1 || { tail $O/famr_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 120 --width 120 > $O/famr_kernels.txt
head -3 $O/famr_kernels.txt
grep "wgrad_reduce\|wgrad_presum" $O/famr_kernels.txt
rm -rf $O/prof

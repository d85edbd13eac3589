#!/bin/bash
# batch-norm partials in the reflect / up2 fold dgrads (affine, shared-slope PReLU): nb tests,
# family-R tests, family-R trace + bench, headline bench (EXT epilogue regression check)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5an
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nb_fuse_gpu.py > $O/nb.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/nb.log | tail -30; exit 1; }
tail -1 $O/nb.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_family_r_gpu.py \
  tests/test_graph_family_r_gpu.py tests/test_cli_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --family ref --batch 64 --steps 5 --warmup 2 > $O/famr_log.txt 2>&1 || { tail $O/famr_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 120 --width 120 > $O/famr_kernels.txt
head -2 $O/famr_kernels.txt
grep "norm_bwd_partial\|fold_band\|sum_final\|loss_final" $O/famr_kernels.txt || true
timeout -k 10 300 python -u bench.py --family ref --batch 64 --steps 20 --warmup 5 > $O/famr.jsonl 2> $O/famr.err || { tail -20 $O/famr.err; exit 1; }
cut -c1-150 $O/famr.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -1 $O/bench.jsonl | cut -c1-120
done

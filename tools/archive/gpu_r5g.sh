#!/bin/bash
# B=1024 kernel trace of the step with both m32 tiles; innermost-gradient numerics over 5 seeds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --batch 1024 --steps 5 --warmup 2 > $O/prof_log.txt 2>&1 || { tail $O/prof_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 45 --width 150 > $O/b1024_kernels.txt
head -50 $O/b1024_kernels.txt
rm -rf $O/prof
timeout -k 10 900 python -u tools/diag_inner_grad.py --B 64 --seeds 11,12,13,14,15 --kinds fp32,eager,native \
  > $O/diag_inner.txt 2>&1 || { tail -20 $O/diag_inner.txt; exit 1; }
tail -12 $O/diag_inner.txt

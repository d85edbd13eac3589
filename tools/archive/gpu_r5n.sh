#!/bin/bash
# per-dispatch listing of the B=1024 step (every kernel of the last step, in order)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --batch 1024 --steps 5 --warmup 2 > $O/prof_log.txt 2>&1 || { tail $O/prof_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 3 --width 100 --calls "" > $O/calls.txt
mv $O/prof/run_kernel_trace.csv $O/trace.csv
rm -rf $O/prof
wc -l $O/calls.txt

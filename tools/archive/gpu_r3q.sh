#!/bin/bash
# Round-3 pass q: fp8 step kernel trace at B = 1024 (where the fp8 step's time goes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3q
mkdir -p $O/trace
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --precision fp8 --steps 3 --warmup 2 > $O/trace/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/trace/run_kernel_trace.csv --steps 3 --top 60 --width 150 > $O/trace/summary.txt
head -50 $O/trace/summary.txt

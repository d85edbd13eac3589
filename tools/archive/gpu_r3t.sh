#!/bin/bash
# Round-3 pass t: fp8 and bf16 kernel traces at B = 256 (where the fp8 / bf16 ratio is judged).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3t
mkdir -p $O/f8 $O/bf
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/f8 -o run -- python bench.py --steps 3 --warmup 2 --batch 256 --precision fp8 > $O/f8/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/f8/run_kernel_trace.csv --steps 3 --top 70 --width 160 > $O/f8/summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/bf -o run -- python bench.py --steps 3 --warmup 2 --batch 256 > $O/bf/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/bf/run_kernel_trace.csv --steps 3 --top 70 --width 160 > $O/bf/summary.txt
head -40 $O/f8/summary.txt

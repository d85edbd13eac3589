#!/bin/bash
# Round-3 pass z: fp8 B = 256 kernel trace of the final build (fp8 halo kernel rows).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3z
mkdir -p $O/f8
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/f8 -o run -- python bench.py --steps 3 --warmup 2 --batch 256 --precision fp8 > $O/f8/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/f8/run_kernel_trace.csv --steps 3 --top 70 --width 160 > $O/f8/summary.txt
head -3 $O/f8/summary.txt
grep "s2t\|<128, 64, 2, 2, 1" $O/f8/summary.txt

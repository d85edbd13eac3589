#!/bin/bash
# Round-3 pass w: kernel trace of the captured headline step at B = 256 (aten-free check).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O/trace
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --steps 3 --warmup 2 --batch 256 > $O/trace/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/trace/run_kernel_trace.csv --steps 3 --top 90 --width 160 > $O/trace/summary.txt
head -3 $O/trace/summary.txt
echo "aten rows:"; grep -c "at::native" $O/trace/summary.txt || true
grep "at::native\|rocclr" $O/trace/summary.txt || true

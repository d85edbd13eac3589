#!/bin/bash
# rocprofv3 kernel trace of the native bench (steady-state summary via tools/prof_summary.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
B=${B:-64}
OUT=gpurun_out/native_prof_b$B
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
  python bench.py --batch $B --steps 5 --warmup 2 ${BENCH_ARGS:-} > $OUT/log.txt 2>&1 || exit $?
python tools/prof_summary.py $OUT/run_kernel_trace.csv --steps 5 --top 60 --width 160 > $OUT/summary.txt

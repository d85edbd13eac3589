#!/bin/bash
# kernel traces of the final build: headline (bf16, B=2048 captured) and fp8 (B=2048 captured)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5aw
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/bf -o run -- \
  python bench.py --steps 5 --warmup 2 > $O/bf_log.txt 2>&1 || { tail $O/bf_log.txt; exit 1; }
python tools/prof_summary.py $O/bf/run_kernel_trace.csv --steps 5 --top 90 --width 120 > $O/bf_kernels.txt
python tools/prof_summary.py $O/bf/run_kernel_trace.csv --steps 5 --streams > $O/bf_streams.txt
head -3 $O/bf_kernels.txt
rm -rf $O/bf
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/f8 -o run -- \
  python bench.py --steps 5 --warmup 2 --precision fp8 > $O/f8_log.txt 2>&1 || { tail $O/f8_log.txt; exit 1; }
python tools/prof_summary.py $O/f8/run_kernel_trace.csv --steps 5 --top 90 --width 120 > $O/f8_kernels.txt
head -3 $O/f8_kernels.txt
rm -rf $O/f8

#!/bin/bash
# per-stream busy of the B=1024 step; wgrad side stream on/off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --batch 1024 --steps 5 --warmup 2 > $O/prof_log.txt 2>&1 || { tail $O/prof_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 5 --width 110 --streams > $O/streams.txt
cat $O/streams.txt
head -1 $O/prof/run_kernel_trace.csv > $O/trace_header.txt
rm -rf $O/prof
for w in 0 1; do
  P2P_WGRAD_STREAM=$w timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  tail -1 $O/bench.jsonl | cut -c1-150
done

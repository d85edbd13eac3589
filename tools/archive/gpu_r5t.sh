#!/bin/bash
# family-R B=64 step: GPU-active vs idle (graph replay gaps); fp8 default-batch capture check
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --family ref --batch 64 --steps 5 --warmup 2 > $O/famr_log.txt 2>&1 || { tail $O/famr_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 3 --width 100 --streams > $O/famr_streams.txt
head -12 $O/famr_streams.txt
mv $O/prof/run_kernel_trace.csv $O/famr_trace.csv; rm -rf $O/prof
timeout -k 10 300 python -u tools/probes/aten_census.py --family ref --batch 8 > $O/aten_famr.txt 2>&1 || { tail -20 $O/aten_famr.txt; exit 1; }
tail -40 $O/aten_famr.txt
timeout -k 10 400 python -u bench.py --precision fp8 --steps 10 --warmup 3 > $O/fp8.jsonl 2> $O/fp8.err || { tail -5 $O/fp8.err; exit 1; }
cut -c1-200 $O/fp8.jsonl; grep -o '"hipgraph[^,]*\|"capture_error[^,]*\|"global_batch[^,]*' $O/fp8.jsonl
timeout -k 10 500 python -u bench.py --precision fp8 --batch 2048 --steps 10 --warmup 3 > $O/fp8_2048.jsonl 2> $O/fp8_2048.err || { tail -5 $O/fp8_2048.err; exit 1; }
cut -c1-200 $O/fp8_2048.jsonl; grep -o '"hipgraph[^,]*\|"capture_error[^,]*' $O/fp8_2048.jsonl

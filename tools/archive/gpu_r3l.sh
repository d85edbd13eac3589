#!/bin/bash
# Round-3 pass l: wgrad 256x256 tile per-layer A/B (census) and the B = 1024 kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O/trace
timeout -k 10 500 python tools/conv_census.py --family pix2pix --batch 256 --top 70 --wgrad_variants P2P_WGRAD_TILE=256 --json $O/census_w.json > $O/census_w.txt 2>&1 || exit $?
grep -i "wgrad" $O/census_w.txt | head -40
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --steps 3 --warmup 2 > $O/trace/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/trace/run_kernel_trace.csv --steps 3 --top 60 --width 160 > $O/trace/summary.txt
head -45 $O/trace/summary.txt

#!/bin/bash
# Round-4 pass a: baseline of the round-3 build on today's box -- headline (B=1024) and B=256
# bench lines, a kernel trace of the captured B=1024 step, and the per-conv census (EXT tagged).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O/tr
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'], d.get('max_mem_gib'))"; }
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2>> $O/err.log || exit $?; echo "$tag $(j $O/$tag.json)"; cat $O/$tag.json >> $O/all.jsonl; }
run headline
run bf16_b256 --batch 256
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 3 --warmup 2 > $O/tr/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/tr/run_kernel_trace.csv --steps 3 --top 70 --width 160 > $O/trace_b1024.txt
head -3 $O/trace_b1024.txt
timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 1024 --reps 3 --top 80 > $O/census_b1024.txt 2>&1 || exit $?
head -40 $O/census_b1024.txt

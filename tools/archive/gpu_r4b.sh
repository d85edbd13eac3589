#!/bin/bash
# Round-4 pass b: the register-epilogue persistent s2t kernel (W = 32 and 64) -- oracle tests,
# then headline A/B (default / one tile per block / implicit GEMM) and the conv census.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_s2t_gpu.py tests/test_fp8_gpu.py tests/test_wgrad_stream_gpu.py tests/test_production_shapes_gpu.py -x -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
grep "errors vs fp32" $O/tests.log
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'], d.get('max_mem_gib'))"; }
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2>> $O/err.log || exit $?; echo "$tag $(j $O/$tag.json)"; cat $O/$tag.json >> $O/all.jsonl; }
run headline
P2P_S2T_GRID=0 run grid0
P2P_NO_S2T=1 run nos2t
run headline2
run bf16_b256 --batch 256
run fp8 --precision fp8
timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 1024 --reps 3 --top 30 > $O/census_b1024.txt 2>&1 || exit $?
head -25 $O/census_b1024.txt

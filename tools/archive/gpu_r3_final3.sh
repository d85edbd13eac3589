#!/bin/bash
# Round-3 final measurement set (after the fp8 halo kernel and the step-bookkeeping kernels): every GPU test, smoke, and the bench lines the README cites
# (headline default, fp8, inference, 512^2, reference family).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3final4
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'], d.get('max_mem_gib'))"; }
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2>> $O/err.log || exit $?; echo "$tag $(j $O/$tag.json)"; cat $O/$tag.json >> $O/all.jsonl; }
run headline
run fp8 --precision fp8
run infer --mode infer --batch 256
run s512_b128 --size 512 --batch 128 --steps 10 --warmup 3
run ref --family ref --batch 64 --steps 10 --warmup 3
run fp8_b256 --batch 256 --precision fp8
run bf16_b256 --batch 256

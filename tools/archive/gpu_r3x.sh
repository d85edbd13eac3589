#!/bin/bash
# Round-3 pass x: family-R loss composition / seeds / BN counters on HIP kernels -- every GPU
# test, the family-R aten census, family-R and headline benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
PYTHONPATH=. timeout -k 10 300 python tools/probes/aten_census.py --family ref --batch 4 > $O/aten_ref.txt 2>&1 || { tail -20 $O/aten_ref.txt; exit 1; }
awk '/^ *[0-9]+  /{s+=$1} END{print "family-R aten launches per step:", s+0}' $O/aten_ref.txt
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'])"; }
timeout -k 10 400 python bench.py --family ref --batch 64 --steps 10 --warmup 3 > $O/ref.json || exit 1; echo "ref $(j $O/ref.json)"
timeout -k 10 300 python bench.py --batch 256 > $O/bf.json || exit 1; echo "bf16 b256 $(j $O/bf.json)"

#!/bin/bash
# Round-3 pass v: step bookkeeping on HIP kernels (loss composition, seeds, Adam step counter,
# dropout seed, bias pad, D-batch halves): every GPU test, the aten census, B=256 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
PYTHONPATH=. timeout -k 10 300 python tools/probes/aten_census.py > $O/aten.txt 2>&1 || { tail -20 $O/aten.txt; exit 1; }
grep -v "^/opt\|UserWarn\|_warn_once\|ROCTracer\|^     at $" $O/aten.txt
timeout -k 10 300 python bench.py --batch 256 > $O/bf.json || exit 1
python -c "import json;d=json.load(open('$O/bf.json'));print('bf16 b256', d['value'], d['ms_per_step'])"

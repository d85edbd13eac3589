#!/bin/bash
# Round-3 pass k: full GPU test suite, then the headline at the new default batch (1024),
# the B = 256 A/B of the s2t kernel, fp8, and family R.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'], d.get('max_mem_gib'))"; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2>> $O/err.log || exit $?; echo "default $(j $O/bench_default.json)"
P2P_NO_S2T=1 timeout -k 10 300 python bench.py --batch 256 > $O/b256_nos2t.json 2>> $O/err.log || exit $?; echo "b256 no-s2t $(j $O/b256_nos2t.json)"
timeout -k 10 300 python bench.py --batch 256 > $O/b256.json 2>> $O/err.log || exit $?; echo "b256 $(j $O/b256.json)"
timeout -k 10 400 python bench.py --precision fp8 > $O/fp8_default.json 2>> $O/err.log || exit $?; echo "fp8 default $(j $O/fp8_default.json)"
timeout -k 10 300 python bench.py --family ref --batch 64 --steps 10 --warmup 3 > $O/ref.json 2>> $O/err.log || exit $?; echo "ref $(j $O/ref.json)"

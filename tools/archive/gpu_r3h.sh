#!/bin/bash
# Round-3 pass h: persistent software-pipelined s2t kernel -- tests, census, bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_s2t_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 256 --top 70 --json $O/census.json > $O/census.txt 2>&1 || exit $?
grep -E "m1 N(256|512) C(128|256) (64x64|32x32) -> (64|128) " $O/census.txt
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --batch 256 --steps 20 --warmup 5 > $O/ab_$tag.json 2>> $O/ab.err || exit $?
  echo "$tag $(python -c "import json;d=json.load(open('$O/ab_$tag.json'));print(d['value'], d['ms_per_step'])")"
}
run base P2P_NO_S2T=1
run s2t
timeout -k 10 300 python bench.py --family ref --batch 64 --steps 10 --warmup 3 > $O/ref.json 2>> $O/ab.err || exit $?
echo "ref $(python -c "import json;d=json.load(open('$O/ref.json'));print(d['value'], d['ms_per_step'])")"

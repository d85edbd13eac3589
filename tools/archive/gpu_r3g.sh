#!/bin/bash
# Round-3 pass g: class-shared halo kernel for stride-2 transposed convs (csrc/conv_s2t.hip) and
# weight gradients on a side stream: tests, then a same-box A/B of the headline step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_s2t_gpu.py tests/test_wgrad_stream_gpu.py tests/test_graph_gpu.py -x -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --batch 256 --steps 20 --warmup 5 > $O/ab_$tag.json 2>> $O/ab.err || exit $?
  echo "$tag $(python -c "import json;d=json.load(open('$O/ab_$tag.json'));print(d['value'], d['ms_per_step'])")"
}
run base1 P2P_NO_S2T=1 P2P_WGRAD_STREAM=0
run s2t1 P2P_WGRAD_STREAM=0
run ws1 P2P_NO_S2T=1
run both1
run base2 P2P_NO_S2T=1 P2P_WGRAD_STREAM=0
run both2
timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 256 --top 70 --json $O/census.json > $O/census.txt 2>&1 || exit $?
head -30 $O/census.txt

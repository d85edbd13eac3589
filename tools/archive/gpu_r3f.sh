#!/bin/bash
# Round-3 pass f: weight gradients on a side stream (ops/hip.py wgrad_overlap): bitwise tests,
# then a same-box A/B of the step with P2P_WGRAD_STREAM=0 / 1 at B = 256 and 512.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wgrad_stream_gpu.py tests/test_graph_gpu.py -x -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for r in 1 2; do
  for f in 0 1; do
    for b in 256 512; do
      P2P_WGRAD_STREAM=$f timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 > $O/ab_${f}_${b}_$r.json 2>> $O/ab.err || exit $?
      echo "ws=$f B=$b r=$r $(python -c "import json;d=json.load(open('$O/ab_${f}_${b}_$r.json'));print(d['value'], d['ms_per_step'])")"
    done
  done
done

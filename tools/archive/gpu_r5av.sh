#!/bin/bash
# same box: bf16 2048 captured vs eager; fp8 1024 vs 2048 captured (capture now fits: hand-off
# registries released + empty_cache before capture)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5av
mkdir -p $O
one() {  # tag args...
  local tag=$1; shift
  timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  echo "$tag $(python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['hipgraph'], d['max_mem_gib'])")"
}
for r in 1 2; do
  one bf_graph_$r
  one bf_eager_$r --no_graph
  one f8_1024_$r --precision fp8 --batch 1024
  one f8_2048_$r --precision fp8 --batch 2048
done

#!/bin/bash
# A/B: s2t halo kernel vs the m32 / glds tiles for the 4x4 s2 dgrads (P2P_NO_S2T=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ad
mkdir -p $O
for r in 1 2; do
  for v in s2t nos2t; do
    if [ $v = nos2t ]; then export P2P_NO_S2T=1; else unset P2P_NO_S2T; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    echo "$v $r $(python -c "import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['hipgraph'])")"
  done
done

#!/bin/bash
# routing A/B on the headline: default vs no s2t for gated / skip-gradient dgrads (m32 / glds
# EXT tiles instead) vs no 128-wide m32 tile (glds instead); 2 interleaved rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5aj
mkdir -p $O
for r in 1 2; do
  for v in base nos2text no128; do
    unset P2P_NO_S2T_EXT P2P_M32_NO128
    [ $v = nos2text ] && export P2P_NO_S2T_EXT=1
    [ $v = no128 ] && export P2P_M32_NO128=1
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    echo "$v $r $(python -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['hipgraph'])")"
  done
done

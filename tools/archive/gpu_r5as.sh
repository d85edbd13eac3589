#!/bin/bash
# after empty_cache before capture: headline 2048 vs 3072 (captured?), fp8 2048
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5as
mkdir -p $O
for r in 1 2; do
  for b in 2048 3072; do
    timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --batch $b > $O/b_${b}_$r.json 2> $O/b_${b}_$r.err || { tail -20 $O/b_${b}_$r.err; exit 1; }
    echo "b $b $r $(python -c "import json; d=json.loads(open('$O/b_${b}_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['hipgraph'], d['max_mem_gib'], str(d['config'].get('capture_error'))[:80])")"
  done
done

#!/bin/bash
# family-R batch: 256 (bench default) vs 512, captured, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ar
mkdir -p $O
for r in 1 2; do
  for b in 256 512; do
    timeout -k 10 500 python -u bench.py --family ref --steps 10 --warmup 3 --batch $b > $O/fr_${b}_$r.json 2> $O/fr_${b}_$r.err || { tail -20 $O/fr_${b}_$r.err; exit 1; }
    echo "famr $b $r $(python -c "import json; d=json.loads(open('$O/fr_${b}_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['hipgraph'], d['max_mem_gib'], str(d['config'].get('capture_error'))[:80])")"
  done
done

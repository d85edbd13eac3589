#!/bin/bash
# fp8 default batch: 1024 vs 1536 (captured?), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ap
mkdir -p $O
for r in 1 2; do
  for b in 1024 1536; do
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --precision fp8 --batch $b > $O/f8_${b}_$r.json 2> $O/f8_${b}_$r.err || { tail -20 $O/f8_${b}_$r.err; exit 1; }
    echo "fp8 $b $r $(python -c "import json; d=json.loads(open('$O/f8_${b}_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['hipgraph'], d['max_mem_gib'], str(d['config'].get('capture_error'))[:80])")"
  done
done

#!/bin/bash
# after empty_cache before capture: headline 2048 vs 3072 (captured?), fp8 2048
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5at
mkdir -p $O
for r in 1; do
  for b in 2048 3072; do
    timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --batch $b > $O/b_${b}_$r.json 2> $O/b_${b}_$r.err || { tail -20 $O/b_${b}_$r.err; exit 1; }
    echo "b $b $r $(python -c "import json; d=json.loads(open('$O/b_${b}_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['hipgraph'], d['max_mem_gib'], str(d['config'].get('capture_error'))[:80])")"
  done
done
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --precision fp8 --batch 2048 > $O/f8_2048.json 2> $O/f8_2048.err || { tail -20 $O/f8_2048.err; exit 1; }
echo "fp8 2048 $(python -c "import json; d=json.loads(open('$O/f8_2048.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['hipgraph'], d['max_mem_gib'], str(d['config'].get('capture_error'))[:80])")"

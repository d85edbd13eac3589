#!/bin/bash
# batch sweep of the headline at the HBM-sized end (captured): 2048 / 3072 / 4096
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6ad; mkdir -p $O
for r in 1 2; do
  for b in 2048 3072 4096; do
    timeout -k 10 500 python bench.py --batch $b --steps 10 --warmup 3 > $O/b${b}_r$r.out 2> $O/b${b}_r$r.err || { echo "batch $b failed"; tail -5 $O/b${b}_r$r.err; exit 1; }
    tail -1 $O/b${b}_r$r.out | python -c "import json,sys;d=json.loads(sys.stdin.read());print('b$b r$r', d['value'], d['ms_per_step'], d['config']['hipgraph'], d['config']['capture_error'], d.get('max_mem_gib'))"
  done
done
echo done

#!/bin/bash
# interleaved bench A/B of env settings: ROUNDS x settings, each line "tag value ms"
# usage: TAG=x ROUNDS=2 BARGS="--precision fp8" bash tools/r6/ab_env.sh "A=1" "A=0 B=2" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r6ab}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    timeout -k 10 400 env $e python bench.py --steps ${STEPS:-15} --warmup 4 ${BARGS:-} > $O/s${i}_r$r.out 2> $O/s${i}_r$r.err || { echo "setting $i ($e) failed"; tail -5 $O/s${i}_r$r.err; exit 1; }
    tail -1 $O/s${i}_r$r.out | python -c "import json,sys;d=json.loads(sys.stdin.read());print('[$e] r$r', d['value'], d['ms_per_step'], 'graph', d['config']['hipgraph'], d['config']['capture_error'])"
  done
done

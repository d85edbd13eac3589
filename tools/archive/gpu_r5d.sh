#!/bin/bash
# headline step: 32x32x16 tiles on / off / on (same box, bracketed)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
for v in 1 0 1; do
  P2P_M32=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  tail -1 $O/bench.jsonl | cut -c1-200
done

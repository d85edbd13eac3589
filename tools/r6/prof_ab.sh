#!/bin/bash
# kernel-trace A/B of two env settings (captured bench, B given), summaries via prof_summary.py
# usage: TAG=x B=1024 bash tools/r6/prof_ab.sh "ENV_A=.." "ENV_B=.."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6p}
mkdir -p $O
B=${B:-1024}
i=0
for e in "$@"; do
  i=$((i+1))
  timeout -k 10 400 env $e rocprofv3 --kernel-trace --output-format csv -d $O/p$i -o run -- \
    python bench.py --batch $B --steps 5 --warmup 2 ${BENCH_ARGS:-} > $O/p$i.log 2>&1 || { echo "run $i failed"; tail -5 $O/p$i.log; exit 1; }
  python tools/prof_summary.py $O/p$i/run_kernel_trace.csv --steps 5 --top 40 --width 150 > $O/summary_$i.txt
  echo "== $e"; head -22 $O/summary_$i.txt
done

#!/bin/bash
# Round-3 pass e: re-validate the restored tree (all GPU tests + smoke), then the 256^2
# batch sweep asked for by VERDICT r2 W9 (B = 256 / 512 / 1024, bf16, with max_mem_gib).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 120 python tools/probes/graph_concurrency_probe.py > $O/graph_conc.txt 2>&1 || exit $?
cat $O/graph_conc.txt
for b in 256 512 1024; do
  timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 >> $O/sweep.jsonl 2>> $O/sweep.err || exit $?
  tail -1 $O/sweep.jsonl | cut -c1-200
done

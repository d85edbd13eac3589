#!/bin/bash
# Round 6: production DP path (AVG at world 1, capture group), pairing test, force_comm A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_capture_group_gpu.py tests/test_graph_gpu.py tests/test_family_r_gpu.py tests/test_ddp_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/plain_r$r.json 2> $O/plain_r$r.err || exit $?
  timeout -k 10 300 python bench.py --steps 15 --warmup 4 --force_comm --comm_dtype bf16 > $O/fc_bf16_r$r.json 2> $O/fc_bf16_r$r.err || exit $?
  timeout -k 10 300 python bench.py --steps 15 --warmup 4 --force_comm > $O/fc_r$r.json 2> $O/fc_r$r.err || exit $?
  for f in plain fc_bf16 fc; do python -c "import json;d=json.load(open('$O/${f}_r$r.json'));print('$f', d['value'], d['ms_per_step'], d.get('hipgraph'), d.get('capture_error'))"; done
done

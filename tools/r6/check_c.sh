#!/bin/bash
# Round 6: s2t LDS epilogue (tests + A/B) and the DP-path checks
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_s2t_gpu.py tests/test_capture_group_gpu.py tests/test_graph_gpu.py tests/test_family_r_gpu.py tests/test_ddp_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
b() { # tag args...
  local t=$1; shift
  timeout -k 10 300 env "$@" python bench.py --steps 15 --warmup 4 ${BARGS:-} > $O/$t.json 2> $O/$t.err || return $?
  python -c "import json;d=json.load(open('$O/$t.json'));print('$t', d['value'], d['ms_per_step'], d.get('hipgraph'), d.get('capture_error'))"
}
for r in 1 2; do
  b lds_r$r P2P_S2T_EPI=1 || exit $?
  b reg_r$r P2P_S2T_EPI=0 || exit $?
done
BARGS="--force_comm --comm_dtype bf16" b fc_bf16 X=1 || exit $?
BARGS="--force_comm" b fc X=1 || exit $?

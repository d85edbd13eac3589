#!/bin/bash
# Round-4 pass q: reducer graph tests (direct gradients under capture), then the benches that
# need re-measuring on the fixed build (DP direct, W32 off, up-fold default).  Every step that
# aborts / faults / times out ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py tests/test_ddp_gpu.py tests/test_s2t_gpu.py -q -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d.get("max_mem_gib"), d.get("comm"))
PY
}
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json >> $O/all.jsonl; }
run headline || exit 1
run force_comm --force_comm
P2P_DIRECT_GRAD=1 run force_comm_direct --force_comm
run headline2
run famR --family ref --batch 64
exit 0

#!/bin/bash
# Round-4 pass s: norm-chain determinism probe; family R and headline on the current build;
# then the direct-gradient DP step with the reducer's stream log (compute-stream fix).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 180 python -u tools/diag_s2t_det.py > $O/det.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/det.txt; fatal $rc
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d.get("max_mem_gib"), d.get("comm"))
PY
}
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json >> $O/all.jsonl; }
run famR --family ref --batch 64
run headline || exit 1
P2P_DDP_DEBUG=1 P2P_DIRECT_GRAD=1 run force_comm_direct --force_comm
grep "^\[reducer\]" $O/force_comm_direct.json | sort | uniq -c | sort -rn | head -20
run force_comm --force_comm
exit 0

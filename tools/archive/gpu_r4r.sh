#!/bin/bash
# Round-4 pass r: norm-chain determinism probe (s2t vs implicit-GEMM route), then the benches
# of pass q (headline, DP reducers with and without direct gradients, family R).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 180 python -u tools/diag_s2t_det.py > $O/det.txt 2>&1; rc=$?; fatal $rc
grep -v amdgpu.ids $O/det.txt
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

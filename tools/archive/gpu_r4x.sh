#!/bin/bash
# Round-4 pass x: family-R step oracle test with / without the residual-join fusion (the shared
# PReLU slope gradient), then the family-R A/Bs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
for f in 0 1; do
  P2P_RES_FUSE=$f timeout -k 10 300 python -u -m pytest tests/test_family_r_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "step_gpu_matches_cpu_oracle" > $O/fam_fuse$f.log 2>&1; rc=$?
  echo "fuse=$f rc=$rc"; fatal $rc
  python - $f <<'PY'
import json, sys
rows = [json.loads(l) for l in open("gpurun_out/bounds.jsonl") if "family_r_step_vs_oracle" in l][-1]["rows"]
json.dump(rows, open(f"gpurun_out/r4x/rows_fuse{sys.argv[1]}.json", "w"))
for r in rows:
    if r[0].endswith("relu.weight") or r[0].startswith("loss"):
        print(r)
PY
done
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d.get("max_mem_gib"))
PY
}
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json >> $O/all.jsonl; }
run famR --family ref --batch 64 || exit 1
P2P_RES_FUSE=0 run famR_nores --family ref --batch 64
P2P_CPHASE_ASSIGN=0 run famR_add --family ref --batch 64
P2P_RES_FUSE=0 P2P_CPHASE_ASSIGN=0 run famR_neither --family ref --batch 64
exit 0

#!/bin/bash
# Same-box A/B of the headline default batch (2048 vs 1024, interleaved), then the family-R
# batch sweep: B = 64 / 128 / 256.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4famb
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d.get("max_mem_gib"))
PY
}
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json >> $O/all.jsonl; }
run h2048 || exit 1
run h1024 --batch 1024 || exit 1
run h2048b || exit 1
run h1024b --batch 1024 || exit 1
run r64 --family ref --batch 64 || exit 1
run r128 --family ref --batch 128 || exit 1
run r256 --family ref --batch 256
exit 0

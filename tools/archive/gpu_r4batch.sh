#!/bin/bash
# Batch sweep of the final build (288 GB HBM sizing): B = 1024 / 1536 / 2048, bf16 and fp8.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4batch
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d.get("max_mem_gib"))
PY
}
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json >> $O/all.jsonl; }
run b1024 --batch 1024 || exit 1
run b1536 --batch 1536 || exit 1
run b2048 --batch 2048 || exit 1
run b1024_2 --batch 1024
run f8_1024 --batch 1024 --precision fp8
run f8_2048 --batch 2048 --precision fp8
exit 0

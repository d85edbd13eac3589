#!/bin/bash
# Final-build numbers for the other BASELINE configs: 512x512 training and generator inference.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4misc
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d.get("max_mem_gib"))
PY
}
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json >> $O/all.jsonl; }
run s512_b256 --size 512 --batch 256 || exit 1
run s512_b512 --size 512 --batch 512
run infer_b256 --mode infer --batch 256
run infer_b256_f8 --mode infer --batch 256 --precision fp8
exit 0

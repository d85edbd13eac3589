#!/bin/bash
# Round-4 pass u: route diagnosis with well-conditioned loss weights; the new split-K reduce
# (bitwise vs the old kernel) and the s2t tests; family R and headline benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 180 python -u tools/diag_s2t_route.py randn > $O/route_randn.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/route_randn.txt | grep -v worst; fatal $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_s2t_gpu.py "tests/test_kernels_gpu.py::test_wgrad_split_reduce_kernels_bitwise" "tests/test_kernels_gpu.py::test_conv_wgrad_large_m" -s > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error|errors vs" $O/tests.log | tail -12; fatal $rc; [ $rc -eq 0 ] || exit $rc
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d.get("max_mem_gib"))
PY
}
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json >> $O/all.jsonl; }
run famR --family ref --batch 64 || exit 1
P2P_WRED_OLD=1 run famR_old --family ref --batch 64
run headline
P2P_WRED_OLD=1 run headline_old
exit 0

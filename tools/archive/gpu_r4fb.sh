#!/bin/bash
# Round-4 fp8 follow-up: the round-3 pk8 halo kernel restored (tests + traces), and the fp8
# halo-kernel routing per variant (P2P_S2T_F8 bits: 1 = ConvT forward, 2 = input gradient).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4fb
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_image_path_gpu.py tests/test_pix2pix_step_gpu.py tests/test_fp8_gpu.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -6; fatal $rc; [ $rc -eq 0 ] || exit $rc
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d.get("max_mem_gib"))
PY
}
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json >> $O/all.jsonl; }
for m in 3 1 2 0; do P2P_S2T_F8=$m run f8_256_m$m --precision fp8 --batch 256 || exit 1; done
run bf_256 --batch 256
tr() {
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- \
    python bench.py --batch 256 --steps 5 --warmup 2 "$@" > $O/$tag.log 2>&1; local rc=$?; fatal $rc
  python tools/prof_summary.py $O/$tag/run_kernel_trace.csv --steps 5 --top 60 --width 160 > $O/$tag.txt
  head -2 $O/$tag.txt | tail -1; grep -E "halo_pk8|conv_s2t" $O/$tag.txt | cut -c1-120
}
tr f8 --precision fp8
tr bf
exit 0

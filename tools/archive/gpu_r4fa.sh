#!/bin/bash
# Round-4 fp8 check: B = 256 fp8 step A/Bs (halo kernel on / off) and its kernel trace, to
# compare against the round-3 fp8 trace (profiles/fp8_b256_kernels_r3t.txt).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4fa
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d.get("max_mem_gib"))
PY
}
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json >> $O/all.jsonl; }
run f8_256 --precision fp8 --batch 256 || exit 1
P2P_NO_S2T=1 run f8_256_nos2t --precision fp8 --batch 256
P2P_WRED_OLD=1 run f8_256_wredold --precision fp8 --batch 256
run bf_256 --batch 256
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/f8 -o run -- \
  python bench.py --precision fp8 --batch 256 --steps 5 --warmup 2 > $O/f8.log 2>&1; rc=$?; fatal $rc
python tools/prof_summary.py $O/f8/run_kernel_trace.csv --steps 5 --top 60 --width 160 > $O/f8.txt
head -40 $O/f8.txt | cut -c1-150
exit 0

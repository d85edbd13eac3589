#!/bin/bash
# Round-4 final profiles: kernel traces of the final build (headline B = 256 / 1024, fp8
# B = 256, family R B = 64) and the PMC roofline at B = 256 (kernel trace + pmc only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4prof
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
tr() {  # tag, batch, extra bench args...
  local tag=$1 b=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- \
    python bench.py --batch $b --steps 5 --warmup 2 "$@" > $O/$tag.log 2>&1; local rc=$?
  fatal $rc; [ $rc -eq 0 ] || { echo "$tag trace rc=$rc"; return 1; }
  python tools/prof_summary.py $O/$tag/run_kernel_trace.csv --steps 5 --top 80 --width 160 > $O/$tag.txt
  head -2 $O/$tag.txt | tail -1
}
tr b256 256 || exit 1
tr b1024 1024 || exit 1
tr f8_b256 256 --precision fp8 || exit 1
tr famr64 64 --family ref || exit 1
OUT=$O/roof B=256 timeout -k 10 700 bash tools/gpu_roofline.sh > $O/roof.log 2>&1; rc=$?; echo "roofline rc=$rc"; fatal $rc
head -45 $O/roof/roofline.md | cut -c1-160
exit 0

#!/bin/bash
# Round-4 pass t: s2t / implicit-GEMM route diagnosis of the norm chain, then kernel traces of
# the current build (family R B = 64, headline B = 256 and B = 1024).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 180 python -u tools/diag_s2t_route.py > $O/route.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/route.txt; fatal $rc
tr() {  # tag, batch, extra bench args...
  local tag=$1 b=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- \
    python bench.py --batch $b --steps 5 --warmup 2 "$@" > $O/$tag.log 2>&1; local rc=$?
  fatal $rc; [ $rc -eq 0 ] || { echo "$tag trace rc=$rc"; return 1; }
  python tools/prof_summary.py $O/$tag/run_kernel_trace.csv --steps 5 --top 60 --width 160 > $O/$tag.txt
  head -3 $O/$tag.txt
}
tr famr64 64 --family ref || exit 1
tr b256 256 || exit 1
tr b1024 1024
exit 0

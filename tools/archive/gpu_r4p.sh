#!/bin/bash
# Round-4 pass p: kernel traces of the final build (headline B = 256 and B = 1024, family R
# B = 64) and the PMC roofline at B = 256 -- rocprofv3 kernel trace / pmc only.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
tr() {  # tag, batch, extra bench args...
  local tag=$1 b=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- \
    python bench.py --batch $b --steps 5 --warmup 2 "$@" > $O/$tag.log 2>&1 || { echo "$tag trace rc=$?"; return 1; }
  python tools/prof_summary.py $O/$tag/run_kernel_trace.csv --steps 5 --top 60 --width 160 > $O/$tag.txt
  head -3 $O/$tag.txt
}
tr b256 256 || exit 1
tr b1024 1024 || exit 1
tr famr64 64 --family ref
OUT=$O/roof B=256 timeout -k 10 600 bash tools/gpu_roofline.sh > $O/roof.log 2>&1; echo "roofline rc=$?"; head -30 $O/roof/roofline.md

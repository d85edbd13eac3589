#!/bin/bash
# PMC roofline of the family-R step (B=64, eager passes) on the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/roofR B=64 BENCH_ARGS="--family ref" bash tools/gpu_roofline.sh > gpurun_out/roofR_run.txt 2>&1
rc=$?
tail -5 gpurun_out/roofR_run.txt
for d in probe sq fetch write; do rm -rf gpurun_out/roofR/$d/*/ 2>/dev/null; done
exit $rc

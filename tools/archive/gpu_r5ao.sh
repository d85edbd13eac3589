#!/bin/bash
# roofline of the final round-5 build: per-kernel counter passes over B=1024 eager steps + probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/roof5f B=1024 bash tools/gpu_roofline.sh > gpurun_out/roof5f_run.txt 2>&1
rc=$?
tail -5 gpurun_out/roof5f_run.txt
for d in probe sq fetch write; do rm -rf gpurun_out/roof5f/$d/*/ 2>/dev/null; done
exit $rc

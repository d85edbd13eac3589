#!/bin/bash
# bisect the family-R eager-vs-replay mismatch: gradient pairing fully off (no held refs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5w
mkdir -p $O
run() { timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_graph_family_r_gpu.py -k replay > $O/$1.log 2>&1; echo "$1: $(tail -1 $O/$1.log)"; }
P2P_GRAD_PAIR=0 run pair_off
P2P_GRAD_PAIR=0 P2P_M32=0 run pair_off_m32_off
run pair_on
exit 0

#!/bin/bash
# Round-4 pass n: same-box bench A/Bs of the round-4 build -- headline (B = 1024) with / without
# the s2t halo kernel and its 32-wide case, fp8, B = 256, DP on one GPU (autograd and direct
# bucket gradients), family R with / without the up-sample dgrad fold.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'], d.get('max_mem_gib'), d.get('comm'))"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2>> $O/err.log || { echo "$tag FAILED rc=$?"; tail -3 $O/err.log; return 1; }; echo "$tag $(j $O/$tag.json)"; cat $O/$tag.json >> $O/all.jsonl; }
timeout -k 10 180 python -u tools/diag_direct.py > $O/diag_direct.txt 2>&1; echo "diag_direct rc=$?"; grep -v "^\[rank" $O/diag_direct.txt | grep -v "^    (" | tail -30
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py tests/test_ddp_gpu.py -q -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1; echo "graph/ddp tests rc=$?"; grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -8
run headline || exit 1
P2P_NO_S2T=1 run nos2t
P2P_S2T_W32=0 run w32off
run headline2
run fp8 --precision fp8
run b256 --batch 256
run force_comm --force_comm
P2P_DIRECT_GRAD=1 run force_comm_direct --force_comm
run famR --family ref --batch 64
P2P_UP_FOLD=1 run famR_upfold --family ref --batch 64
exit 0

#!/bin/bash
# Round-4 pass i: direct-gradient reducer diagnosis; family-R fold / stats benches; norm
# bandwidth A/B; inner-gradient diagnosis; then the full GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 180 python tools/diag_direct.py > $O/diag_direct.txt 2>&1; echo "diag_direct rc=$?"; grep -v "^\[rank\|^  " $O/diag_direct.txt | tail -30
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'], d.get('max_mem_gib'), d.get('comm'))"; }
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$tag.json 2>> $O/err.log || { echo "$tag FAILED"; tail -5 $O/err.log; return 1; }; echo "$tag $(j $O/$tag.json)"; cat $O/$tag.json >> $O/all.jsonl; }
run force_comm --force_comm
run famR --family ref --batch 64
P2P_FOLD_EPI=0 run famR_nofold --family ref --batch 64
for nt in 0 1 3; do P2P_NORM_NT=$nt timeout -k 10 120 python tools/norm_bw.py > $O/norm_bw_nt$nt.txt 2>&1 || exit $?; tail -1 $O/norm_bw_nt$nt.txt; done
timeout -k 10 240 python tools/diag_inner_grad.py > $O/diag_inner.txt 2>&1; echo "diag rc=$?"; tail -12 $O/diag_inner.txt
rem=$((1140 - SECONDS)); [ $rem -gt 840 ] && rem=840; echo "suite budget ${rem}s"
timeout -k 10 $rem python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "passed|failed|Error|error" $O/tests.log | tail -30; exit 1; }
tail -1 $O/tests.log
grep "convergence:" $O/tests.log

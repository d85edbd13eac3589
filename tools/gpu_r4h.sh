#!/bin/bash
# Round-4 pass h: s2t epilogue rework headline A/B (W32 on / off); DP direct gradients (tests
# + force_comm bench); convergence test.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_s2t_gpu.py tests/test_fp8_gpu.py tests/test_production_shapes_gpu.py tests/test_graph_gpu.py tests/test_ddp_gpu.py tests/test_wgrad_stream_gpu.py tests/test_convergence_gpu.py -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "passed|failed|Error|error" $O/tests.log | tail -30; exit 1; }
tail -1 $O/tests.log
grep "convergence:" $O/tests.log
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'], d.get('max_mem_gib'), d.get('comm'))"; }
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.json 2>> $O/err.log || exit $?; echo "$tag $(j $O/$tag.json)"; cat $O/$tag.json >> $O/all.jsonl; }
run headline
P2P_S2T_W32=0 run w32off
P2P_NO_S2T=1 run nos2t
run force_comm --force_comm
P2P_WGRAD_STREAM=0 run nostream
run headline2
P2P_S2T_W32=0 run w32off2
run force_comm2 --force_comm
timeout -k 10 300 python tools/diag_inner_grad.py > $O/diag_inner.txt 2>&1; echo "diag rc=$?"; tail -12 $O/diag_inner.txt

#!/bin/bash
# production-shape bounds (m32 kernel list, ILL_K 1.5), DDP (direct default), graph; L2 diag
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5l
mkdir -p $O
rm -f gpurun_out/bounds.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_production_shapes_gpu.py tests/test_ddp_gpu.py tests/test_graph_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log | tail -12
cp gpurun_out/bounds.jsonl $O/bounds.jsonl
timeout -k 10 900 python -u tools/diag_inner_grad.py --B 64 --seeds 11,12,13 --kinds fp32,eager,native \
  > $O/diag_inner.txt 2>&1 || { tail -20 $O/diag_inner.txt; exit 1; }
grep "^L2" $O/diag_inner.txt

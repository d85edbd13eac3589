#!/bin/bash
# Round-4 pass o: direct-gradient reducer event trace first, then the GPU tests that failed in
# r4m2 (convergence seed ensemble, fp8 production bound, reducer graph test) and the DDP
# rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 180 python -u tools/diag_direct.py > $O/diag_direct.txt 2>&1; echo "diag_direct rc=$?"; grep -v "^\[rank" $O/diag_direct.txt | tail -80
timeout -k 10 600 python -u -m pytest tests/test_convergence_gpu.py tests/test_production_shapes_gpu.py tests/test_ddp_gpu.py tests/test_graph_gpu.py -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error|convergence:|production-shape" $O/tests.log | tail -20
exit $rc

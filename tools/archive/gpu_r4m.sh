#!/bin/bash
# Round-4 pass l: the full GPU suite (unserialised, the driver's round-end order), then the
# direct-gradient reducer event trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4m2
mkdir -p $O
timeout -k 10 840 python -u -m pytest tests -m gpu --maxfail=8 -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -20; grep "convergence:\|production-shape" $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tools/diag_direct.py > $O/diag_direct.txt 2>&1; echo "diag_direct rc=$?"; grep -v "^\[rank" $O/diag_direct.txt | tail -70

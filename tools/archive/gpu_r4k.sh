#!/bin/bash
# Round-4 pass k: the exact r4i test prefix (pix2pix CLI eager / graph / fp8, family-R CLI,
# conv fuzz) with every launch serialised: an out-of-bounds access then raises at its own
# launch.  Then the direct-gradient reducer trace (tools/diag_direct.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
export AMD_SERIALIZE_KERNEL=3
timeout -k 10 600 python -u -m pytest tests/test_cli_gpu.py tests/test_conv_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread > $O/serial.txt 2>&1; rc=$?; echo "serial rc=$rc"; grep -E "passed|failed|Error|error|Traceback|File \"/" $O/serial.txt | tail -40; [ $rc -eq 0 ] || exit $rc
unset AMD_SERIALIZE_KERNEL
timeout -k 10 180 python -u tools/diag_direct.py > $O/diag_direct.txt 2>&1; echo "diag_direct rc=$?"; grep -v "^\[rank" $O/diag_direct.txt | tail -40

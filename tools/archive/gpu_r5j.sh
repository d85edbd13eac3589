#!/bin/bash
# W5b: where the direct-gradient watchdog abort comes from (debug trace of the reducer)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
P2P_DDP_DEBUG=1 P2P_DIRECT_GRAD=1 timeout -k 10 300 python -u bench.py --force_comm --steps 3 --warmup 2 > $O/dbg.txt 2>&1
echo "exit $?"
grep -v "^frame\|^Exception\|^$" $O/dbg.txt | cut -c1-220 | tail -60
exit 0

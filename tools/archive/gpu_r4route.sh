#!/bin/bash
# Conv routing census of one eager headline step (B = 256): which MODE-1 convs take the
# stride-2 halo kernel and which fall back to the implicit GEMM, with the reason fields.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4route
mkdir -p $O
P2P_ROUTE_LOG=1 timeout -k 10 300 python bench.py --batch 256 --steps 1 --warmup 1 --no_graph > $O/b256.json 2> $O/b256.err; rc=$?
echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep "^\[route\] mode 1" $O/b256.err | sort | uniq -c | sort -rn | head -40

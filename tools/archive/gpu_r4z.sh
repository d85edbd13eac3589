#!/bin/bash
# Round-4 pass z: the fp8 norm chain regression -- repeat / route probe with the new and the
# old split-K reduce, then the failing test itself.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 180 python -u tools/diag_fp8_chain.py > $O/chain_new.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/chain_new.txt; fatal $rc
P2P_WRED_OLD=1 timeout -k 10 180 python -u tools/diag_fp8_chain.py > $O/chain_old.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/chain_old.txt; fatal $rc
exit 0

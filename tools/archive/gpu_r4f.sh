#!/bin/bash
# Round-4 pass f: s2t timeline probe (co-residency, loop vs epilogue time, overlap).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 120 python tools/s2t_timeline.py > $O/tl_w64.txt 2>&1 || { tail $O/tl_w64.txt; exit 1; }
cat $O/tl_w64.txt
P2P_S2T_STAGGER=6000 timeout -k 10 120 python tools/s2t_timeline.py > $O/tl_w64_st.txt 2>&1 || exit 1
echo "--- stagger 6000 (per-CU arrival)"; cat $O/tl_w64_st.txt
timeout -k 10 120 python tools/s2t_timeline.py --act none > $O/tl_w64_none.txt 2>&1 || exit 1
echo "--- no gate"; cat $O/tl_w64_none.txt
timeout -k 10 120 python tools/s2t_timeline.py --C 256 --H 32 --Cout 128 > $O/tl_w32.txt 2>&1 || exit 1
echo "--- W32"; cat $O/tl_w32.txt

#!/bin/bash
# Round-4 pass g: s2t with the up-front buffer-resource EXT epilogue -- tests, layer timing,
# timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_s2t_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
L() { timeout -k 10 120 python tools/s2t_layer.py --mode dgrad --iters 10 "$@" 2>>$O/err.log | tail -1 || exit $?; }
for shape in "--N 1024 --C 128 --H 64 --Cout 64" "--N 1024 --C 256 --H 32 --Cout 128"; do
  for act in lrelu none; do
    L $shape --act $act
    P2P_S2T_GRID=0 L $shape --act $act
    P2P_NO_S2T=1 L $shape --act $act
  done
done
timeout -k 10 120 python tools/s2t_timeline.py > $O/tl_w64.txt 2>&1 || exit 1
cat $O/tl_w64.txt
timeout -k 10 120 python tools/s2t_timeline.py --C 256 --H 32 --Cout 128 > $O/tl_w32.txt 2>&1 || exit 1
cat $O/tl_w32.txt

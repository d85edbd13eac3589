#!/bin/bash
# Round-4 pass e: s2t stagger by grid halves; convergence test.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
L() { timeout -k 10 120 python tools/s2t_layer.py --mode dgrad --iters 10 "$@" 2>>$O/err.log | tail -1 || exit $?; }
for shape in "--N 1024 --C 128 --H 64 --Cout 64" "--N 1024 --C 256 --H 32 --Cout 128"; do
  for st in 0 3000 6000 10000 15000; do
    echo "stagger-halves $st: $(P2P_S2T_STAGGER_MODE=1 P2P_S2T_STAGGER=$st L $shape)"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_convergence_gpu.py -x -v -s --timeout 380 --timeout-method thread > $O/conv.log 2>&1; echo "convergence rc=$?"
grep -E "convergence:|passed|failed|Error" $O/conv.log | tail -5

#!/bin/bash
# Round 6: K-tile order A/B of the 32x32 conv tiles (P2P_TAP_ORDER), numerics + bench + L2 hits
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
P2P_TAP_ORDER=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_m32_gpu.py -k oracle > $O/m32_tests_o3.log 2>&1 || { tail -20 $O/m32_tests_o3.log; exit 1; }
tail -2 $O/m32_tests_o3.log
for r in 1 2; do
  for o in 0 1 3; do
    P2P_TAP_ORDER=$o timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/bench_o${o}_r$r.json 2> $O/bench_o${o}_r$r.err || { tail -5 $O/bench_o${o}_r$r.err; exit 1; }
    echo "order $o run $r: $(python -c "import json;d=json.load(open('$O/bench_o${o}_r$r.json'));print(d['value'],d['ms_per_step'])")"
  done
done
for o in 0 3; do
  P2P_TAP_ORDER=$o timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/l2_o$o -o run -- \
    python bench.py --batch 1024 --steps 2 --warmup 1 --no_graph > $O/l2_o$o.log 2>&1 || { tail -5 $O/l2_o$o.log; exit 1; }
done
echo done

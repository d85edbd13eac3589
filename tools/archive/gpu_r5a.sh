#!/bin/bash
# Round 5, first GPU call: family-R capture fix, m32 tile numerics, per-layer conv A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_conv_m32_gpu.py tests/test_graph_family_r_gpu.py > $O/tests.log 2>&1
rc=$?
tail -25 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|Fault|fault" $O/tests.log | head -20; exit 1; fi
for v in 1 0; do
  P2P_M32=$v timeout -k 10 400 python -u tools/conv_bench.py --batch 256 --iters 10 --layers e3,e4,d4,d3,c3,c4 \
    --json_out $O/conv_m32_$v.json > $O/conv_m32_$v.log 2>&1 || { tail -20 $O/conv_m32_$v.log; exit 1; }
done
paste <(cut -c1-150 $O/conv_m32_1.log) /dev/null
echo ----
cut -c1-150 $O/conv_m32_0.log
timeout -k 10 300 python -u bench.py --family ref --batch 64 --steps 10 --warmup 3 > $O/famr64.json 2> $O/famr64.err || { tail -20 $O/famr64.err; exit 1; }
cat $O/famr64.json

#!/bin/bash
# wgrad 32x32x16 tile: numerics, per-layer A/B (wgrad), headline step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_m32_gpu.py tests/test_graph_gpu.py tests/test_ddp_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/conv_bench.py --batch 256 --iters 10 --rounds 3 --m32 1,0 \
  --layers e3,e4,e5,d5,d4,d3,c3,c4 --ops wgrad --json_out $O/ab.json > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
python - <<'PY'
import json
for r in json.load(open("gpurun_out/r5f/ab.json")):
    a, b = r.get("wgrad_m321_us"), r.get("wgrad_m320_us")
    if a and b:
        print(f'{r["layer"]:4s} wgrad m32 {a:8.1f} us  16x16 {b:8.1f} us  ({(b / a - 1) * 100:+5.1f} %)  {r.get("wgrad_m321_tflops")} TF/s')
PY
for v in 1 0; do
  P2P_M32=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  tail -1 $O/bench.jsonl | cut -c1-150
done

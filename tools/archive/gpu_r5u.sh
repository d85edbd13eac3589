#!/bin/bash
# 128x128 two-per-CU m32 tile (level 2): numerics, per-layer A/B vs the 256x128 tile, headline step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5u
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_m32_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/conv_bench.py --batch 256 --iters 10 --rounds 3 --m32 2,1 \
  --layers e2,c2,e3,c3,d3 --ops fwd,dgrad --json_out $O/ab.json > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
python - <<'PY'
import json
for r in json.load(open("gpurun_out/r5u/ab.json")):
    out = [r["layer"]]
    for op in ("fwd", "dgrad"):
        a, b = r.get(op + "_m322_us"), r.get(op + "_m321_us")
        if a and b:
            out.append(f"{op} 128x128x2 {a:8.1f} us  256x128 {b:8.1f} us  ({(b / a - 1) * 100:+5.1f} %)")
    print("  ".join(out))
PY
for v in 2 1 2 1; do
  P2P_M32=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  echo "P2P_M32=$v $(tail -1 $O/bench.jsonl | cut -c1-120)"
done

#!/bin/bash
# in-process interleaved A/B of the 32x32x16 conv tiles vs the 16x16x32 tiles, per layer
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 600 python -u tools/conv_bench.py --batch 256 --iters 10 --rounds 3 --m32 1,0 \
  --layers e2,e3,e4,e5,d5,d4,d3,d2,c2,c3,c4 --ops fwd,dgrad --json_out $O/ab.json > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
python - <<'PY'
import json
rows = json.load(open("gpurun_out/r5b/ab.json"))
for r in rows:
    out = [r["layer"]]
    for op in ("fwd", "dgrad"):
        a, b = r.get(op + "_m321_us"), r.get(op + "_m320_us")
        if a and b:
            out.append(f"{op} m32 {a:8.1f} us  16x16 {b:8.1f} us  ({(b / a - 1) * 100:+5.1f} %)")
    print("  ".join(out))
PY

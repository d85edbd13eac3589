#!/bin/bash
# A/B kernel builds (tools/build_ext.py --out) on the per-layer conv bench: LIBS="a.so b.so"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in base ${LIBS}; do
  if [ "$lib" = base ]; then unset P2P_LIB; else export P2P_LIB=$lib; fi
  timeout -k 10 300 python tools/conv_bench.py --batch 64 --iters ${ITERS:-10} --layers ${LAYERS:-c4,e4,d4,e3,d3,d2,e2} --ops ${OPS:-fwd,dgrad,wgrad} > gpurun_out/ab_$(basename $lib .so).jsonl 2>/dev/null || exit $?
done
python - <<'PY'
import json, glob, os
rows = {}
for f in sorted(glob.glob("gpurun_out/ab_*.jsonl")):
    tag = os.path.basename(f)[3:-6]
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); rows.setdefault(d["layer"], {})[tag] = d
tags = sorted({t for r in rows.values() for t in r})
print("layer  " + "  ".join(f"{t:>26s}" for t in tags))
for lay, r in rows.items():
    print(f"{lay:6s} " + "  ".join(f"{r[t].get('fwd_us',0):7.1f}/{r[t].get('dgrad_us',0):7.1f}/{r[t].get('wgrad_us',0):7.1f}" if t in r else " " * 26 for t in tags))
PY

#!/bin/bash
# m32 swapped-operand epilogue: numerics, per-layer A/B, then a B=1024 kernel trace of the step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_m32_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/conv_bench.py --batch 256 --iters 10 --rounds 3 --m32 1,0 \
  --layers e2,e3,e4,d4,d3,c2,c3,c4 --ops fwd,dgrad --json_out $O/ab.json > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
python - <<'PY'
import json
for r in json.load(open("gpurun_out/r5e/ab.json")):
    out = [r["layer"]]
    for op in ("fwd", "dgrad"):
        a, b = r.get(op + "_m321_us"), r.get(op + "_m320_us")
        if a and b:
            out.append(f"{op} m32 {a:8.1f} us  16x16 {b:8.1f} us  ({(b / a - 1) * 100:+5.1f} %)")
    print("  ".join(out))
PY
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --batch 1024 --steps 5 --warmup 2 > $O/prof_log.txt 2>&1 || { tail $O/prof_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 45 --width 150 > $O/b1024_kernels.txt
head -50 $O/b1024_kernels.txt

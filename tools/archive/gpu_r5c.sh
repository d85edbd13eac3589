#!/bin/bash
# m32 tiles: numerics, in-process A/B per layer, per-block phase stamps, SQ counters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_m32_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u tools/conv_bench.py --batch 256 --iters 10 --rounds 3 --m32 1,0 \
  --layers e2,e3,e4,d4,d3,d2,c2,c3,c4 --ops fwd,dgrad --json_out $O/ab.json > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
python - <<'PY'
import json
rows = json.load(open("gpurun_out/r5c/ab.json"))
for r in rows:
    out = [r["layer"]]
    for op in ("fwd", "dgrad"):
        a, b = r.get(op + "_m321_us"), r.get(op + "_m320_us")
        if a and b:
            out.append(f"{op} m32 {a:8.1f} us  16x16 {b:8.1f} us  ({(b / a - 1) * 100:+5.1f} %)")
    print("  ".join(out))
PY
P2P_LIB=p2p_pytorch_amd/_C/m32_stamps.so timeout -k 10 300 python -u tools/m32_stamps.py --layers c4,c3,e3,e2,d4,d3 \
  > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
CNT="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d $O/sq -o sq -- \
  python tools/conv_bench.py --batch 256 --iters 3 --rounds 1 --m32 1,0 --layers c4,c3 --ops fwd \
  > $O/log_sq.txt 2>&1 || { tail -20 $O/log_sq.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/g -o g -- \
  python tools/conv_bench.py --batch 256 --iters 3 --rounds 1 --m32 1,0 --layers c4,c3 --ops fwd \
  > $O/log_g.txt 2>&1 || { tail -20 $O/log_g.txt; exit 1; }
python tools/pmc_summary.py $O > $O/summary.txt
grep -A24 "conv_fwd" $O/summary.txt | head -120

#!/bin/bash
# Round-3 pass i: counters of the s2t kernel vs the implicit GEMM on one layer geometry.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
for m in convt dgrad; do
  timeout -k 10 120 python tools/s2t_layer.py --mode $m || exit $?
  P2P_NO_S2T=1 timeout -k 10 120 python tools/s2t_layer.py --mode $m || exit $?
done
CNT="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for m in convt dgrad; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d $O/pmc_$m -o run -- python tools/s2t_layer.py --mode $m --iters 5 > $O/pmc_$m.log 2>&1 || exit $?
  P2P_NO_S2T=1 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d $O/pmc0_$m -o run -- python tools/s2t_layer.py --mode $m --iters 5 > $O/pmc0_$m.log 2>&1 || exit $?
done
CNT2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for m in convt dgrad; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT2 --output-format csv -d $O/pmcb_$m -o run -- python tools/s2t_layer.py --mode $m --iters 5 > $O/pmcb_$m.log 2>&1 || exit $?
done
python - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/r3i/pmc*_*")):
    fs = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"]
        if "conv" not in k:
            continue
        k = k.split("(")[0][-60:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        print(d.split("/")[-1], k, {c: round(x / 1e6, 3) for c, x in sorted(v.items())})
PY

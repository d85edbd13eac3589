#!/bin/bash
# PMC counters (kernel-trace only, never with sys/runtime trace) for the per-layer conv
# kernels: issue stalls vs parked waves vs MFMA busy, LDS bank conflicts, clock.
#   LAYERS=c4,d3 OPS=fwd bash tools/gpu_pmc.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
CNT="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d $OUT -o sq -- \
  python tools/conv_bench.py --batch 64 --iters 3 --layers ${LAYERS:-c4,d3,e2} --ops ${OPS:-fwd,dgrad,wgrad} \
  > $OUT/log_sq.txt 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $OUT -o g -- \
  python tools/conv_bench.py --batch 64 --iters 3 --layers ${LAYERS:-c4,d3,e2} --ops ${OPS:-fwd,dgrad,wgrad} \
  > $OUT/log_g.txt 2>&1 || exit $?
python tools/pmc_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt

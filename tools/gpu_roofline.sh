#!/bin/bash
# Per-kernel counter passes over whole (eager) B=256 training steps, one rocprofv3 run per
# counter group (kernel trace + pmc only; never with sys/runtime traces), then the
# roofline table (tools/roofline.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/roof
mkdir -p $OUT
B=${B:-256}
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 420 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
    python bench.py --batch $B --steps 2 --warmup 1 --no_graph > $OUT/$name.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE || exit $?
run fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
run write WRITE_SIZE GRBM_GUI_ACTIVE || exit $?
python tools/roofline.py $OUT --steps 3 > $OUT/roofline.md
head -40 $OUT/roofline.md

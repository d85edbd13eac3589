#!/bin/bash
# Per-kernel counter passes over whole (eager) training steps, one rocprofv3 run per counter
# group (kernel trace + pmc only; never with sys/runtime traces), then the roofline table
# (tools/roofline.py, MFMA counters calibrated on tools/probes/mfma_count_probe.hip).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/roof}
mkdir -p $OUT
B=${B:-256}
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
    python bench.py --batch $B --steps 2 --warmup 1 --no_graph ${BENCH_ARGS:-} > $OUT/$name.log 2>&1
}
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/probe -o run -- ./tools/probes/bin/mfma_count_probe > $OUT/probe.log 2>&1 || exit $?
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE || exit $?
run fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
run write WRITE_SIZE GRBM_GUI_ACTIVE || exit $?
python tools/roofline.py $OUT --steps 3 --probe $OUT/probe > $OUT/roofline.md
head -60 $OUT/roofline.md

#!/bin/bash
# Instruction-mix counters over a whole (un-captured) training step, per kernel:
# VALU / SALU / LDS instructions per MFMA and issue-active fraction (tools/pmc_summary.py --table).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_step
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
  --output-format csv -d $OUT -o step -- python bench.py --batch ${B:-64} --steps 2 --warmup 1 --no_graph > $OUT/log.txt 2>&1 || exit $?
python tools/pmc_summary.py $OUT --table > $OUT/table.txt
head -40 $OUT/table.txt

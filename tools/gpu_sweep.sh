#!/bin/bash
# Batch sweep sized to the 288 GB HBM: the headline step at 256x256 for
# B = 128 .. 1024, and 512x512 up to B = 512; one bench.py process per point (bf16, hipGraph),
# max_mem_gib recorded in each line.  Stops at the first failing point (e.g. out of memory).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sweep
O=gpurun_out/sweep/batch_sweep.jsonl
: > $O
for B in 128 256 384 512 768 1024; do
  timeout -k 10 300 python bench.py --batch $B --steps 10 --warmup 3 >> $O 2> gpurun_out/sweep/b$B.err || exit $?
  tail -1 $O | cut -c1-200
done
for B in 64 128 256 384; do
  timeout -k 10 300 python bench.py --size 512 --batch $B --steps 6 --warmup 2 >> $O 2> gpurun_out/sweep/s512_b$B.err || exit $?
  tail -1 $O | cut -c1-200
done

#!/bin/bash
# Round-end measurement set: headline (B256 default, B128), fp8, inference, reference family.
# Appends one JSON line per run to gpurun_out/final_bench.jsonl; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/final_bench.jsonl
run() { timeout -k 10 300 python bench.py "$@" >> $OUT 2>> gpurun_out/final_bench.err || exit $?; tail -1 $OUT | cut -c1-150; }
run --steps 20 --warmup 5
run --batch 128 --steps 20 --warmup 5
run --precision fp8 --steps 20 --warmup 5
run --precision fp8 --batch 128 --steps 20 --warmup 5
run --mode infer --steps 20 --warmup 5
run --mode infer --precision fp8 --steps 20 --warmup 5
run --family ref --batch 16 --steps 10 --warmup 3
run --family ref --batch 64 --steps 10 --warmup 3

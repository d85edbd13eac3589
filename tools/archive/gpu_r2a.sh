#!/bin/bash
# Round-2 first GPU pass: all GPU tests (incl. graph-replay equivalence, RCCL capture,
# family-R parity), smoke, bench at B=256 without / with 1-rank RCCL reducers in the graph.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/kt.log 2>&1; rc=$?
echo "gpu tests rc=$rc: $(tail -1 gpurun_out/kt.log)"; grep -E "FAILED|Error" gpurun_out/kt.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_b256.jsonl 2> gpurun_out/bench.err || exit $?
cut -c1-300 gpurun_out/bench_b256.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force_comm >> gpurun_out/bench_b256.jsonl 2>> gpurun_out/bench.err || exit $?
tail -1 gpurun_out/bench_b256.jsonl | cut -c1-300
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force_comm --comm_dtype bf16 >> gpurun_out/bench_b256.jsonl 2>> gpurun_out/bench.err || exit $?
tail -1 gpurun_out/bench_b256.jsonl | cut -c1-300

#!/bin/bash
# Full GPU pass: every gpu test, smoke, headline bench (B256 + the driver default), family-R bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/kt.log 2>&1; rc=$?
echo "gpu tests rc=$rc: $(tail -1 gpurun_out/kt.log)"; grep -E "FAILED|ERROR" gpurun_out/kt.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 python bench.py > gpurun_out/bench_default.jsonl 2> gpurun_out/bench_default.err || exit $?
cut -c1-220 gpurun_out/bench_default.jsonl
timeout -k 10 400 python bench.py --family ref --batch 64 --steps 10 --warmup 3 --c_phase_backward 0 > gpurun_out/bench_ref_nocphase.jsonl 2>&1 || exit $?
cut -c1-220 gpurun_out/bench_ref_nocphase.jsonl

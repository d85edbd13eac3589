#!/bin/bash
# full GPU tests, headline bench, 512^2 config-4 sizing, 2-rank gloo bench (graph-capture
# consensus fallback)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && rm -f gpurun_out/bounds.jsonl
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/kt.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/kt.log)"; grep -E "^FAILED|^E  " gpurun_out/kt.log | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_b256.jsonl 2> gpurun_out/bench.err || exit $?
cut -c1-200 gpurun_out/bench_b256.jsonl
for b in 128 256; do
timeout -k 10 400 python bench.py --size 512 --batch $b --steps 10 --warmup 3 >> gpurun_out/bench512.jsonl 2>> gpurun_out/bench.err || exit $?
tail -1 gpurun_out/bench512.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print('512', d['config']['per_gpu_batch'], d['value'], d['ms_per_step'], d['max_mem_gib'])"
done
P2P_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --batch 16 --steps 3 --warmup 2 > gpurun_out/bench_gloo2.jsonl 2> gpurun_out/bench_gloo2.err; echo "gloo2 rc=$?"; tail -2 gpurun_out/bench_gloo2.err; cut -c1-200 gpurun_out/bench_gloo2.jsonl

set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python tools/conv_bench.py --batch 64 --iters 10 --variants auto,g6 --layers e2,d2,c2,d3 > gpurun_out/convbench_g6.jsonl 2>&1 || exit $?
timeout -k 10 400 python bench.py --size 512 --batch 32 --steps 6 --warmup 2 > gpurun_out/bench512.jsonl 2> gpurun_out/bench512.err || exit $?
cat gpurun_out/bench512.jsonl | cut -c1-220
timeout -k 10 400 python bench.py --size 512 --batch 32 --steps 6 --warmup 2 --impl torch >> gpurun_out/bench512.jsonl 2>> gpurun_out/bench512.err || exit $?
tail -1 gpurun_out/bench512.jsonl | cut -c1-220

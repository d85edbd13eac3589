set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for b in 16 64; do
timeout -k 10 300 python bench.py --family ref --batch $b --steps 5 --warmup 2 >> gpurun_out/ref.jsonl 2>> gpurun_out/ref.err || { echo "native b=$b failed"; tail -5 gpurun_out/ref.err; exit 1; }
tail -1 gpurun_out/ref.jsonl | cut -c1-200
timeout -k 10 300 python bench.py --family ref --batch $b --steps 5 --warmup 2 --impl torch >> gpurun_out/ref.jsonl 2>> gpurun_out/ref.err || { echo "torch b=$b failed"; tail -5 gpurun_out/ref.err; exit 1; }
tail -1 gpurun_out/ref.jsonl | cut -c1-200
done

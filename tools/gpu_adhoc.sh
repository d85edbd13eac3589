set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
for f in 0 1; do
P2P_SKIP_GRAD_FUSE=$f timeout -k 10 400 python bench.py --steps 20 --warmup 5 >> gpurun_out/skip_ab.jsonl 2>> gpurun_out/skip_ab.err || exit $?
echo "fuse=$f $(tail -1 gpurun_out/skip_ab.jsonl | cut -c80-160)"
done
done

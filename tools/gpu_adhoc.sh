set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "pack_pairs or skip_grad" > gpurun_out/pack_t.log 2>&1; rc=$?; tail -5 gpurun_out/pack_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 >> gpurun_out/pack_bench.jsonl 2>> gpurun_out/pack_bench.err || exit $?
echo "$(tail -1 gpurun_out/pack_bench.jsonl | cut -c80-160)"
done
B=256 timeout -k 10 700 bash tools/gpu_prof_native.sh || exit $?
head -45 gpurun_out/native_prof_b256/summary.txt | cut -c1-150

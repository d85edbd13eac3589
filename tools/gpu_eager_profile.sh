#!/bin/bash
# Profile the stock PyTorch-ROCm eager baseline (MIOpen/hipBLASLt, bf16 autocast) for the
# headline config: per-kernel time distribution with rocprofv3 --kernel-trace --stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/eager_prof
for b in 128; do
  timeout -k 10 400 python bench.py --impl torch --batch $b --steps 10 --warmup 3 >> gpurun_out/eager.jsonl 2>> gpurun_out/eager.err || exit 1
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eager_prof -o run -- \
  python bench.py --impl torch --batch 64 --steps 5 --warmup 2 > gpurun_out/eager_prof.log 2>&1 || exit 1

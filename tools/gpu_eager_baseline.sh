#!/bin/bash
# Measure the stock PyTorch-ROCm eager baseline (MIOpen/hipBLASLt, bf16 autocast,
# channels_last) for the headline config at several per-GPU batch sizes.
set -o pipefail
mkdir -p gpurun_out
python -c "import torch;p=torch.cuda.get_device_properties(0);print(p);print(torch.__version__)" > gpurun_out/dev.txt 2>&1 || exit 1
for b in 1 16 64; do
  timeout -k 10 400 python bench.py --impl torch --batch $b --steps 10 --warmup 3 >> gpurun_out/eager.jsonl 2>> gpurun_out/eager.err || exit 1
done

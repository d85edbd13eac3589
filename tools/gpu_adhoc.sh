#!/bin/bash
# LATE (prefetch distance 2) A/B + conv numerics
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_fuzz_gpu.py tests/test_determinism_gpu.py -q -k "conv or determin" --timeout 300 --timeout-method thread > gpurun_out/kt.log 2>&1; echo "tests rc=$?: $(tail -1 gpurun_out/kt.log)"; grep -E "^FAILED" gpurun_out/kt.log | head
for r in 1 2; do
for lib in "" p2p_pytorch_amd/_C/ab/libp2p_nolate.so; do
  P2P_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b.json 2>/dev/null || exit $?
  echo "lib=[$lib] $(python -c "import json;d=json.load(open('gpurun_out/b.json'));print(d['value'], d['ms_per_step'])")"
done; done

#!/bin/bash
# tile variants g8 (256x64, 2 waves) / g89 (+256x128, 4 waves) A/B, conv numerics under each
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in g89; do
P2P_CONV_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_fuzz_gpu.py -q -k "conv" --timeout 300 --timeout-method thread > gpurun_out/kt_$v.log 2>&1; echo "tests $v rc=$?: $(tail -1 gpurun_out/kt_$v.log)"; grep -E "^FAILED" gpurun_out/kt_$v.log | head -5
done
for r in 1 2; do
for v in "" g8 g89; do
  P2P_CONV_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b.json 2>/dev/null || exit $?
  echo "variant=[$v] $(python -c "import json;d=json.load(open('gpurun_out/b.json'));print(d['value'], d['ms_per_step'])")"
done; done

#!/bin/bash
# A/B the conv kernel variants: numerics (conv tests) per variant, then per-layer timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in g2 g3 g4; do
  P2P_CONV_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "conv" > gpurun_out/kt_$v.log 2>&1; rc=$?
  echo "variant $v tests rc=$rc: $(tail -1 gpurun_out/kt_$v.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
timeout -k 10 600 python tools/conv_bench.py --batch 64 --iters 10 --variants v1,g2,g3,g4 --ops fwd,dgrad > gpurun_out/convbench_var.jsonl 2>&1; rc=$?
echo "bench rc=$rc"; cat gpurun_out/convbench_var.jsonl
exit $rc

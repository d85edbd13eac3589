#!/bin/bash
# conv tile-variant sweep on the headline bench + the two fixed GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_family_r_gpu.py tests/test_kernels_gpu.py -q -k "family_r_step or pack_pairs" --timeout 300 --timeout-method thread > gpurun_out/kt.log 2>&1; echo "tests rc=$?: $(tail -1 gpurun_out/kt.log)"
for v in "" g6 "" g6; do
  P2P_CONV_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b.json 2>/dev/null || exit $?
  echo "variant=[$v] $(python -c "import json;d=json.load(open('gpurun_out/b.json'));print(d['value'], d['ms_per_step'])")"
done

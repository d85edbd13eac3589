#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_fuzz_gpu.py tests/test_norm_fuzz_gpu.py -x -v --timeout 350 --timeout-method thread -p no:cacheprovider > gpurun_out/fuzz.log 2>&1; rc=$?
echo rc=$rc; tail -2 gpurun_out/fuzz.log; grep -E "^E |Falsifying|case=" gpurun_out/fuzz.log | head -12

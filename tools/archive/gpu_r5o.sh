#!/bin/bash
# P2P_BOUNDS_ASSERT build: the family-R CLI test, the conv / norm fuzz
# tests, the s2t, family-R step and graph tests with every out-of-range index counted; then the
# family-R step test (PReLU slope self-consistency) on the normal build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5o
mkdir -p $O
P2P_LIB=$PWD/p2p_pytorch_amd/_C/libp2p_hip_bounds.so P2P_BOUNDS_CHECK=1 timeout -k 10 1000 \
  python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_cli_gpu.py tests/test_conv_fuzz_gpu.py \
  tests/test_norm_fuzz_gpu.py tests/test_s2t_gpu.py tests/test_family_r_gpu.py tests/test_graph_family_r_gpu.py \
  tests/test_conv_m32_gpu.py > $O/bounds_tests.log 2>&1
echo "bounds build exit $?"
grep -E "PASS|FAIL|ERROR|passed|failed|out-of-range" $O/bounds_tests.log | tail -40

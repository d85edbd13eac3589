#!/bin/bash
# P2P_BOUNDS_ASSERT build over the round-5 late store paths: batch-norm partials through folds
# (flat chunks, fold_band<true>), the halo kernels' fold store, fused shuffle / unshuffle, the
# family-R step and graph tests; every out-of-range index is counted (tests/conftest.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ba
mkdir -p $O
rm -f gpurun_out/bounds.jsonl
P2P_LIB=$PWD/p2p_pytorch_amd/_C/libp2p_hip_bounds.so P2P_BOUNDS_CHECK=1 timeout -k 10 1000 \
  python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_nb_fuse_gpu.py tests/test_family_r_gpu.py \
  tests/test_graph_family_r_gpu.py tests/test_kernels_gpu.py -k "nb or family or graph or halo or fold or reflect or l2_normalize or quantize or bounds" \
  > $O/bounds_tests.log 2>&1
echo "bounds build exit $?"
grep -E "passed|failed|out-of-range" $O/bounds_tests.log | tail -10

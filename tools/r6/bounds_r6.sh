#!/bin/bash
# P2P_BOUNDS_ASSERT build over the round-6 store paths: the 512-row m32 tile (EXT / stats /
# norm partials), the fp8 m32 tile, the logits input-gradient kernel, the packed-image halo
# kernels' hoisted epilogues, the s2t LDS epilogue, the R=128 wgrad tile, the float4 reduce;
# every out-of-range index is counted (tests/conftest.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6bounds; mkdir -p $O
rm -f gpurun_out/bounds.jsonl
P2P_LIB=$PWD/alt/libp2p_hip_bounds.so P2P_BOUNDS_CHECK=1 timeout -k 10 1000 \
  python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_conv_m32_gpu.py tests/test_fp8_gpu.py \
  tests/test_image_path_gpu.py tests/test_s2t_gpu.py tests/test_kernels_gpu.py tests/test_pix2pix_step_gpu.py \
  -k "512 or m32 or logits_conv or image or pk8 or union or s2t or wgrad or step" > $O/bounds_tests.log 2>&1
rc=$?
echo "bounds build exit $rc"
grep -E "passed|failed|out-of-range" $O/bounds_tests.log | tail -6
exit $rc

#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fp8_gpu.py tests/test_conv_m32_gpu.py tests/test_determinism_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
TAG=r6h1 ROUNDS=2 BARGS="--precision fp8" bash tools/r6/ab_env.sh "P2P_M32_F8=0" "P2P_M32_F8=1" || exit $?
TAG=r6h2 ROUNDS=2 bash tools/r6/ab_env.sh "P2P_WGRAD_XCD=0" "P2P_WGRAD_XCD=1" "P2P_CLASS_MAJOR=1" || exit $?
for lib in main alt; do
  if [ $lib = alt ]; then L="P2P_LIB=alt/libp2p_nolaunder.so"; else L="X=1"; fi
  timeout -s KILL 300 env $L rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$lib -o run -- \
    python bench.py --family ref --batch 64 --steps 2 --warmup 1 --no_graph > $O/pmc_$lib.log 2>&1 || { echo "pmc $lib failed"; tail -5 $O/pmc_$lib.log; exit 1; }
done
echo done

#!/bin/bash
# Round-4 pass c: s2t layer A/B (new register-epilogue kernel / no epilogue / round-3 kernel /
# implicit GEMM) at the U-Net e2 / e3 input-gradient shapes, B = 1024, + PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
L() { timeout -k 10 120 python tools/s2t_layer.py --mode dgrad --iters 10 "$@" 2>>$O/err.log | tail -1 || exit $?; }
for shape in "--N 1024 --C 128 --H 64 --Cout 64" "--N 1024 --C 256 --H 32 --Cout 128"; do
  for act in lrelu none; do
    L $shape --act $act
    P2P_S2T_GRID=0 L $shape --act $act
    P2P_LIB=exp/libp2p_noepi.so L $shape --act $act
    P2P_LIB=exp/libp2p_old.so L $shape --act $act
    P2P_NO_S2T=1 L $shape --act $act
  done
done
CNT1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
CNT2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for v in new old; do
  lib=""; [ $v = old ] && lib=exp/libp2p_old.so
  P2P_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT1 --output-format csv -d $O/pmc_$v -o sq -- python tools/s2t_layer.py --mode dgrad --iters 3 --N 1024 > $O/pmc_$v.log 2>&1 || exit $?
  P2P_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CNT2 --output-format csv -d $O/pmc_$v -o ins -- python tools/s2t_layer.py --mode dgrad --iters 3 --N 1024 >> $O/pmc_$v.log 2>&1 || exit $?
  P2P_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$v -o f -- python tools/s2t_layer.py --mode dgrad --iters 3 --N 1024 >> $O/pmc_$v.log 2>&1 || exit $?
  P2P_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_$v -o w -- python tools/s2t_layer.py --mode dgrad --iters 3 --N 1024 >> $O/pmc_$v.log 2>&1 || exit $?
  python tools/pmc_summary.py $O/pmc_$v | grep -A40 s2t > $O/pmc_$v.txt
  cat $O/pmc_$v.txt
done

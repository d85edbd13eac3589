#!/bin/bash
# split-K reduce: float4 reduce vs the scalar build (P2P_REDUCE_SCALAR), split target 512 vs 1024
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 500 env P2P_LIB=alt/libp2p_redscalar.so rocprofv3 --kernel-trace --output-format csv -d $O/trs -o run -- python bench.py --steps 5 --warmup 2 > $O/trs.log 2>&1 || { echo "trace failed"; tail -5 $O/trs.log; exit 1; }
python tools/prof_summary.py $O/trs/run_kernel_trace.csv --steps 5 --top 70 --width 160 > $O/summary_scalar_b2048.txt
head -2 $O/summary_scalar_b2048.txt; grep -E "reduce|presum" $O/summary_scalar_b2048.txt
TAG=r6m1 ROUNDS=2 bash tools/r6/ab_env.sh "P2P_WGRAD_BLOCKS=512" "P2P_WGRAD_BLOCKS=1024" "P2P_LIB=alt/libp2p_redscalar.so" || exit $?
echo done

#!/bin/bash
# Round-6 final-build profiles: captured kernel traces (bf16 / fp8 B=2048, family R B=64) and
# the calibrated PMC roofline passes (B=1024 eager, bf16 and fp8)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6prof}; mkdir -p $O
tr() {  # tag args...
  local t=$1; shift
  timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/$t -o run -- python bench.py --steps 5 --warmup 2 "$@" > $O/$t.log 2>&1 || { echo "trace $t failed"; tail -5 $O/$t.log; return 1; }
  python tools/prof_summary.py $O/$t/run_kernel_trace.csv --steps 5 --top 70 --width 160 > $O/summary_$t.txt
  head -3 $O/summary_$t.txt
}
tr bf16_b2048 || exit 1
tr fp8_b2048 --precision fp8 || exit 1
tr famr_b64 --family ref --batch 64 || exit 1
[ -n "$NO_PMC" ] && exit 0
OUT=$O/roof_bf16 B=1024 bash tools/gpu_roofline.sh > $O/roof_bf16.log 2>&1 || { echo "roofline bf16 failed"; tail -5 $O/roof_bf16.log; exit 1; }
head -3 $O/roof_bf16/roofline.md
OUT=$O/roof_fp8 B=1024 BENCH_ARGS="--precision fp8" bash tools/gpu_roofline.sh > $O/roof_fp8.log 2>&1 || { echo "roofline fp8 failed"; tail -5 $O/roof_fp8.log; exit 1; }
echo done

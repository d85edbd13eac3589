#!/bin/bash
# fp8 weight-site zeroing on a HIP kernel (no aten fill): fp8 suite, fp8 trace + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ax
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp8_gpu.py tests/test_convergence_gpu.py > $O/fp8.log 2>&1 || { tail -30 $O/fp8.log; exit 1; }
tail -1 $O/fp8.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/f8 -o run -- \
  python bench.py --steps 5 --warmup 2 --precision fp8 > $O/f8_log.txt 2>&1 || { tail $O/f8_log.txt; exit 1; }
python tools/prof_summary.py $O/f8/run_kernel_trace.csv --steps 5 --top 120 --width 120 > $O/f8_kernels.txt
head -2 $O/f8_kernels.txt; grep -c "at::native" $O/f8_kernels.txt || true
rm -rf $O/f8
timeout -k 10 400 python -u bench.py --precision fp8 > $O/f8.json 2> $O/f8.err || { tail -20 $O/f8.err; exit 1; }
cut -c1-140 $O/f8.json

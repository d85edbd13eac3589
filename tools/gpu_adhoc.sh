#!/bin/bash
# reference-family: targeted kernel tests, family-R step / graph tests, bench, conv census, profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "halo_k9 or family_r or spectral or l1_gated or losses" > gpurun_out/t_adhoc.log 2>&1 || { tail -30 gpurun_out/t_adhoc.log; exit 1; }
tail -1 gpurun_out/t_adhoc.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_family_r_gpu.py tests/test_graph_gpu.py > gpurun_out/t_adhoc2.log 2>&1 || { tail -30 gpurun_out/t_adhoc2.log; exit 1; }
tail -1 gpurun_out/t_adhoc2.log
timeout -k 10 300 python bench.py --family ref --batch 64 --steps 10 --warmup 3 > gpurun_out/bench_ref.jsonl 2> gpurun_out/bench_ref.err || exit $?
cut -c1-200 gpurun_out/bench_ref.jsonl
timeout -k 10 300 python -u tools/conv_census.py --family ref --batch 64 --top 30 > gpurun_out/census_ref.txt 2>&1 || exit $?
OUT=gpurun_out/prof_ref; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python bench.py --family ref --batch 64 --steps 5 --warmup 2 > $OUT/log.txt 2>&1 || exit $?
python tools/prof_summary.py $OUT/run_kernel_trace.csv --steps 5 --top 45 --width 150 > $OUT/summary.txt
head -30 $OUT/summary.txt

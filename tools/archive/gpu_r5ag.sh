#!/bin/bash
# C's PixelShuffle in the l2-normalise pass; quantise + unshuffle for the expander head: kernel
# tests, family-R tests, aten census, family-R kernel trace + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5af
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "l2_normalize or quantize or pixel_shuffle or family_r" > $O/ktests.log 2>&1 || { tail -40 $O/ktests.log; exit 1; }
tail -1 $O/ktests.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_family_r_gpu.py \
  tests/test_graph_family_r_gpu.py tests/test_cli_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PYTHONPATH=$PWD timeout -k 10 300 python -u tools/probes/aten_census.py --family ref --batch 8 > $O/aten_famr.txt 2>&1 || { tail -20 $O/aten_famr.txt; exit 1; }
grep -c "at::native" $O/aten_famr.txt || true
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --family ref --batch 64 --steps 5 --warmup 2 > $O/famr_log.txt 2>&1 || { tail $O/famr_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 120 --width 120 > $O/famr_kernels.txt
head -3 $O/famr_kernels.txt
grep "pixel_shuffle\|pad_channels\|quantize\|l2norm" $O/famr_kernels.txt || true
timeout -k 10 300 python -u bench.py --family ref --batch 64 --steps 20 --warmup 5 > $O/famr.jsonl 2> $O/famr.err || { tail -20 $O/famr.err; exit 1; }
cut -c1-150 $O/famr.jsonl

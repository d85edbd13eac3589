#!/bin/bash
# Round-3 second pass: fp8 wgrad validation + A/B, norm-in-fragment experiment census,
# calibrated counter roofline, kernel trace of the headline step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_nb_fuse_gpu.py tests/test_pix2pix_step_gpu.py tests/test_production_shapes_gpu.py -x -q --timeout 240 --timeout-method thread > $O/nb.log 2>&1 || exit $?
echo "nb/step tests: $(tail -1 $O/nb.log)"
timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 240 --timeout-method thread > $O/fp8.log 2>&1; rc=$?
echo "fp8 tests rc=$rc: $(tail -1 $O/fp8.log)"
grep -E "FAILED|Error|assert" $O/fp8.log | head -20
if [ $rc -eq 0 ]; then
  for w in 0 1; do
    P2P_FP8_WGRAD=$w timeout -k 10 300 python bench.py --precision fp8 --steps 20 --warmup 5 > $O/bench_fp8_w$w.jsonl 2> $O/bench_fp8_w$w.err || exit $?
    cut -c1-200 $O/bench_fp8_w$w.jsonl
  done
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_bf16.jsonl 2> $O/bench_bf16.err || exit $?
cut -c1-200 $O/bench_bf16.jsonl
P2P_LIB=p2p_pytorch_amd/_C/exp_normfrag.so timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 256 --top 70 --json $O/census_normfrag.json > $O/census_normfrag.txt 2>&1 || exit $?
head -3 $O/census_normfrag.txt
timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 256 --top 70 --json $O/census_base.json > $O/census_base.txt 2>&1 || exit $?
head -3 $O/census_base.txt
mkdir -p $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --batch 256 --steps 5 --warmup 2 > $O/trace/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/trace/run_kernel_trace.csv --steps 5 --top 60 --width 160 > $O/trace/summary.txt
head -30 $O/trace/summary.txt
OUT=$O/roof bash tools/gpu_roofline.sh || exit $?

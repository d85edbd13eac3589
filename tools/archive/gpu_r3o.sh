#!/bin/bash
# Round-3 pass o: family R (reference compression GAN) after the VGG(real_b) reuse: tests,
# bench, and a kernel trace of the step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O/trace
timeout -k 10 400 python -u -m pytest tests/test_family_r_gpu.py tests/test_wgrad_stream_gpu.py -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'])"; }
timeout -k 10 300 python bench.py --family ref --batch 64 --steps 10 --warmup 3 > $O/ref.json 2>> $O/err.log || exit $?; echo "ref $(j $O/ref.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --family ref --batch 64 --steps 3 --warmup 2 > $O/trace/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/trace/run_kernel_trace.csv --steps 3 --top 70 --width 170 > $O/trace/summary.txt
head -60 $O/trace/summary.txt

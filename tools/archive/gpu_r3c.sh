#!/bin/bash
# Round-3 third pass: glds staging-rate probe, norm-in-fragment census A/B, kernel trace and
# calibrated counter roofline of the headline step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 120 ./tools/probes/bin/glds_rate_probe > $O/glds_rate.txt 2>&1 || exit $?
cat $O/glds_rate.txt
P2P_LIB=p2p_pytorch_amd/_C/exp_normfrag.so timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 256 --top 70 --json $O/census_normfrag.json > $O/census_normfrag.txt 2>&1 || exit $?
head -3 $O/census_normfrag.txt
timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 256 --top 70 --json $O/census_base.json > $O/census_base.txt 2>&1 || exit $?
head -3 $O/census_base.txt
mkdir -p $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --batch 256 --steps 5 --warmup 2 > $O/trace/log.txt 2>&1 || exit $?
python tools/prof_summary.py $O/trace/run_kernel_trace.csv --steps 5 --top 60 --width 160 > $O/trace/summary.txt
head -30 $O/trace/summary.txt
OUT=$O/roof bash tools/gpu_roofline.sh || exit $?

#!/bin/bash
# Round-3 first pass: counter calibration probe, full gpu test suite, smoke, default bench,
# per-layer conv census of the headline step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3a
export TMPDIR=/tmp
O=gpurun_out/r3a
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1
echo "counter list rc=$?"
timeout -k 10 60 ./tools/probes/bin/mfma_count_probe > $O/probe.txt 2>&1 || exit $?
cat $O/probe.txt
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d $O/probe_pmc -o run -- ./tools/probes/bin/mfma_count_probe > $O/probe_pmc.log 2>&1 || exit $?
echo probe pmc ok
timeout -k 10 60 ./tools/probes/bin/ds_read_tr_b8_probe > $O/tr_b8.txt 2>&1 || exit $?
head -3 $O/tr_b8.txt
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 240 --timeout-method thread > $O/kt.log 2>&1; rc=$?
echo "gpu tests rc=$rc: $(tail -1 $O/kt.log)"; grep -E "FAILED|ERROR" $O/kt.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 300 python bench.py > $O/bench_default.jsonl 2> $O/bench_default.err || exit $?
cut -c1-300 $O/bench_default.jsonl
timeout -k 10 600 python tools/conv_census.py --family pix2pix --batch 256 --top 60 --wgrad_variants P2P_WGRAD_TILE=256 --json $O/census_b256.json > $O/census_b256.txt 2>&1 || exit $?
head -70 $O/census_b256.txt
P2P_LIB=p2p_pytorch_amd/_C/exp_normfrag.so timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 256 --top 60 --json $O/census_b256_normfrag.json > $O/census_b256_normfrag.txt 2>&1 || exit $?
head -12 $O/census_b256_normfrag.txt

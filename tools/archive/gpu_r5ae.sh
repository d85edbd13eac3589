#!/bin/bash
# family-R fan-out (multi-consumer activation gradients summed by HIP adds): tests, aten census, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ae
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_family_r_gpu.py \
  tests/test_graph_family_r_gpu.py tests/test_cli_gpu.py tests/test_ddp_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PYTHONPATH=$PWD timeout -k 10 300 python -u tools/probes/aten_census.py --family ref --batch 8 > $O/aten_famr.txt 2>&1 || { tail -20 $O/aten_famr.txt; exit 1; }
grep -c "at::native" $O/aten_famr.txt; grep "op aten" $O/aten_famr.txt | head -20
timeout -k 10 300 python -u bench.py --family ref --batch 64 --steps 10 --warmup 3 > $O/famr.jsonl 2> $O/famr.err || { tail -20 $O/famr.err; exit 1; }
cut -c1-160 $O/famr.jsonl

#!/bin/bash
# full GPU suite of the current build, then family-R aten census + bench, headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5z
mkdir -p $O
rm -f gpurun_out/bounds.jsonl
timeout -k 10 1500 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > $O/suite.log 2>&1
rc=$?
echo "suite rc $rc: $(tail -1 $O/suite.log)"
grep -E "FAILED|ERROR|Segmentation|Fatal" $O/suite.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
PYTHONPATH=$PWD timeout -k 10 300 python -u tools/probes/aten_census.py --family ref --batch 8 > $O/aten_famr.txt 2>&1 || { tail -20 $O/aten_famr.txt; exit 1; }
tail -20 $O/aten_famr.txt
timeout -k 10 300 python -u bench.py --family ref --batch 64 --steps 10 --warmup 3 > $O/famr.jsonl 2> $O/famr.err || { tail -20 $O/famr.err; exit 1; }
cut -c1-160 $O/famr.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -1 $O/bench.jsonl | cut -c1-120
done

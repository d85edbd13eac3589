#!/bin/bash
# fp8 capture fix: the new capture test, the fp8 suite, then the fp8 bench (captured)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ac
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fp8_gpu.py > $O/fp8_tests.log 2>&1 || { tail -30 $O/fp8_tests.log; exit 1; }
tail -3 $O/fp8_tests.log
for b in 1024 2048; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --precision fp8 --batch $b > $O/f8_$b.json 2> $O/f8_$b.err || { tail -20 $O/f8_$b.err; exit 1; }
  echo "fp8 $b $(cut -c1-100 $O/f8_$b.json) $(grep -o '"hipgraph": [a-z]*' $O/f8_$b.json) $(grep -o '"capture_error": [^,]*' $O/f8_$b.json | cut -c1-200)"
done

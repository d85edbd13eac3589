#!/bin/bash
# Round-end rehearsal: the driver's smoke(), a default bench.py run (no flags) and the family-R
# bench with its default batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4smoke
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; grep "^{" $O/bench.json | tail -1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --family ref > $O/famr.json 2>> $O/bench.err; rc=$?
echo "famR default rc=$rc"; grep "^{" $O/famr.json | tail -1 | cut -c1-200
exit $rc

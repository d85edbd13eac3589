#!/bin/bash
# W5b: watchdog-drain fix -- minimal repro drained vs race; direct-gradient force_comm A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 120 python -u tools/diag_capture_event.py --mode drained > $O/cev_drained.txt 2>&1 || { tail -20 $O/cev_drained.txt; exit 1; }
tail -1 $O/cev_drained.txt
for d in 1 0 1; do
  P2P_DIRECT_GRAD=$d timeout -k 10 300 python -u bench.py --force_comm --steps 20 --warmup 5 >> $O/force_comm.jsonl 2> $O/fc_$d.err || { tail -20 $O/fc_$d.err; exit 1; }
  tail -1 $O/force_comm.jsonl | cut -c1-200
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $O/force_comm.jsonl 2> $O/plain.err || { tail -20 $O/plain.err; exit 1; }
tail -1 $O/force_comm.jsonl | cut -c1-200
timeout -k 10 900 python -u tools/diag_inner_grad.py --B 64 --seeds 11,12,13,14,15 --kinds fp32,eager,eager_f32x,native \
  > $O/diag_inner.txt 2>&1 || { tail -20 $O/diag_inner.txt; exit 1; }
tail -24 $O/diag_inner.txt
# last: the race (expected to abort if the hypothesis holds)
timeout -k 10 120 python -u tools/diag_capture_event.py --mode race > $O/cev_race.txt 2>&1
echo "race exit $?"
grep -m4 "round\|PASS\|capturing stream" $O/cev_race.txt
exit 0

#!/bin/bash
# W5b: the watchdog abort vs the c10d event cache; direct-gradient --force_comm A/B; W7 emulation
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
TORCH_NCCL_CUDA_EVENT_CACHE=0 timeout -k 10 120 python -u tools/diag_capture_event.py > $O/cev_off.txt 2>&1 || { tail -20 $O/cev_off.txt; exit 1; }
tail -2 $O/cev_off.txt
for d in 0 1; do
  TORCH_NCCL_CUDA_EVENT_CACHE=0 P2P_DIRECT_GRAD=$d timeout -k 10 300 python -u bench.py --force_comm --steps 20 --warmup 5 >> $O/force_comm.jsonl 2> $O/fc_$d.err || { tail -20 $O/fc_$d.err; exit 1; }
  tail -1 $O/force_comm.jsonl | cut -c1-200
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $O/force_comm.jsonl 2> $O/plain.err || { tail -20 $O/plain.err; exit 1; }
tail -1 $O/force_comm.jsonl | cut -c1-200
timeout -k 10 900 python -u tools/diag_inner_grad.py --B 64 --seeds 11,12,13,14,15 --kinds fp32,eager,eager_f32x,native \
  > $O/diag_inner.txt 2>&1 || { tail -20 $O/diag_inner.txt; exit 1; }
tail -24 $O/diag_inner.txt
# last: the default event cache (expected to abort if the hypothesis holds)
timeout -k 10 120 python -u tools/diag_capture_event.py > $O/cev_on.txt 2>&1
echo "cache-on exit $?"
grep -m3 "round\|PASS\|hipErrorCapturedEvent\|capturing stream" $O/cev_on.txt
exit 0

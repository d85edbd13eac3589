#!/bin/bash
# family-R step: capture + kernel census at B=64; W7 fp32-pre-norm emulation over 5 seeds;
# --force_comm with and without direct gradients
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 300 python -u bench.py --family ref --batch 64 --steps 10 --warmup 3 > $O/famr.jsonl 2> $O/famr.err || { tail -20 $O/famr.err; exit 1; }
cut -c1-400 $O/famr.jsonl
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python bench.py --family ref --batch 64 --steps 5 --warmup 2 > $O/prof_log.txt 2>&1 || { tail $O/prof_log.txt; exit 1; }
python tools/prof_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 60 --width 150 > $O/famr_kernels.txt
head -64 $O/famr_kernels.txt
rm -rf $O/prof
for d in 0 1; do
  P2P_DIRECT_GRAD=$d timeout -k 10 300 python -u bench.py --force_comm --steps 20 --warmup 5 >> $O/force_comm.jsonl 2> $O/fc_$d.err || { tail -20 $O/fc_$d.err; exit 1; }
  tail -1 $O/force_comm.jsonl | cut -c1-200
done
timeout -k 10 900 python -u tools/diag_inner_grad.py --B 64 --seeds 11,12,13,14,15 --kinds fp32,eager,eager_f32x,native \
  > $O/diag_inner.txt 2>&1 || { tail -20 $O/diag_inner.txt; exit 1; }
tail -16 $O/diag_inner.txt

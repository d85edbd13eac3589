#!/bin/bash
# final full GPU suite of the round-5 build; 2-rank rehearsal (gloo, one GPU) for both families; smoke(); headline bench
# direct gradients on by default since round 5) for both families; smoke(); headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ay
mkdir -p $O
rm -f gpurun_out/bounds.jsonl
timeout -k 10 1500 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > $O/suite.log 2>&1
rc=$?
echo "suite rc $rc: $(tail -1 $O/suite.log)"
grep -E "FAILED|ERROR|Segmentation|Fatal" $O/suite.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for fam in pix2pix ref; do
  P2P_DIST_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
    --batch 16 --family $fam > $O/dist_$fam.json 2> $O/dist_$fam.err || { tail -30 $O/dist_$fam.err; exit 1; }
  echo "dist $fam: $(grep '^{' $O/dist_$fam.json | tail -1 | cut -c1-200)"
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-160 $O/bench.jsonl

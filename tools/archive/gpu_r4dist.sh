#!/bin/bash
# bench.py's multi-rank path rehearsed on one GPU: 2 ranks over the gloo backend (graph capture
# off for gloo by design), small batch -- checks the launcher contract, the barrier /
# max-over-ranks timing and the single JSON line, not throughput.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4dist
mkdir -p $O
P2P_DIST_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
  --batch 32 > $O/b2.json 2> $O/b2.err; rc=$?
echo "rc=$rc"; grep "^{" $O/b2.json | tail -1 | cut -c1-400; [ $rc -eq 0 ] || tail -20 $O/b2.err
exit $rc

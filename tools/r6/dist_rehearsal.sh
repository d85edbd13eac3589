#!/bin/bash
# multi-rank rehearsal of the data-parallel path on ONE GPU: 2 ranks share the device, gloo
# collectives (the RCCL path at world 8 is the driver's); both model families
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6dist; mkdir -p $O
for fam in pix2pix ref; do
  P2P_DIST_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
    --batch 16 --family $fam > $O/dist_$fam.json 2> $O/dist_$fam.err || { tail -30 $O/dist_$fam.err; exit 1; }
  grep '^{' $O/dist_$fam.json | tail -1 >> $O/dist.jsonl
  echo "dist $fam: $(grep '^{' $O/dist_$fam.json | tail -1 | cut -c1-200)"
done
echo done

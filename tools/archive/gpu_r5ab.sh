#!/bin/bash
# same-box A/B: the committed build (libp2p_hip_head.so) vs the working tree's build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ab
mkdir -p $O
for r in 1 2; do
  for lib in head cur; do
    if [ $lib = head ]; then L=$PWD/p2p_pytorch_amd/_C/libp2p_hip_head.so; else L=$PWD/p2p_pytorch_amd/_C/libp2p_hip.so; fi
    P2P_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b_${lib}_$r.json 2> $O/b_${lib}_$r.err || { tail -20 $O/b_${lib}_$r.err; exit 1; }
    echo "$lib $r $(cut -c1-110 $O/b_${lib}_$r.json)"
  done
done
# family R captured at the verdict's B=64 and the default B=256; fp8 at its default batch
L=$PWD/p2p_pytorch_amd/_C/libp2p_hip.so
for cfg in "--family ref --batch 64" "--family ref --batch 256" "--precision fp8"; do
  tag=$(echo $cfg | tr -d ' -')
  P2P_LIB=$L timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 $cfg > $O/x_$tag.json 2> $O/x_$tag.err || { tail -20 $O/x_$tag.err; exit 1; }
  echo "$tag $(cut -c1-110 $O/x_$tag.json) $(grep -o '"hipgraph": [a-z]*' $O/x_$tag.json)"
done

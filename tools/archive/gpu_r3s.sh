#!/bin/bash
# Round-3 pass s: s2t B-prefetch distance 2 (exp_pd2.so) vs 1 on the layer micro-benchmark,
# then the headline at B = 1024 / 2048.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for m in convt dgrad; do
  timeout -k 10 120 python tools/s2t_layer.py --mode $m || exit $?
  P2P_LIB=p2p_pytorch_amd/_C/exp_pd2.so timeout -k 10 120 python tools/s2t_layer.py --mode $m || exit $?
done
for b in 1024 2048; do
  timeout -k 10 400 python bench.py --batch $b --steps 12 --warmup 3 > gpurun_out/bs_$b.json 2>>gpurun_out/bs.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bs_$b.json'));print($b, d['value'], d['ms_per_step'], d['max_mem_gib'])"
done

#!/bin/bash
# Round-3 pass n: 8-row operand prefetch in the EXT dgrad epilogue of the 256-row tiles:
# same-box A/B against the previous build (exp_base.so), census + bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_nb_fuse_gpu.py tests/test_production_shapes_gpu.py tests/test_s2t_gpu.py -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'])"; }
for r in 1 2; do
  P2P_LIB=p2p_pytorch_amd/_C/exp_base.so timeout -k 10 300 python bench.py --batch 256 > $O/base$r.json 2>> $O/err.log || exit $?; echo "base $(j $O/base$r.json)"
  timeout -k 10 300 python bench.py --batch 256 > $O/new$r.json 2>> $O/err.log || exit $?; echo "new $(j $O/new$r.json)"
done
timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 256 --top 70 > $O/census.txt 2>&1 || exit $?
grep -E " m1 " $O/census.txt | head -12

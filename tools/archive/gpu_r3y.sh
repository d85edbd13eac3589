#!/bin/bash
# Round-3 pass y: rowsum split over row chunks (the norm-partial column sums were one
# under-parallel pass: +1.2 ms at B=256) -- kernel tests, bias-gradient tests, benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3y
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_nb_fuse_gpu.py tests/test_production_shapes_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'])"; }
timeout -k 10 300 python bench.py --batch 256 > $O/bf256.json || exit 1; echo "bf16 b256 $(j $O/bf256.json)"
timeout -k 10 400 python bench.py > $O/bf1024.json || exit 1; echo "bf16 b1024 $(j $O/bf1024.json)"
timeout -k 10 400 python bench.py --precision fp8 > $O/f8_1024.json || exit 1; echo "fp8 b1024 $(j $O/f8_1024.json)"
timeout -k 10 300 python bench.py --batch 256 --precision fp8 > $O/f8_256.json || exit 1; echo "fp8 b256 $(j $O/f8_256.json)"

#!/bin/bash
# Round-3 pass u: fp8 class-shared halo kernel -- oracle / routing tests, then same-box fp8 and
# bf16 benches at B = 256 with the fp8 kernel on and off (P2P_NO_S2T=1 switches both off).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_s2t_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|s2t vs" $O/tests.log | tail -4
j() { python -c "import json;d=json.load(open('$1'));print(d['value'], d['ms_per_step'])"; }
timeout -k 10 300 python bench.py --batch 256 --precision fp8 > $O/f8.json || exit 1; echo "fp8 s2t  $(j $O/f8.json)"
P2P_NO_S2T=1 timeout -k 10 300 python bench.py --batch 256 --precision fp8 > $O/f8_nos2t.json || exit 1; echo "fp8 glds $(j $O/f8_nos2t.json)"
timeout -k 10 300 python bench.py --batch 256 > $O/bf.json || exit 1; echo "bf16     $(j $O/bf.json)"
timeout -k 10 300 python bench.py --batch 256 --precision fp8 > $O/f8b.json || exit 1; echo "fp8 s2t  $(j $O/f8b.json)"

#!/bin/bash
# Round-3 pass d: the prep/fire loader split (address math beside the MFMAs, glds interleaved):
# correctness of every conv path, then same-box A/B against the previous build (exp_base.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_fuzz_gpu.py tests/test_determinism_gpu.py tests/test_production_shapes_gpu.py tests/test_fp8_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for r in 1 2; do
  P2P_LIB=p2p_pytorch_amd/_C/exp_base.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/ab_base.jsonl 2>> $O/ab.err || exit $?
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/ab_new.jsonl 2>> $O/ab.err || exit $?
done
python - <<'PY'
import json
for t in ("base", "new"):
    v = [json.loads(l)["value"] for l in open(f"gpurun_out/r3d/ab_{t}.jsonl")]
    print(t, v)
PY
timeout -k 10 300 python bench.py --precision fp8 --steps 20 --warmup 5 > $O/bench_fp8.jsonl 2>> $O/ab.err || exit $?
cut -c1-160 $O/bench_fp8.jsonl
timeout -k 10 400 python tools/conv_census.py --family pix2pix --batch 256 --top 70 --json $O/census_new.json > $O/census_new.txt 2>&1 || exit $?
head -40 $O/census_new.txt

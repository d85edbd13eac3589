#!/bin/bash
# family-R PReLU slope self-consistency, s2t tests (normal build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
rm -f gpurun_out/bounds.jsonl
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_family_r_gpu.py tests/test_s2t_gpu.py > $O/tests2.log 2>&1 || { tail -30 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
python - <<'PY'
import json
for l in open("gpurun_out/bounds.jsonl"):
    r = json.loads(l)
    for row in r["rows"]:
        if "relu.weight" in str(row[0]):
            print(r["test"], row)
PY

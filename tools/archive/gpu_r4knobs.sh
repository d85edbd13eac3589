#!/bin/bash
# Round-4 knob sweep on the final build, headline B = 1024, one box (default bracketed).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4knobs
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1: stopping"; exit $1;; esac; }
j() { python - "$1" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"])
PY
}
run() { local tag=$1; shift; timeout -k 10 300 env "$@" python bench.py > $O/$tag.json 2>> $O/err.log; local rc=$?; fatal $rc; [ $rc -eq 0 ] || { echo "$tag FAILED rc=$rc"; return 1; }; echo "$tag $(j $O/$tag.json)"; grep "^{" $O/$tag.json | sed "s/^{/{\"tag\": \"$tag\", /" >> $O/all.jsonl; }
run default P2P_DUMMY=0 || exit 1
run nos2t P2P_NO_S2T=1
run w32 P2P_S2T_W32=1
run classmajor P2P_CLASS_MAJOR=1
run nowgradstream P2P_WGRAD_STREAM=0
run nonbfuse P2P_NB_FUSE=0
run g89 P2P_CONV_VARIANT=g89
run g6 P2P_CONV_VARIANT=g6
run default2 P2P_DUMMY=0
exit 0

#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 300 python -X faulthandler bench.py --steps 15 --warmup 4 --force_comm > $O/fc.json 2> $O/fc.err
echo "fc rc=$?"; tail -c 600 $O/fc.json; tail -5 $O/fc.err
timeout -k 10 300 python -X faulthandler bench.py --steps 15 --warmup 4 --force_comm --comm_dtype bf16 > $O/fcb.json 2> $O/fcb.err
echo "fcb rc=$?"; tail -c 600 $O/fcb.json; tail -5 $O/fcb.err

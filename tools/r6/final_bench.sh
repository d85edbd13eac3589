#!/bin/bash
# Round-6 final-build measurements: every BASELINE config the single GPU can run, plus
# inference, the reference family and the DP path at world 1.  One JSON line per run.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r6final}; mkdir -p $O
run() {  # tag args...
  local t=$1; shift
  timeout -k 10 500 python bench.py "$@" > $O/$t.out 2> $O/$t.err || { echo "$t failed rc=$?"; tail -5 $O/$t.err; return 1; }
  tail -1 $O/$t.out >> $O/bench_final.jsonl
  tail -1 $O/$t.out | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$t', d['value'], d['ms_per_step'], d['config']['hipgraph'], d['config']['capture_error'], d.get('max_mem_gib'))"
}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
run bf16_a || exit 1
run fp8_a --precision fp8 || exit 1
run bf16_b || exit 1
run fp8_b --precision fp8 || exit 1
run s512 --size 512 --batch 512 || exit 1
run infer_bf16 --mode infer || exit 1
run infer_fp8 --mode infer --precision fp8 || exit 1
run famr_b64 --family ref --batch 64 || exit 1
run famr_b512 --family ref || exit 1
run fc_bf16 --force_comm --comm_dtype bf16 || exit 1
run s512_fp8 --size 512 --batch 512 --precision fp8 || exit 1
run eager_b128 --impl torch --batch 128 --steps 10 --warmup 3 || echo "eager baseline failed (not fatal)"
echo done

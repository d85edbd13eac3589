cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && rm -f gpurun_out/bounds.jsonl
timeout -k 10 300 python tools/diag_graph.py > gpurun_out/diag_graph.jsonl 2> gpurun_out/diag.err; echo diag rc=$?
cat gpurun_out/diag_graph.jsonl
DROP=0 timeout -k 10 300 python tools/diag_graph.py > gpurun_out/diag_graph_nodrop.jsonl 2>> gpurun_out/diag.err; echo diag2 rc=$?
cat gpurun_out/diag_graph_nodrop.jsonl
timeout -k 10 400 python -u -m pytest tests/test_family_r_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/famr.log 2>&1; echo famr rc=$?; tail -3 gpurun_out/famr.log

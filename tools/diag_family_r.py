"""Diag: family-R G-gradient error vs fp32 -- run-to-run spread (rows -> gpurun_out/fr_rows.json)."""
import json
import sys
sys.path[:0] = [".", "tests"]
import test_kernels_gpu as T

rows = []
T._record = lambda name, r: rows.append(r)
for rep in range(6):
    try:
        T.test_family_r_networks_match_oracle()
        print(rep, "PASS", flush=True)
    except AssertionError as e:
        print(rep, "FAIL", str(e)[:200], flush=True)
json.dump(rows, open("gpurun_out/fr_rows.json", "w"))

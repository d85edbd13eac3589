"""Host-side sanitizer run: the __host__ __device__ index helpers of
csrc/common.h (FastDiv, xcd_remap, reflect_idx) built with ASan + UBSan on the host pass
(GPU sanitizers are not available on this pool) and checked exhaustively / by sampling."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_host_index_math_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_checks"
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "--offload-arch=gfx950",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined",
           f"-I{os.path.join(ROOT, 'csrc')}", os.path.join(ROOT, "tests", "native", "host_checks.cpp"),
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]

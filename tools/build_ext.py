#!/usr/bin/env python
"""Build the in-tree HIP/CDNA4 extension ``p2p_pytorch_amd/_C/libp2p_hip.so``.

Plain hipcc, no hipify and no JIT cache: every ``csrc/*.hip`` is compiled for gfx950
only (``--offload-arch=gfx950``), ``csrc/bindings.cpp`` against the PyTorch headers, and
everything is linked into one shared library that ``torch.ops.load_library`` registers as
``torch.ops.p2p``.  Objects are rebuilt only when a source or header changed (content
hash), so a no-op build takes well under a second.  The .so travels with the repository
snapshot to the GPU box.

    python tools/build_ext.py [--jobs N] [--force] [--verbose]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "hip")
OUT_DIR = os.path.join(ROOT, "p2p_pytorch_amd", "_C")
OUT = os.path.join(OUT_DIR, "libp2p_hip.so")
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _headers_hash():
    h = hashlib.sha256()
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".h"):
            with open(os.path.join(CSRC, f), "rb") as fh:
                h.update(f.encode() + fh.read())
    return h.hexdigest()


def _compile(src, flags, hh, force, verbose):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    stamp = obj + ".sha"
    with open(src, "rb") as fh:
        digest = hashlib.sha256(fh.read() + hh.encode() + " ".join(flags).encode()).hexdigest()
    if not force and os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == digest:
                return obj, False
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip() and verbose:
        print(r.stderr, file=sys.stderr)
    with open(stamp, "w") as fh:
        fh.write(digest)
    return obj, True


def build(jobs: int = 8, force: bool = False, verbose: bool = False, defines=(), out: str | None = None) -> str:
    """defines: extra -D macros (kernel experiments); out: alternative .so path (objects
    go to their own build dir), loaded with P2P_LIB=<path>."""
    global BUILD, OUT
    if out:
        tag = hashlib.sha256(" ".join(defines).encode()).hexdigest()[:8]
        BUILD = os.path.join(ROOT, "build", "hip_" + tag)
        OUT = os.path.abspath(out)
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    inc, lib, abi = _torch_paths()
    hh = _headers_hash()
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", "-Wno-unused-result"] + [f"-D{d}" for d in defines]
    hip_flags = common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
    cpp_flags = common + [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
                          "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=p2p_hip",
                          f"-I{sysconfig.get_paths()['include']}"] + [f"-I{p}" for p in inc]
    jobs_list = []
    for f in sorted(os.listdir(CSRC)):
        path = os.path.join(CSRC, f)
        if f.endswith(".hip"):
            jobs_list.append((path, hip_flags))
        elif f.endswith(".cpp"):
            jobs_list.append((path, cpp_flags))
    objs, changed = [], False
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(_compile, s, fl, hh, force, verbose) for s, fl in jobs_list]
        for fu in futs:
            o, c = fu.result()
            objs.append(o)
            changed |= c
    if changed or force or not os.path.exists(OUT):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT + ".tmp"] + objs + [
            f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch",
            f"-Wl,-rpath,{lib}"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        # a kernel whose host launch stub hipcc silently dropped links fine and only fails at
        # dlopen (undefined __device_stub__ symbol): refuse such a library here
        nm = subprocess.run(["nm", "-u", "-C", OUT + ".tmp"], capture_output=True, text=True)
        bad = [ln.strip() for ln in nm.stdout.splitlines() if "__device_stub__" in ln or "p2p::" in ln]
        if bad:
            raise RuntimeError("undefined kernel symbols in the linked library:\n" + "\n".join(bad[:20]))
        os.replace(OUT + ".tmp", OUT)
    return OUT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--define", action="append", default=[], help="extra -D macro (repeatable)")
    ap.add_argument("--out", default=None, help="alternative output .so (load with P2P_LIB)")
    a = ap.parse_args()
    print(build(a.jobs, a.force, a.verbose, a.define, a.out))


if __name__ == "__main__":
    main()

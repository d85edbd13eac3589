"""bench.py's driver contract on CPU (BASELINE config 1: 64x64, 4-level U-Net + pixel PatchGAN).

The driver runs ``python bench.py --gpus N --steps K --warmup W`` (N > 1 under
``torch.distributed.run``) and parses ONE JSON line from rank 0 with a fixed key set; the
multi-rank value is the whole-job aggregate over the slowest rank.  Both launch shapes are
exercised here on the CPU plumbing config (gloo for 2 ranks, 127.0.0.1 rendezvous).
"""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}
ARGS = ["--size", "64", "--netG", "unet_4", "--netD", "pixel", "--batch", "1", "--steps", "2", "--warmup", "1"]


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_bench_single_process_json_line():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1"] + ARGS, cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert KEYS <= set(d), KEYS - set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert abs(d["value"] - d["config"]["global_batch"] * 1000.0 / d["ms_per_step"]) <= 0.02 * d["value"]
    assert d["config"]["parallelism"] == "dp1"


def test_bench_two_ranks_one_json_line():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2"] + ARGS,
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout        # rank 0 only
    d = lines[0]
    assert KEYS <= set(d)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 2 * d["config"]["per_gpu_batch"]   # weak scaling: per-GPU work fixed
    assert d["scaling"] == "weak"

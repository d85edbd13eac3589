"""Checkpoint save / resume (reference train.py:103-121, :504-528; test.py:21-23).

Reference-compatible schema: ``checkpoint/<dataset>/net_<name>_
epoch_<epoch>.pth`` holding ``{'epoch': epoch + 1, 'state_dict_g': G.state_dict(),
'state_dict_c': C.state_dict()}`` with fp32 tensors and the reference key names, so a
generator trained here loads into the reference ``ExpandNetwork`` and vice versa.

Fixed on top (reference quirk A4: its resume reads keys it never writes): the same file
additionally carries ``state_dict_d``, ``optimizer_g/d``, ``scheduler_g/d``,
``losslogger``, the device-side optimizer step counters and the RNG states, so
``--epoch_count N`` really resumes.  Writes are atomic (tmp file + rename) and done by
rank 0 only; every rank loads.  Loading uses ``weights_only=True`` -- these files contain
tensors, numbers and lists only.
"""
from __future__ import annotations

import glob
import os
import re

import torch


def checkpoint_path(root, dataset, name, epoch):
    return os.path.join(root, dataset, f"net_{name}_epoch_{epoch}.pth")


def _cpu_state(module):
    return {k: v.detach().to("cpu", copy=True) for k, v in module.state_dict().items()}


def save_checkpoint(path, epoch, net_g, net_c=None, net_d=None, opt_g=None, opt_d=None,
                    sched_g=None, sched_d=None, losslogger=None, extra=None, rank=0,
                    opt_c=None, sched_c=None):
    """Write the reference dict (+ full-resume keys) atomically; no-op on ranks != 0."""
    if rank != 0:
        return None
    state = {"epoch": int(epoch) + 1, "state_dict_g": _cpu_state(net_g)}
    if net_c is not None:
        state["state_dict_c"] = _cpu_state(net_c)
    if net_d is not None:
        state["state_dict_d"] = _cpu_state(net_d)
    if opt_g is not None:
        state["optimizer_g"] = opt_g.state_dict()
    if opt_d is not None:
        state["optimizer_d"] = opt_d.state_dict()
    if sched_g is not None:
        state["scheduler_g"] = sched_g.state_dict()
    if sched_d is not None:
        state["scheduler_d"] = sched_d.state_dict()
    if opt_c is not None:
        state["optimizer_c"] = opt_c.state_dict()
    if sched_c is not None:
        state["scheduler_c"] = sched_c.state_dict()
    state["losslogger"] = list(losslogger or [])
    state["rng_cpu"] = torch.get_rng_state()
    if torch.cuda.is_available():
        state["rng_cuda"] = torch.cuda.get_rng_state()
    if extra:
        state.update(extra)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def _move_optimizer_state(opt, device):
    for st in opt.state.values():
        for k, v in st.items():
            if isinstance(v, torch.Tensor) and k != "step":
                st[k] = v.to(device)


def has_scheduler_state(path) -> bool:
    """True when ``path`` carries scheduler state (a file written here, not by the reference)."""
    return "scheduler_g" in torch.load(path, map_location="cpu", weights_only=True, mmap=True)


def scheduler_offset(path):
    """The ``epoch_count`` offset the saved schedulers' lambda was built with (the run that
    wrote the file records it as ``sched_epoch_count``; files from before that default to
    1), or None when ``path`` carries no scheduler state (a reference-written file)."""
    state = torch.load(path, map_location="cpu", weights_only=True, mmap=True)
    if "scheduler_g" not in state:
        return None
    return int(state.get("sched_epoch_count", 1))


def load_checkpoint(path, net_g=None, net_c=None, net_d=None, opt_g=None, opt_d=None,
                    sched_g=None, sched_d=None, device=None, strict=True, opt_c=None,
                    sched_c=None):
    """Restore whatever the file holds; returns (start_epoch, losslogger).

    A reference-written file (epoch + G + C only) restores the networks and the epoch;
    optimizer / scheduler / D state come back only from files written here."""
    state = torch.load(path, map_location="cpu", weights_only=True)
    if net_g is not None:
        net_g.load_state_dict(state["state_dict_g"], strict=strict)
    if net_c is not None and "state_dict_c" in state:
        net_c.load_state_dict(state["state_dict_c"], strict=strict)
    if net_d is not None and "state_dict_d" in state:
        net_d.load_state_dict(state["state_dict_d"], strict=strict)
    for opt, key in ((opt_g, "optimizer_g"), (opt_d, "optimizer_d"), (opt_c, "optimizer_c")):
        if opt is not None and key in state:
            opt.load_state_dict(state[key])
            if device is not None:
                _move_optimizer_state(opt, device)
    for sch, key in ((sched_g, "scheduler_g"), (sched_d, "scheduler_d"), (sched_c, "scheduler_c")):
        if sch is not None and key in state:
            sch.load_state_dict(state[key])
    if "rng_cpu" in state:
        torch.set_rng_state(state["rng_cpu"])
    if "rng_cuda" in state and torch.cuda.is_available():
        try:
            torch.cuda.set_rng_state(state["rng_cuda"])
        except RuntimeError:
            pass
    return int(state.get("epoch", 1)), list(state.get("losslogger", []))


def latest_checkpoint(root, dataset, name):
    """Path and epoch of the newest ``net_<name>_epoch_<N>.pth``, or (None, 0)."""
    pat = os.path.join(root, dataset, f"net_{name}_epoch_*.pth")
    best, best_ep = None, 0
    for p in glob.glob(pat):
        m = re.search(r"_epoch_(\d+)\.pth$", p)
        if m and int(m.group(1)) > best_ep:
            best, best_ep = p, int(m.group(1))
    return best, best_ep


def load_generator(path, net_g, device=None, allow_pickle=False):
    """test.py loader: the dict form (``state_dict_g``) or a bare state dict; a legacy
    whole-module pickle (what the reference test.py expects, quirk A5) only with
    ``allow_pickle=True`` -- it executes code from the file."""
    try:
        state = torch.load(path, map_location="cpu", weights_only=True)
    except Exception:
        if not allow_pickle:
            raise RuntimeError(
                f"{path} is not a tensor-only checkpoint (legacy pickled module?); pass "
                "--allow_pickle to load it (this runs code stored in the file)")
        module = torch.load(path, map_location="cpu", weights_only=False)
        state = module.state_dict()
    if isinstance(state, dict) and "state_dict_g" in state:
        state = state["state_dict_g"]
    net_g.load_state_dict(state)
    if device is not None:
        net_g.to(device)
    return net_g

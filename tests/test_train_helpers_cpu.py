"""The reference train.py's module-level helpers are importable from our train.py with the
same names, signatures and semantics (/root/reference/train.py:33-126), and a resumed run
follows the same learning-rate schedule as an uninterrupted one."""
import json
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_reference_helpers_importable_from_train():
    from train import (calc_c_loss, calc_Gram_Loss, calc_tv_Loss, extract_features, gram,
                       load_checkpoint, psnr, ssim, tensor2img, tensor2np)
    x = torch.rand(1, 3, 16, 16)
    arr = tensor2np(x)
    assert arr.shape == (16, 16, 3) and arr.dtype == np.uint8
    assert tensor2img(x).size == (16, 16)
    assert psnr(x, x) == float("inf")
    y = (x + 0.05).clamp(0, 1)
    a = np.asarray(tensor2np(x), dtype=float)
    b = np.asarray(tensor2np(y), dtype=float)
    assert psnr(x, y) == pytest.approx(10 * np.log10(255 ** 2 / np.mean((a - b) ** 2)), rel=1e-5)
    assert ssim(x, x) == pytest.approx(1.0)
    assert ssim(y, x) < 1.0
    f = torch.rand(2, 4, 5, 5)
    g = gram(f)
    assert g.shape == (2, 4, 4)
    assert torch.allclose(g, torch.bmm(f.view(2, 4, 25), f.view(2, 4, 25).transpose(1, 2)) / 25)
    assert float(calc_Gram_Loss([f], [f])) == 0.0
    assert float(calc_c_loss([f, f], [f, f + 1])) == pytest.approx(0.5)
    tv = calc_tv_Loss(x)
    ref = (x[:, :, :, :-1] - x[:, :, :, 1:]).abs().mean() + (x[:, :, :-1] - x[:, :, 1:]).abs().mean()
    assert float(tv) == pytest.approx(float(ref), rel=1e-6)
    model = [torch.nn.Conv2d(3, 4, 3), torch.nn.ReLU(), torch.nn.Conv2d(4, 4, 3)]
    feats = extract_features(model, x, [1, 2])
    assert [t.shape[1] for t in feats] == [4, 4]
    with pytest.raises(SystemExit):
        load_checkpoint(None, None, None, None, None, None, [], "/nonexistent/ckpt.pth")


def _lrs(path):
    out = {}
    with open(path) as f:
        for line in f:
            d = json.loads(line)
            if "lr_g" in d:
                out[d["epoch"]] = d["lr_g"]
    return out


def test_resume_follows_uninterrupted_lr_schedule(tmp_path, monkeypatch):
    """a resumed LambdaLR must not count --epoch_count twice."""
    monkeypatch.chdir(tmp_path)
    import train
    common = ["--synthetic", "--image_size", "32", "--netG", "unet_4", "--netD", "pixel",
              "--ngf", "8", "--ndf", "8", "--steps_per_epoch", "1", "--epochsave", "1",
              "--niter", "1", "--niter_decay", "4", "--no_eval", "--log_every", "1"]
    train.main(common + ["--name", "full", "--nepoch", "4", "--log_json", "full.jsonl"])
    train.main(common + ["--name", "part", "--nepoch", "2", "--log_json", "part.jsonl"])
    train.main(common + ["--name", "part", "--nepoch", "4", "--epoch_count", "3",
                         "--log_json", "part.jsonl"])
    full, part = _lrs("full.jsonl"), _lrs("part.jsonl")
    assert sorted(full) == sorted(part) == [1, 2, 3, 4]
    for e in full:
        assert part[e] == pytest.approx(full[e]), (e, full, part)
    assert full[4] < full[1]          # the schedule really decays inside this window


def _rewrite(path, keep=None, drop=()):
    """Rewrite a checkpoint written by this test (own file: safe loader, tensors only)."""
    st = torch.load(path, map_location="cpu", weights_only=True)
    if keep is not None:
        st = {k: v for k, v in st.items() if k in keep}
    for k in drop:
        st.pop(k, None)
    torch.save(st, path)


@pytest.mark.parametrize("variant", ["offset_chain", "no_offset_key", "reference_file"])
def test_resume_keeps_scheduler_offset(tmp_path, monkeypatch, variant):
    """the saved scheduler offset (sched_epoch_count) survives a chain of resumes.

    * offset_chain: 1-2, then ``--epoch_count 3`` to 4 (its file records offset 1, not 3),
      then ``--resume`` to 6 -- the LR of every epoch equals the uninterrupted 1-6 run's;
    * no_offset_key: the epoch-2 file loses ``sched_epoch_count`` (a file from before the
      key existed): the restored scheduler defaults to offset 1;
    * reference_file: the epoch-2 file keeps only the reference's keys (epoch, G, C): a
      fresh scheduler offset by ``--epoch_count`` (the reference's rule) lands on the same LRs.
    """
    monkeypatch.chdir(tmp_path)
    import train
    common = ["--synthetic", "--image_size", "32", "--netG", "unet_4", "--netD", "pixel",
              "--ngf", "8", "--ndf", "8", "--steps_per_epoch", "1", "--epochsave", "1",
              "--niter", "1", "--niter_decay", "6", "--no_eval", "--log_every", "1"]
    train.main(common + ["--name", "full", "--nepoch", "6", "--log_json", "full.jsonl"])
    train.main(common + ["--name", "part", "--nepoch", "2", "--log_json", "part.jsonl"])
    ck2 = os.path.join("checkpoint", "synthetic", "net_part_epoch_2.pth")
    if variant == "no_offset_key":
        _rewrite(ck2, drop=("sched_epoch_count",))
    elif variant == "reference_file":
        _rewrite(ck2, keep=("epoch", "state_dict_g", "state_dict_c"))
    train.main(common + ["--name", "part", "--nepoch", "4", "--epoch_count", "3",
                         "--log_json", "part.jsonl"])
    from p2p_pytorch_amd.engine.checkpoint import scheduler_offset
    assert scheduler_offset(os.path.join("checkpoint", "synthetic", "net_part_epoch_4.pth")) == \
        (3 if variant == "reference_file" else 1)
    train.main(common + ["--name", "part", "--nepoch", "6", "--resume", "--log_json", "part.jsonl"])
    full, part = _lrs("full.jsonl"), _lrs("part.jsonl")
    assert sorted(full) == sorted(part) == [1, 2, 3, 4, 5, 6]
    for e in full:
        assert part[e] == pytest.approx(full[e]), (variant, e, full, part)
    assert full[6] < full[3] < full[1]

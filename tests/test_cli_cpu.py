"""End-to-end CLI plumbing on CPU (BASELINE config 1 and the reference family):
generate_dataset.py -> train.py (checkpoint) -> resume -> test.py, in a temp directory."""
import os
import sys

import numpy as np
import pytest
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture()
def workdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(0)
    src = tmp_path / "src"
    src.mkdir()
    for i in range(2):
        arr = (rng.random((64, 96, 3)) * 255).astype(np.uint8)
        Image.fromarray(arr).save(src / f"img.{i}.png")   # multi-dot name (quirk fix)
    import generate_dataset
    for split in ("train", "test"):
        n = generate_dataset.cli(["--target_dataset_folder", f"dataset/toy/{split}",
                                  "--dataset_path", str(src), "--crop_size", "32",
                                  "--max_patches", "2", "--bit_size", "3"])
        assert n == 4
    return tmp_path


def test_generate_dataset_quantises(workdir):
    a = np.asarray(Image.open(workdir / "dataset/toy/train/a/img.0_0.png"))
    b = np.asarray(Image.open(workdir / "dataset/toy/train/b/img.0_0.png"))
    assert a.shape == b.shape == (32, 32, 3)
    levels = np.unique(b)
    assert len(levels) <= 8                  # 3-bit quantised copy
    assert np.abs(a.astype(int) - b.astype(int)).max() <= 255 // 14 + 1


def test_train_resume_test_reference_family(workdir):
    import train
    import test as test_cli
    train.main(["--dataset", "toy", "--name", "r", "--nepoch", "1", "--epochsave", "1",
                "--log_every", "2", "--threads", "0"])
    ck = workdir / "checkpoint/toy/net_r_epoch_1.pth"
    assert ck.exists()
    state = torch.load(ck, weights_only=True)
    assert state["epoch"] == 2
    assert len(state["state_dict_g"]) == 169 and "relu.weight" in state["state_dict_g"]
    assert "state_dict_c" in state and "optimizer_g" in state and "state_dict_d" in state
    # resume at epoch 2 from the full-resume keys (the reference raises KeyError here)
    train.main(["--dataset", "toy", "--name", "r", "--nepoch", "2", "--epochsave", "1",
                "--epoch_count", "2", "--log_every", "2", "--threads", "0", "--no_eval"])
    assert (workdir / "checkpoint/toy/net_r_epoch_2.pth").exists()
    n = test_cli.main(["--dataset", "toy", "--name", "r", "--nepochs", "2", "--image_size", "32",
                       "--with_compress"])
    assert n == 4 and len(os.listdir(workdir / "result/toy")) == 4


def test_train_pix2pix_plumbing_config(workdir):
    import train
    import test as test_cli
    train.main(["--dataset", "toy", "--name", "p", "--netG", "unet_4", "--netD", "pixel",
                "--nepoch", "1", "--epochsave", "1", "--threads", "0", "--lamb", "100"])
    n = test_cli.main(["--dataset", "toy", "--name", "p", "--nepochs", "1", "--netG", "unet_4",
                       "--image_size", "64"])
    assert n == 4

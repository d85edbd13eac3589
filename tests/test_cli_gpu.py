"""End-to-end CLI on the MI355X (native HIP path): generate_dataset.py -> train.py with
checkpoint -> resume -> test.py, for the pix2pix family (U-Net-256 + PatchGAN at 256x256,
bf16, hipGraph-captured steps, fp8 conv path) and the reference family."""
import os
import sys

import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture()
def workdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(0)
    src = tmp_path / "src"
    src.mkdir()
    for i in range(2):
        Image.fromarray((rng.random((256, 512, 3)) * 255).astype(np.uint8)).save(src / f"img{i}.png")
    import generate_dataset
    for split in ("train", "test"):
        generate_dataset.cli(["--target_dataset_folder", f"dataset/toy/{split}", "--dataset_path", str(src),
                              "--crop_size", "256", "--max_patches", "2"])
    return tmp_path


@pytest.mark.parametrize("extra", [[], ["--graph"], ["--precision", "fp8"]], ids=["eager", "graph", "fp8"])
def test_train_resume_test_pix2pix_gpu(workdir, extra):
    import train
    import test as test_cli
    import p2p_pytorch_amd as p2p
    try:
        base = ["--dataset", "toy", "--name", "g", "--netG", "unet_256", "--netD", "basic", "--cuda",
                "--batch_size", "2", "--lamb", "100", "--threads", "0", "--epochsave", "1", "--device_cache",
                "--log_json", "m.jsonl"] + extra
        train.main(base + ["--nepoch", "1"])
        import json
        recs = [r for r in (json.loads(l) for l in open(workdir / "m.jsonl")) if "img_s" in r]
        assert recs and all(r["img_s"] > 0 for r in recs)
        if "--graph" not in extra:   # per-phase HIP-event ms in the JSONL stream
            assert set(recs[-1]["phase_ms"]) >= {"G_fwd", "D_fwd", "D_bwd_opt", "G_bwd_opt"}
        ck = workdir / "checkpoint/toy/net_g_epoch_1.pth"
        assert ck.exists()
        st = torch.load(ck, weights_only=True)
        assert all(torch.isfinite(v).all() for v in st["state_dict_g"].values() if v.is_floating_point())
        train.main(base + ["--nepoch", "2", "--epoch_count", "2", "--no_eval"])
        assert (workdir / "checkpoint/toy/net_g_epoch_2.pth").exists()
        n = test_cli.main(["--dataset", "toy", "--name", "g", "--nepochs", "2", "--netG", "unet_256", "--cuda"])
        assert n == 4 and len(os.listdir(workdir / "result/toy")) == 4
    finally:
        p2p.set_precision("bf16")


def test_train_reference_family_gpu(workdir):
    import train
    train.main(["--dataset", "toy", "--name", "r", "--cuda", "--nepoch", "1", "--epochsave", "1",
                "--threads", "0", "--batch_size", "2"])
    st = torch.load(workdir / "checkpoint/toy/net_r_epoch_1.pth", weights_only=True)
    assert len(st["state_dict_g"]) == 169
    assert all(torch.isfinite(v).all() for v in st["state_dict_g"].values() if v.is_floating_point())

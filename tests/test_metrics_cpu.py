"""Device PSNR / SSIM vs an independent numpy/scipy transcription of the reference path
(train.py:54-65: tensor2img -> float arrays -> skimage structural_similarity with
multichannel=True; skimage is not installed, so its algorithm -- scipy uniform_filter,
7x7, sample covariance, crop (win-1)/2, float data_range 2.0 -- is re-implemented here)."""
import numpy as np
import torch
from scipy.ndimage import uniform_filter

from p2p_pytorch_amd.data.image_io import tensor2np
from p2p_pytorch_amd.engine.metrics import psnr, ssim


def _skimage_ssim(x, y, data_range=2.0, win=7):
    x = x.astype(np.float64)
    y = y.astype(np.float64)
    vals = []
    for ch in range(x.shape[2]):
        a, b = x[..., ch], y[..., ch]
        ux, uy = uniform_filter(a, win), uniform_filter(b, win)
        uxx, uyy, uxy = uniform_filter(a * a, win), uniform_filter(b * b, win), uniform_filter(a * b, win)
        cov = win * win / (win * win - 1.0)
        vx, vy, vxy = cov * (uxx - ux * ux), cov * (uyy - uy * uy), cov * (uxy - ux * uy)
        C1, C2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
        S = ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux ** 2 + uy ** 2 + C1) * (vx + vy + C2))
        pad = (win - 1) // 2
        vals.append(S[pad:-pad, pad:-pad].mean())
    return float(np.mean(vals))


def test_psnr_ssim_reference_semantics():
    g = torch.Generator().manual_seed(0)
    t = torch.rand(3, 3, 40, 40, generator=g) * 2 - 1
    p = (t + 0.2 * torch.randn(3, 3, 40, 40, generator=g)).clamp(-1, 1)
    ps, ss = psnr(t, p), ssim(p, t)
    for i in range(3):
        a = tensor2np(t[i:i + 1]).astype(float)
        b = tensor2np(p[i:i + 1]).astype(float)
        ref_psnr = 10 * np.log10(255 ** 2 / np.mean((a - b) ** 2))
        assert abs(ps[i].item() - ref_psnr) < 1e-3
        assert abs(ss[i].item() - _skimage_ssim(b, a)) < 1e-5


def test_ssim_identity_and_corrected_mode():
    x = torch.rand(2, 3, 16, 16) * 2 - 1
    assert torch.allclose(ssim(x, x), torch.ones(2))
    assert torch.isinf(psnr(x, x)).all()
    y = (x + 0.1).clamp(-1, 1)
    s = ssim(y, x, ref_compat=False)
    assert 0.0 < s.min() <= 1.0


def test_reference_instance_norm_channels_last_n1():
    """The CPU oracle must not inherit PyTorch's channels_last N==1 instance_norm backward
    bug: its gradient equals the NCHW-contiguous one."""
    import torch
    from p2p_pytorch_amd.ops import reference as ref
    torch.manual_seed(0)
    x = torch.randn(1, 8, 4, 4) * 2 + 1
    gy = torch.randn(1, 8, 4, 4)
    grads = []
    for cl in (False, True):
        xx = (x.contiguous(memory_format=torch.channels_last) if cl else x.clone()).requires_grad_(True)
        ref.instance_norm(xx).backward(gy)
        grads.append(xx.grad)
    assert torch.allclose(grads[0], grads[1], atol=1e-5)

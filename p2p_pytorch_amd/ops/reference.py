"""Pure-PyTorch oracle implementations of every fused op.

These run on CPU (the 64x64 plumbing config, unit-test oracles) and are what the
``P2P_BACKEND=torch`` eager *baseline* uses on the GPU.  The HIP kernels in ``csrc/``
implement exactly these semantics; ``tests/test_kernels_gpu.py`` compares the two.

Conventions shared with the kernels:
  * ``act`` names: None | 'relu' | 'lrelu' (slope 0.2) | 'tanh' | 'sigmoid'.
  * A conv input given as a tuple ``(a, b)`` is a *virtual concat* along channels
    (the U-Net skip concat, reference pix2pix template ``cat([x, model(x)], 1)``).
  * ``act_in`` is applied to the (virtually concatenated) input *before* padding, so
    zero padding stays zero in the activated domain.
  * ``upsample`` is a nearest-neighbour factor applied before padding
    (reference ``UpsampleConvLayer``, /root/reference/networks.py:408-423).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

LRELU_SLOPE = 0.2


def apply_act(x: torch.Tensor, act: str | None, slope: float = LRELU_SLOPE) -> torch.Tensor:
    if act is None or act == "none":
        return x
    if act == "relu":
        return F.relu(x)
    if act == "lrelu":
        return F.leaky_relu(x, slope)
    if act == "tanh":
        return torch.tanh(x)
    if act == "sigmoid":
        return torch.sigmoid(x)
    raise ValueError(f"unknown activation {act!r}")


def _cat(x):
    if isinstance(x, (tuple, list)):
        return torch.cat(list(x), 1)
    return x


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def conv2d(x, weight, bias=None, stride=1, padding=0, pad_mode="zeros", upsample=1,
           act_in=None, act_out=None):
    x = apply_act(_cat(x), act_in)
    if upsample and upsample > 1:
        x = F.interpolate(x, scale_factor=upsample, mode="nearest")
    ph, pw = _pair(padding)
    if pad_mode == "reflect" and (ph or pw):
        x = F.pad(x, (pw, pw, ph, ph), mode="reflect")
        ph = pw = 0
    y = F.conv2d(x, weight.to(x.dtype), None if bias is None else bias.to(x.dtype),
                 stride=stride, padding=(ph, pw))
    return apply_act(y, act_out)


def conv_transpose2d(x, weight, bias=None, stride=2, padding=1, act_in=None, act_out=None,
                     output_padding=0):
    x = apply_act(_cat(x), act_in)
    y = F.conv_transpose2d(x, weight.to(x.dtype), None if bias is None else bias.to(x.dtype),
                           stride=stride, padding=padding, output_padding=output_padding)
    return apply_act(y, act_out)


def instance_norm(x, eps=1e-5, act=None, weight=None, bias=None):
    # PyTorch 2.10's CPU instance_norm returns a wrong input gradient for channels_last
    # inputs with N == 1 (found by tests/test_norm_fuzz_gpu.py): go NCHW there only (the
    # GPU eager baseline keeps its channels_last layout)
    if not x.is_cuda and x.shape[0] == 1:
        x = x.contiguous()
    y = F.instance_norm(x, weight=weight, bias=bias, eps=eps)
    return apply_act(y, act)


def batch_norm(x, running_mean, running_var, weight, bias, training, momentum=0.1, eps=1e-5,
               act=None):
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    return apply_act(y, act)


def prelu(x, weight):
    return F.prelu(x, weight)


def dropout(x, p, training):
    return F.dropout(x, p, training)


# ---------------------------------------------------------------- losses
def mse_const(pred: torch.Tensor, target: float) -> torch.Tensor:
    """MSE against a constant label without materialising the target tensor."""
    return torch.mean((pred.float() - target) ** 2)


def bce_logits_const(pred: torch.Tensor, target: float) -> torch.Tensor:
    return F.binary_cross_entropy_with_logits(pred.float(), torch.full_like(pred.float(), target))


def bce_const(prob: torch.Tensor, target: float) -> torch.Tensor:
    return F.binary_cross_entropy(prob.float(), torch.full_like(prob.float(), target))


def l1(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return torch.mean(torch.abs(a.float() - b.float()))


def mse(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return torch.mean((a.float() - b.float()) ** 2)


def tv(x: torch.Tensor) -> torch.Tensor:
    """Anisotropic TV (reference ``calc_tv_Loss``, /root/reference/train.py:123-126)."""
    x = x.float()
    return (torch.mean(torch.abs(x[:, :, :, :-1] - x[:, :, :, 1:]))
            + torch.mean(torch.abs(x[:, :, :-1, :] - x[:, :, 1:, :])))


def quantize(x: torch.Tensor, bits: int) -> torch.Tensor:
    """round(clamp(x,0,1)*(2^b-1))/(2^b-1) (reference ``compress``, generate_dataset.py:29-34)."""
    m = float(2 ** bits - 1)
    return torch.round(torch.clamp(x, 0.0, 1.0) * m) / m


def avg_pool3_s2(x: torch.Tensor) -> torch.Tensor:
    """AvgPool2d(3, s2, p1, count_include_pad=False) (reference networks.py:732)."""
    return F.avg_pool2d(x, 3, stride=2, padding=1, count_include_pad=False)


def l2_normalize_channels(x: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    return F.normalize(x, p=2, dim=1, eps=eps)

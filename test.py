#!/usr/bin/env python
"""Inference entry point, flag-compatible with the reference test.py (:11-16).

Loads the generator from ``checkpoint/<dataset>/netG_model_epoch_<nepochs>.pth`` (the
reference's path) or, if that does not exist, the trainer's
``checkpoint/<dataset>/net_<name>_epoch_<nepochs>.pth``; accepts the dict format
(``state_dict_g``) and -- with ``--allow_pickle`` only, since it executes code from the
file -- a legacy whole-module pickle (quirk A5).  Every test image is resized to 256x256
(bicubic, utils.load_img), run through G (``--with_compress`` first applies C and the
quantiser, which the reference omits: quirk A6) and written to ``result/<dataset>/``.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None):
    p = argparse.ArgumentParser(description="pix2pix-pytorch-implementation")
    p.add_argument("--dataset", required=True, help="facades")
    p.add_argument("--direction", type=str, default="b2a", help="a2b or b2a")
    p.add_argument("--nepochs", type=int, default=200, help="saved model of which epochs")
    p.add_argument("--cuda", action="store_true", help="use cuda")
    p.add_argument("--name", default="run", help="training name (trainer checkpoint path)")
    p.add_argument("--checkpoint", default=None, help="explicit checkpoint file")
    p.add_argument("--netG", default="expand", help="expand | unet_256 | ...")
    p.add_argument("--ngf", type=int, default=64)
    p.add_argument("--norm", default="instance")
    p.add_argument("--image_size", type=int, default=256)
    p.add_argument("--with_compress", action="store_true", help="apply C + quantiser first")
    p.add_argument("--bits", type=int, default=3)
    p.add_argument("--allow_pickle", action="store_true")
    p.add_argument("--backend", default=None, choices=["native", "torch"])
    opt = p.parse_args(argv)
    print(opt)

    import p2p_pytorch_amd as p2p
    from p2p_pytorch_amd import ops
    from p2p_pytorch_amd.data import is_image_file, load_img, normalize, save_img, to_tensor
    from p2p_pytorch_amd.engine.checkpoint import load_generator
    from p2p_pytorch_amd.models import define_C, define_G

    device = torch.device("cuda:0" if opt.cuda else "cpu")
    p2p.set_backend(opt.backend or "native")
    path = opt.checkpoint
    if path is None:
        path = "checkpoint/{}/netG_model_epoch_{}.pth".format(opt.dataset, opt.nepochs)
        if not os.path.exists(path):
            path = "checkpoint/{}/net_{}_epoch_{}.pth".format(opt.dataset, opt.name, opt.nepochs)
    if opt.netG.startswith("unet"):
        net_g = define_G(netG=opt.netG, ngf=opt.ngf, norm=opt.norm, gpu_id="cpu", verbose=False)
    else:
        net_g = define_G(gpu_id="cpu", verbose=False)
    load_generator(path, net_g, device, allow_pickle=opt.allow_pickle)
    net_g.eval()   # BN running statistics, as the trainer's per-epoch evaluation
    net_c = None
    if opt.with_compress:
        net_c = define_C(gpu_id="cpu", verbose=False)
        state = torch.load(path, map_location="cpu", weights_only=True)
        net_c.load_state_dict(state["state_dict_c"])
        net_c.to(device).eval()
    dtype = torch.bfloat16 if (device.type == "cuda" and p2p.get_backend() == "native") else torch.float32

    image_dir = "dataset/{}/test/{}/".format(opt.dataset, "a" if opt.direction == "a2b" else "b")
    out_dir = os.path.join("result", opt.dataset)
    os.makedirs(out_dir, exist_ok=True)
    names = sorted(x for x in os.listdir(image_dir) if is_image_file(x))
    with torch.no_grad():
        for name in names:
            img = normalize(to_tensor(load_img(os.path.join(image_dir, name), opt.image_size)))
            x = img.unsqueeze(0).to(device, dtype).contiguous(memory_format=torch.channels_last)
            if net_c is not None:
                x = ops.quantize(net_c(x), opt.bits)
            out = net_g(x)
            save_img(out.detach().squeeze(0).float().cpu(), os.path.join(out_dir, name))
            print("Image saved as {}".format(os.path.join(out_dir, name)))
    return len(names)


if __name__ == "__main__":
    main()

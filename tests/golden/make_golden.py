"""Generate golden fixtures from the reference's own importable Python code (run in the build container,
where /root/reference exists; the fixtures are committed so tests never need the reference at run time).

  golden_sh.npz      colours from utils/sh_utils.eval_sh exactly as render() computes them when
                     pipe.convert_SHs_python is set (gaussian_renderer/__init__.py:106-111): this is the
                     reference's own Python definition of the SH->RGB step of preprocessCUDA
                     (forward.cu:25-76), incl. the +0.5 and clamp_min(0).
  golden_camera.npz  world_view_transform / full_proj_transform / camera_center built with
                     utils/graphics_utils.getWorld2View2 + getProjectionMatrix as scene/cameras.py:102-107 does.
  golden_loss.npz    utils/loss_utils.l1_loss / ssim values and their autograd gradients w.r.t. the rendered image,
                     and the full training loss of train_single.py:106-118 (L1, D-SSIM and the masked inverse-depth
                     L1) with its gradients w.r.t. image and inverse depth, in float32 on the CPU.

Only data (inputs and expected outputs) is written; no reference source is copied.
"""
import math
import os
import sys

import numpy as np
import torch

REF = os.environ.get("HLGS_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, REF)
    from utils.graphics_utils import focal2fov, getProjectionMatrix, getWorld2View2
    from utils.sh_utils import eval_sh

    rng = np.random.default_rng(1234)
    # ---- SH: every degree, 400 Gaussians each
    out = {}
    for deg in range(4):
        P = 400
        M = (deg + 1) ** 2
        shs = rng.normal(0, 0.4, (P, 16, 3)).astype(np.float32)
        shs[:, 0, :] = rng.normal(0, 0.8, (P, 3))
        means = rng.uniform(-5, 5, (P, 3)).astype(np.float32)
        campos = rng.uniform(-1, 1, 3).astype(np.float32)
        feats = torch.tensor(shs[:, :M, :])
        shs_view = feats.transpose(1, 2).view(-1, 3, M)
        dir_pp = torch.tensor(means) - torch.tensor(campos).repeat(P, 1)
        dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(eval_sh(deg, shs_view, dir_pp_normalized) + 0.5, 0.0)
        out[f"shs_{deg}"] = shs[:, :M, :]
        out[f"means_{deg}"] = means
        out[f"campos_{deg}"] = campos
        out[f"rgb_{deg}"] = rgb.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "golden_sh.npz"), **out)

    # ---- cameras: a few poses / resolutions (fx = fy = 0.9 W, primx = primy = 0.5, znear 0.01, zfar 100)
    cams = {}
    poses = [(np.eye(3), np.zeros(3)), ]
    for k in range(3):
        a = 0.3 * (k + 1)
        c, s = math.cos(a), math.sin(a)
        Rz = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
        Ry = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
        poses.append((Ry @ Rz, rng.uniform(-2, 2, 3)))
    sizes = [(1920, 1080), (256, 256), (100, 75), (1028, 688)]
    for i, ((R, T), (W, H)) in enumerate(zip(poses, sizes)):
        fx = 0.9 * W
        fovx, fovy = focal2fov(fx, W), focal2fov(fx, H)
        wv = torch.tensor(getWorld2View2(R, T, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
        pr = getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy, primx=0.5, primy=0.5).transpose(0, 1)
        full = wv.unsqueeze(0).bmm(pr.unsqueeze(0)).squeeze(0)
        cc = wv.inverse()[3, :3]
        cams[f"R_{i}"], cams[f"T_{i}"], cams[f"WH_{i}"] = R, T, np.array([W, H])
        cams[f"view_{i}"], cams[f"proj_{i}"], cams[f"campos_{i}"] = wv.numpy(), full.numpy(), cc.numpy()
    np.savez_compressed(os.path.join(OUT, "golden_camera.npz"), **cams)

    # ---- losses: the reference's own l1_loss / ssim and the train_single.py loss expression
    from utils.loss_utils import l1_loss, ssim
    loss = {}
    for i, (C, H, W) in enumerate([(3, 37, 53), (3, 64, 48), (1, 20, 31)]):
        img = rng.uniform(0, 1, (C, H, W)).astype(np.float32)
        gt = np.clip(img + rng.normal(0, 0.15, (C, H, W)), 0, 1).astype(np.float32)
        gt[:, :3, :5] = img[:, :3, :5]  # exact ties: |x - y| = 0 has gradient 0
        inv = rng.uniform(0.05, 0.5, (1, H, W)).astype(np.float32)
        mono = (inv + rng.normal(0, 0.05, (1, H, W))).astype(np.float32)
        mask = (rng.uniform(0, 1, (1, H, W)) < 0.8).astype(np.float32)
        lam, dw = 0.2, 0.5
        ti = torch.tensor(img, requires_grad=True)
        s_val = ssim(ti, torch.tensor(gt))
        (g_ssim,) = torch.autograd.grad(s_val, ti)
        ti = torch.tensor(img, requires_grad=True)
        l_val = l1_loss(ti, torch.tensor(gt))
        (g_l1,) = torch.autograd.grad(l_val, ti)
        ti = torch.tensor(img, requires_grad=True)
        tinv = torch.tensor(inv, requires_grad=True)
        Ll1 = l1_loss(ti, torch.tensor(gt))
        Lssim = (1.0 - ssim(ti, torch.tensor(gt)))
        total = (1.0 - lam) * Ll1 + lam * Lssim
        Ld = torch.abs((tinv - torch.tensor(mono)) * torch.tensor(mask)).mean()
        total = total + dw * Ld
        g_img, g_inv = torch.autograd.grad(total, (ti, tinv))
        for k, v in dict(img=img, gt=gt, inv=inv, mono=mono, mask=mask, ssim=s_val.detach().numpy(),
                         g_ssim=g_ssim.numpy(), l1=l_val.detach().numpy(), g_l1=g_l1.numpy(),
                         loss=total.detach().numpy(), depth_l1=Ld.detach().numpy(), g_img=g_img.numpy(),
                         g_inv=g_inv.numpy(), lam=np.float32(lam), dw=np.float32(dw)).items():
            loss[f"{k}_{i}"] = v
    np.savez_compressed(os.path.join(OUT, "golden_loss.npz"), **loss)
    print("wrote golden_sh.npz, golden_camera.npz, golden_loss.npz")


if __name__ == "__main__":
    main()

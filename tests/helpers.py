"""Shared test helpers: run one scene through the MI355X path (public API) and through the oracle."""
import numpy as np
import torch

from hlgs_core import synthetic as S


def settings_for(cam, sh_degree, device, do_depth=True, debug=False, hierarchy=None):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    e_i = torch.empty(0, dtype=torch.int32, device=device)
    e_f = torch.empty(0, dtype=torch.float32, device=device)
    h = hierarchy or {}
    return GaussianRasterizationSettings(
        image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
        bg=cam["bg"].to(device), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(device),
        projmatrix=cam["projmatrix"].to(device), sh_degree=sh_degree, campos=cam["campos"].to(device),
        prefiltered=False, debug=debug, render_indices=h.get("render_indices", e_i),
        parent_indices=h.get("parent_indices", e_i), interpolation_weights=h.get("interpolation_weights", e_f),
        num_node_kids=h.get("num_node_kids", e_i), do_depth=do_depth)


def gpu_render(scene, cam, do_depth=True, grads=None, use_colors=False, use_cov=False, device="cuda"):
    """Forward (+ backward when `grads` is given) through GaussianRasterizer on the GPU."""
    from diff_gaussian_rasterization import GaussianRasterizer
    t = lambda a: torch.tensor(np.ascontiguousarray(a), device=device, requires_grad=True)  # noqa: E731
    means3D = t(scene["means3D"])
    means2D = torch.zeros_like(means3D, requires_grad=True)
    opac = t(scene["opacities"])
    kw = {}
    if use_colors:
        kw["colors_precomp"] = t(scene["colors_precomp"])
    else:
        kw["shs"] = t(scene["shs"])
    if use_cov:
        kw["cov3D_precomp"] = t(scene["cov3D_precomp"])
    else:
        kw["scales"] = t(scene["scales"])
        kw["rotations"] = t(scene["rotations"])
    rs = settings_for(cam, scene.get("sh_degree", 0), device, do_depth=do_depth)
    rast = GaussianRasterizer(rs)
    color, radii, invd = rast(means3D=means3D, means2D=means2D, opacities=opac, **kw)
    out = dict(color=color.detach().cpu().numpy(), radii=radii.cpu().numpy(), invdepth=invd.detach().cpu().numpy())
    if grads is not None:
        g, gd = grads
        loss = (color * torch.tensor(g, device=device)).sum() if g is not None else 0.0
        if do_depth and gd is not None:
            loss = loss + (invd * torch.tensor(gd, device=device)).sum()
        loss.backward()
        out["dmean3D"] = means3D.grad.cpu().numpy()
        out["dmean2D"] = means2D.grad.cpu().numpy()
        out["dopacity"] = opac.grad.cpu().numpy()
        for k, v in kw.items():
            out["d_" + k] = v.grad.cpu().numpy()
    return out


def drops_empty(P):
    """Whether the HIP binning of a P-Gaussian frame leaves out the instances whose quadrant mask is 0
    (hlgs_point_list_drops_empty): an oracle frame whose tile lists or n_contrib are compared with the GPU's is run
    with the same drop_empty.  Images and gradients do not depend on it."""
    from hlgs_core import _lib as L
    return bool(L.load().hlgs_point_list_drops_empty(int(P)))


def binned(fr):
    """Entries an oracle frame binned: the tile lists' total, without the sentinel entries of culled or dropped
    instances that sort behind them (compare this many point_list entries)."""
    return int((fr.ranges[:, 1].astype(np.int64) - fr.ranges[:, 0].astype(np.int64)).sum())


def oracle_render(scene, cam, do_depth=True, grads=None, use_colors=False, use_cov=False, lib=False, drop_empty=False):
    """lib: the oracle build (False: the serial reference of every parity check; "fma": the same source with FMA
    contraction, for build-to-build variance).  drop_empty: see drops_empty."""
    from oracle import oracle as O
    sc = dict(means3D=scene["means3D"], opacities=scene["opacities"], sh_degree=scene.get("sh_degree", 0))
    if use_colors:
        sc["colors_precomp"] = scene["colors_precomp"]
    else:
        sc["shs"] = scene["shs"]
    if use_cov:
        sc["cov3D_precomp"] = scene["cov3D_precomp"]
    else:
        sc["scales"] = scene["scales"]
        sc["rotations"] = scene["rotations"]
    camn = S.cam_numpy(cam)
    fr = O.forward(sc, camn, do_depth=do_depth, omp=lib, drop_empty=drop_empty)
    out = dict(color=fr.color, radii=fr.radii, invdepth=fr.invdepth, frame=fr)
    if grads is not None:
        g, gd = grads
        gr = O.backward(fr, sc, g, gd if do_depth else None)
        out["dmean3D"] = gr["dmean3D"]
        out["dmean2D"] = gr["dmean2D"]
        out["dopacity"] = gr["dopacity"]
        if use_colors:
            out["d_colors_precomp"] = gr["dcolor"]
        else:
            out["d_shs"] = gr["dsh"]
        if use_cov:
            out["d_cov3D_precomp"] = gr["dcov3D"]
        else:
            out["d_scales"] = gr["dscale"]
            out["d_rotations"] = gr["drot"]
    return out


def rel_err(a, b):
    """max |a-b| / max |b| (per tensor) -- the 1e-3 gradient criterion of BASELINE.json north_star."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    if b.size == 0:
        return 0.0 if a.size == 0 else float("inf")
    den = max(np.abs(b).max(), 1e-12)
    return float(np.abs(a - b).max() / den)


def grad_check(a, b, rtol=1e-3, atol_rel=1e-5, row_rtol=0.0):
    """Element-wise gradient criterion: |a - b| <= rtol * |b| + atol_rel * max|b| for every entry, so small entries
    (distant Gaussians' SH rows, cancelling sums) are checked too, not only the tensor's largest.  Returns
    (worst ratio |a - b| / bound, ok).  The floor atol_rel * max|b| covers entries whose float sum cancels: the GPU
    sums per-tile moments in another order than the oracle's per-pixel loop (measured ~1e-6 of max|b|)."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    if b.size == 0:
        return (0.0, a.size == 0)
    bound = rtol * np.abs(b) + atol_rel * max(np.abs(b).max(), 1e-30)
    if row_rtol > 0 and b.ndim > 1:
        # per-Gaussian floor: row_rtol x the largest entry of the same Gaussian's gradient (its own scale)
        rows = b.reshape(b.shape[0], -1)
        rmax = np.abs(rows).max(1).reshape((b.shape[0],) + (1,) * (b.ndim - 1))
        bound = np.maximum(bound, rtol * np.abs(b) + row_rtol * rmax)
    ratio = float((np.abs(a - b) / bound).max())
    return ratio, ratio <= 1.0


def assert_grad(name, a, b, tol=1e-3, row_rtol=0.0):
    """Both gradient criteria: north_star's max|a-b| / max|b| <= tol, and grad_check element-wise (row_rtol > 0 adds
    grad_check's per-Gaussian floor)."""
    e = rel_err(a, b)
    assert e <= tol, f"{name}: rel err {e}"
    ratio, ok = grad_check(a, b, row_rtol=row_rtol)
    assert ok, f"{name}: element-wise |a-b| / (1e-3|b| + 1e-5 max|b|) = {ratio}"


def image_check(gpu, ref, tol=1e-4, max_bad_frac=0.0):
    """Forward criterion: per-pixel L-inf <= tol.  The GPU path and the oracle decide alpha >= 1/255, power > 0 and
    T < 1e-4 bit-identically (DESIGN A-17), so no pixel may exceed tol (max_bad_frac = 0); a caller comparing
    against arithmetic that decides those thresholds differently (the oracle's reference_order mode) passes an
    explicit max_bad_frac and reports the count."""
    d = np.abs(np.asarray(gpu, np.float64) - np.asarray(ref, np.float64))
    if d.ndim == 3:
        d = d.max(0)
    bad = (d > tol).sum()
    return float(d.max()) if d.size else 0.0, int(bad), bad <= max(0, int(max_bad_frac * d.size))

"""BASELINE.json configs, each on its own workload, through the HIP path against the oracle.

  configs[0]  10k Gaussians, SH degree 0, one 256x256 camera: forward + backward parity.
  configs[1]  1M Gaussians, SH degree 3, 1920x1080 (the bench workload, same seeds): the whole frame against the
              serial oracle -- radii bit-exact, every pixel within 1e-4, every gradient element-wise.
  configs[2]  the hierarchical-LOD training step of render_post (gaussian_renderer/__init__.py:304-347;
              render_hierarchy.py:48-92, debug_utils.py:155-197) at 1080p on a synthetic binary hierarchy over 1M
              leaves (the example dataset is not available offline): expand_to_size_dynamic -> weights -> lerp ->
              rasterize -> backward through the lerp.  Each stage is checked against the oracle on the previous
              stage's GPU output (cut bit-exact, weights / lerp within float rounding, frame and gradients as
              configs[1]), and the leaf gradients against the oracle's lerp backward of the oracle's raster
              gradients.
  configs[3]  4M Gaussians per GPU: tests/test_gpu_scale.py (single-GPU properties at full size) and
              tests/test_dp_cpu.py (the gradient exchange, gloo, world size 2).
  configs[4]  train_post.py's step on a synthetic 2-chunk merged hierarchy (mainHierarchyMerger.cpp:94-140,
              hlgs_core.synthetic.make_merged_hierarchy) at 1080p: SPT cache step -> activations -> alt rasterizer
              (antialiasing, SH degree 1) -> L1 + D-SSIM + masked inverse-depth L1 -> backward -> dense Adam, two
              views in a row.  Cache lists and moved rows bit-exact against oracle/spt_ref.py; the frame and its
              gradients against the oracle's alt restatement; the loss and dL/dimage against oracle/loss_ref.py;
              Adam against spt_ref.adam_dense.
"""
import numpy as np
import pytest
import torch

from hlgs_core import synthetic as S
from helpers import assert_grad, gpu_render, grad_check, image_check, oracle_render, rel_err
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
FWD_TOL = 1e-4


def _check_frame(gpu, ref, row_rtol=0.0):
    np.testing.assert_array_equal(gpu["radii"], ref["radii"])
    for k in ("color", "invdepth"):
        mx, nbad, ok = image_check(gpu[k], ref[k], FWD_TOL)
        assert ok, f"{k}: L-inf {mx}, {nbad} pixels over {FWD_TOL}"
    for k in ref:
        if k.startswith("d"):
            assert_grad(k, gpu[k][..., :ref[k].shape[-1]], ref[k], row_rtol=row_rtol)


ILL = ("d_scales", "d_rotations")  # gradients behind the ill-conditioned conic -> cov3D backward of wide splats


VARIANCE_CEILING = 40.0  # element-wise ratio; the oracle builds' own measured ~33 (d_rotations) / ~30 (d_scales)


def _assert_grad_within_variance(name, a, b, b_alt, row_rtol=1e-3):
    """(b_alt may be a callable returning the contracted build's gradient: it is then computed only when needed.)"""
    return _assert_grad_within_variance_(name, a, b, b_alt, row_rtol)


def _assert_grad_within_variance_(name, a, b, b_alt, row_rtol=1e-3):
    """north_star's per-tensor rule (max|a - b| / max|b| <= 1e-3) always; element-wise, grad_check with the per-Gaussian
    floor, or else no further from the oracle b than b_alt -- the same oracle source built with FMA contraction -- is,
    and never above VARIANCE_CEILING: the builds' variance comes from an x86 contraction pattern, not from the
    reference's nvcc build, so it may not loosen the gate without bound.  Measured on the configs[2] frame
    (tools/diag/lod_chain_variance.py): the builds differ by ~33 (d_rotations) and ~30 (d_scales); the GPU by less."""
    e = rel_err(a, b)
    assert e <= 1e-3, f"{name}: rel err {e}"
    ratio, ok = grad_check(a, b, row_rtol=row_rtol)
    if not ok:
        var, _ = grad_check(b_alt() if callable(b_alt) else b_alt, b, row_rtol=row_rtol)
        print(f"{name}: element-wise ratio {ratio:.3f} (GPU vs oracle), {var:.3f} (oracle builds)")
        assert ratio <= min(var, VARIANCE_CEILING), \
            f"{name}: element-wise ratio {ratio} above the oracle builds' own {var} (ceiling {VARIANCE_CEILING})"


@pytest.mark.parametrize("P,deg,W,H", [(10_000, 0, 256, 256), (1_000_000, 3, 1920, 1080)],
                         ids=["configs0", "configs1"])
def test_configs_frame_matches_oracle(P, deg, W, H):
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, deg, cam, seed=0)
    g = S.upstream_grads(W, H, seed=1)
    _check_frame(gpu_render(sc, cam, grads=g), oracle_render(sc, cam, grads=g))


@pytest.mark.parametrize("realcam", [None, 5], ids=["synthetic_cam", "reference_cam5"])
def test_configs2_lod_chain_1080p(realcam):
    """realcam: one of the reference's own cameras (tests/golden/golden_realcam.npz, rotated, fx != fy) at 1080p with
    its own FoV; the hierarchy is built over leaves in front of it, and the view direction handed to the LOD
    functions is world_view_transform[:3, :3] @ (0, 0, 1), as debug_utils.py:150-153 forms it."""
    import gaussian_hierarchy as GH
    from diff_gaussian_rasterization import GaussianRasterizer
    from helpers import settings_for
    W, H, deg, tau_px = 1920, 1080, 3, 6.0
    cam = S.make_camera(W, H) if realcam is None else S.real_camera(S.load_real_cameras()[realcam], W=W, H=H)
    h = S.make_dynamic_hierarchy(S.make_gaussians(1_000_000, deg, cam, seed=0), seed=0)
    N = h["nodes"].shape[0]
    tau = (2 * (tau_px + 0.5)) * cam["tanfovx"] / (0.5 * W)  # bench.py's config3 threshold
    vp = cam["campos"].numpy()
    vd = (cam["viewmatrix"][:3, :3] @ torch.tensor([0.0, 0.0, 1.0])).numpy().astype(np.float32)
    d = lambda a, **kw: torch.tensor(np.ascontiguousarray(a), device=DEV, **kw)  # noqa: E731
    nodes = d(h["nodes"])
    leaves = [d(h[k], requires_grad=True) for k in ("means3D", "scales", "rotations", "opacities", "shs")]
    xyz, scales = leaves[0], leaves[1]
    ri, pi, ni, kids = (torch.zeros(N, dtype=torch.int32, device=DEV) for _ in range(4))
    ts = torch.zeros(N, device=DEV)
    n = GH.expand_to_size_dynamic(nodes, xyz.detach(), scales.detach(), tau, cam["campos"].to(DEV),
                                  torch.tensor(vd), ri, pi, ni)
    on, ori, opi, oni = O.expand_to_size_dynamic(h["nodes"], h["means3D"], h["scales"], tau, vp, vd)
    assert n == on and n > 100_000
    for got, want in ((ri, ori), (ni, oni)):
        np.testing.assert_array_equal(got[:n].cpu().numpy(), want[:n])
    has_parent = h["nodes"][ori[:n], 1] >= 0  # parent_indices is written only where a parent exists (A-11)
    np.testing.assert_array_equal(pi[:n].cpu().numpy()[has_parent], opi[:n][has_parent])
    GH.get_interpolation_weights_dynamic(ni[:n], tau, nodes, xyz.detach(), scales.detach(), cam["campos"],
                                         torch.tensor(vd), ts, kids)
    ots, okids = O.interp_weights_dynamic(oni[:n], tau, h["nodes"], h["means3D"], h["scales"], vp)
    np.testing.assert_array_equal(ts[:n].cpu().numpy(), ots)  # lod.hip is built uncontracted, as the oracle
    np.testing.assert_array_equal(kids[:n].cpu().numpy(), okids)
    pi_c = pi.clone()
    pi_c[n:] = 0
    pi_c[:n][~torch.tensor(has_parent, device=DEV)] = 0  # roots lerp with row 0 at weight 0 (A-11)
    outs = GH.interpolate_lod(*leaves, ri[:n], pi_c, ts, 0)
    ref_l = O.lod_interp_forward(0, ri[:n].cpu().numpy(), pi_c[:n].cpu().numpy(), ts[:n].cpu().numpy(),
                                 h["means3D"], h["scales"], h["rotations"], h["opacities"], h["shs"])
    keys = ("means", "scales", "rots", "opac", "shs")
    for got, k in zip(outs, keys):
        np.testing.assert_allclose(got.detach().cpu().numpy().reshape(ref_l[k].shape), ref_l[k], rtol=1e-6,
                                   atol=1e-6)
    for o in outs:
        o.retain_grad()
    m2 = torch.zeros_like(outs[0], requires_grad=True)
    rast = GaussianRasterizer(settings_for(cam, deg, DEV))
    color, radii, invd = rast(means3D=outs[0], means2D=m2, opacities=outs[3], shs=outs[4], scales=outs[1],
                              rotations=outs[2])
    g, gd = S.upstream_grads(W, H, seed=1)
    torch.autograd.backward([color, invd], [d(g), d(gd)])
    # the raster stage against the oracle on the GPU's lerped Gaussians
    sc = dict(means3D=outs[0].detach().cpu().numpy(), scales=outs[1].detach().cpu().numpy(),
              rotations=outs[2].detach().cpu().numpy(), opacities=outs[3].detach().cpu().numpy(),
              shs=outs[4].detach().cpu().numpy(), sh_degree=deg)
    ref = oracle_render(sc, cam, grads=(g, gd))
    gpu = dict(color=color.detach().cpu().numpy(), invdepth=invd.detach().cpu().numpy(), radii=radii.cpu().numpy(),
               dmean3D=outs[0].grad.cpu().numpy(), dmean2D=m2.grad.cpu().numpy(), dopacity=outs[3].grad.cpu().numpy(),
               d_shs=outs[4].grad.cpu().numpy(), d_scales=outs[1].grad.cpu().numpy(),
               d_rotations=outs[2].grad.cpu().numpy())
    # The lerped parents are wide (radius up to ~45 px, 15-30 tiles) and their conic -> cov2D -> cov3D backward is
    # ill-conditioned ((denom - c_xx c_yy) cancels to -c_xy^2): the GPU sums each splat's dconic per tile, the
    # oracle per pixel, and that rounding difference moves ~10 of 600k scale / rotation gradient entries by up to
    # 0.17% of the same Gaussian's largest entry (tools/diag/lod_chain_grads.py).  Those tensors are therefore
    # checked per Gaussian: |gpu - ref| <= 1e-3 |ref| + 1e-3 max|ref of that Gaussian| (and the per-tensor rule) --
    # or, where even that is tighter than float32 allows, against the oracle's own build-to-build variance: the same
    # oracle source built with a*b+c contracted (as nvcc's default --fmad=true builds the reference) differs from the
    # uncontracted build by an element-wise ratio of ~33 on d_rotations and ~30 on d_scales of this frame
    # (tools/diag/lod_chain_variance.py), so the GPU passes if it is no further from the oracle than that build is.
    ref_fma = oracle_render(sc, cam, grads=(g, gd), lib="fma")
    _check_frame({k: v for k, v in gpu.items() if k not in ILL}, {k: v for k, v in ref.items() if k not in ILL},
                 row_rtol=1e-3)
    for k in ILL:
        _assert_grad_within_variance(k, gpu[k], ref[k], ref_fma[k])
    # the lerp backward: the oracle's restatement of autograd through render_post's lerp, fed the oracle's
    # raster gradients, against the leaf gradients the GPU chain produced
    dl = O.lod_interp_backward(0, ri[:n].cpu().numpy(), pi_c[:n].cpu().numpy(), ts[:n].cpu().numpy(), h["rotations"],
                               N, dict(means=ref["dmean3D"], scales=ref["d_scales"], rots=ref["d_rotations"],
                                       opac=ref["dopacity"], shs=ref["d_shs"]))
    dl_fma = O.lod_interp_backward(0, ri[:n].cpu().numpy(), pi_c[:n].cpu().numpy(), ts[:n].cpu().numpy(),
                                   h["rotations"], N, dict(means=ref_fma["dmean3D"], scales=ref_fma["d_scales"],
                                                           rots=ref_fma["d_rotations"], opac=ref_fma["dopacity"],
                                                           shs=ref_fma["d_shs"]))
    for leaf, k in zip(leaves, keys):
        got = leaf.grad.cpu().numpy().reshape(dl[k].shape)
        if k in ("scales", "rots"):
            _assert_grad_within_variance("leaf " + k, got, dl[k], dl_fma[k])
        else:
            assert_grad("leaf " + k, got, dl[k], row_rtol=1e-3)


@pytest.mark.parametrize("leaves", [80_000, 1_000_000], ids=["80k_leaves", "bench_1M_leaves"])
def test_configs4_merged_two_chunk_train_post_step(leaves):
    """leaves = 1M is bench.py's config5 workload size: the SPT cache lists and moved rows, the
    frame and every gradient, the loss and Adam, at the size the bench times."""
    from alt_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from hlgs_core import spt
    from hlgs_core.loss import photometric_loss
    from hlgs_core.spt_cache import SPTCache
    from oracle import loss_ref as LR
    from oracle import spt_ref as SR
    from test_gpu_cache import NAMES, _dev_list, _Oracle
    W, H, act_deg = 1920, 1080, 1
    cam0 = S.make_camera(W, H)
    c0 = S.make_gaussians(leaves // 2, 3, cam0, seed=1)
    c1 = S.make_gaussians(leaves - leaves // 2, 3, cam0, seed=2)
    c1["means3D"] = c1["means3D"] + np.array([4.0, 0.0, 6.0], np.float32)
    h = S.make_merged_hierarchy([c0, c1], np.array([[0, 0, 12], [4, 0, 18]], np.float32))
    assert h["nodes"][0, 2] == 2 and (h["nodes"][h["chunk_roots"], 1] == 0).all()
    nodes = torch.tensor(h["nodes"])
    log_s = torch.log(torch.tensor(h["scales"]))
    b = spt.build_hierarchical_spt(nodes, torch.tensor(h["means3D"]), log_s, 0, 0.5, 0.00228, 256)
    op = torch.tensor(h["opacities"]).clamp(1e-4, 1 - 1e-4)
    shs = torch.tensor(h["shs"])
    storage = dict(xyz=torch.tensor(h["means3D"]), f_dc=shs[:, :1].contiguous(), f_rest=shs[:, 1:].contiguous(),
                   opacity=torch.log(op / (1 - op)), scaling=log_s, rotation=torch.tensor(h["rotations"]))
    cache = SPTCache(storage, b, 0, reuse_tolerance=0.9)
    orc = _Oracle(b, storage, 0, 0.9, 10 ** 9)
    rng = np.random.default_rng(1)
    gt = torch.tensor(rng.uniform(0, 1, (3, H, W)).astype(np.float32), device=DEV)
    mono = torch.tensor(rng.uniform(0.05, 0.5, (1, H, W)).astype(np.float32), device=DEV)
    mask = torch.tensor((rng.uniform(0, 1, (1, H, W)) < 0.8).astype(np.float32), device=DEV)
    lam, dw = 0.2, 0.5
    lrs = dict(xyz=1.6e-4, f_dc=2.5e-3, f_rest=2.5e-3 / 20, opacity=5e-2, scaling=5e-3, rotation=1e-3)
    kept = 0
    for it in range(2):
        cam = S.make_camera(W, H, T=np.array([0.05 * it, 0.0, 0.1 * it]))
        got = cache.step(cam["projmatrix"], cam["campos"])
        want = orc.step(cam)
        np.testing.assert_array_equal(got.cpu().numpy(), want["render_indices"])
        for t, (gd_, w) in enumerate(zip(_dev_list(cache), orc.dev)):
            np.testing.assert_array_equal(gd_.detach().cpu().numpy(), w, err_msg=f"tensor {t} view {it}")
        kept += want["n_kept"]
        p = cache.params
        acts = dict(means3D=p["xyz"], opacities=torch.sigmoid(p["opacity"]), scales=torch.exp(p["scaling"]),
                    rotations=torch.nn.functional.normalize(p["rotation"]), dc=p["f_dc"], shs=p["f_rest"])
        for k in ("opacities", "scales", "rotations"):
            acts[k].retain_grad()
        s = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=cam["tanfovx"],
                                          tanfovy=cam["tanfovy"], bg=torch.zeros(3, device=DEV), scale_modifier=1.0,
                                          viewmatrix=cam["viewmatrix"].to(DEV), projmatrix=cam["projmatrix"].to(DEV),
                                          sh_degree=act_deg, campos=cam["campos"].to(DEV), prefiltered=False,
                                          debug=False, antialiasing=True)
        means2D = torch.zeros_like(acts["means3D"], requires_grad=True)
        img, radii, invd = GaussianRasterizer(s)(means2D=means2D, **acts)
        img.retain_grad()
        invd.retain_grad()
        loss = photometric_loss(img.clamp(0, 1), gt, lam, invd, mono, mask, dw)[0]
        ref_loss = LR.photometric(img.detach().clamp(0, 1).cpu(), gt.cpu(), lam, invd.detach().cpu(), mono.cpu(),
                                  mask.cpu(), dw)
        assert abs(float(loss.detach()) - float(ref_loss)) <= 1e-5 * abs(float(ref_loss))
        loss.backward()
        # upstream gradient of the rasterizer against the float64 restatement's autograd
        ti = img.detach().cpu().double().requires_grad_(True)
        tv = invd.detach().cpu().double().requires_grad_(True)
        dimg, dinv = torch.autograd.grad(LR.photometric(ti.clamp(0, 1), gt.cpu(), lam, tv, mono.cpu(), mask.cpu(),
                                                        dw), (ti, tv))
        assert_grad("dL/dimage", img.grad.cpu().numpy(), dimg.numpy())
        assert_grad("dL/dinvdepth", invd.grad.cpu().numpy(), dinv.numpy())
        # the alt rasterizer stage against the oracle on the same activated Gaussians and upstream gradients
        sc = {k: v.detach().cpu().numpy() for k, v in acts.items()}
        sc.update(sh_degree=act_deg, alt=True, antialiasing=True)
        fr = O.forward(sc, S.cam_numpy(cam))
        gr = O.backward(fr, sc, img.grad.cpu().numpy(), invd.grad.cpu().numpy())
        np.testing.assert_array_equal(radii.cpu().numpy(), fr.radii)
        for k, ref_img in (("color", fr.color), ("invdepth", fr.invdepth)):
            got_img = (img if k == "color" else invd).detach().cpu().numpy()
            mx, nbad, ok = image_check(got_img, ref_img, FWD_TOL)
            assert ok, f"view {it} {k}: L-inf {mx}, {nbad} pixels"
        # the scale and rotation gradients of the cut's coarse interior nodes (rects over hundreds of tiles) go through the
        # ill-conditioned conic -> cov3D backward, as in configs[2]: there the bound is the oracle's own build-to-build
        # variance (the same source with FMA contraction) when the element-wise rule is tighter than float32 allows
        fma_cache = {}

        def gr_fma_of(k):  # the contracted oracle build, computed only if an element-wise check needs it
            if not fma_cache:
                fr_fma = O.forward(sc, S.cam_numpy(cam), omp="fma")
                fma_cache.update(O.backward(fr_fma, sc, img.grad.cpu().numpy(), invd.grad.cpu().numpy()))
            return fma_cache[k]
        for name, t, k in (("means3D", p["xyz"], "dmean3D"), ("opacity", acts["opacities"], "dopacity"),
                           ("scales", acts["scales"], "dscale"), ("rotations", acts["rotations"], "drot"),
                           ("f_dc", p["f_dc"], "ddc"), ("f_rest", p["f_rest"], "dsh")):
            got_g = t.grad.cpu().numpy().reshape(gr[k].shape)
            if k in ("dscale", "drot"):
                _assert_grad_within_variance(f"view {it} {name}", got_g, gr[k], lambda k=k: gr_fma_of(k), row_rtol=0.0)
            else:
                assert_grad(f"view {it} {name}", got_g, gr[k])
        # dense Adam on the resident rows against the restatement, fed the same gradients
        grads = [cache.params[k].grad.detach().cpu().clone() for k in NAMES]
        cache.optimizer_step(it, lrs)
        k6 = len(NAMES)
        for i, k in enumerate(NAMES):
            pt, m, v = (torch.tensor(orc.dev[j]) for j in (i, k6 + i, 2 * k6 + i))
            SR.adam_dense(pt, grads[i].clone(), m, v, lrs[k], it + 1, 0)
            got = [cache.params[k].detach(), cache.exp_avgs[k], cache.exp_avg_sqs[k]]
            for gt_, w, what in zip(got, (pt, m, v), ("param", "exp_avg", "exp_avg_sq")):
                np.testing.assert_allclose(gt_.cpu().numpy(), w.numpy(), rtol=2e-6, atol=1e-7,  # as test_gpu_cache
                                           err_msg=f"adam {k} {what} view {it}")
            # carry the GPU's rows on, so the next view's moved rows compare bit-exact
            orc.dev[i], orc.dev[k6 + i], orc.dev[2 * k6 + i] = (t.cpu().numpy().copy() for t in got)
        for q in cache.params.values():
            q.grad = None
    assert kept > 0  # the second view reused SPTs from the first

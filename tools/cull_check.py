"""Brute-force check that the ellipse-vs-8x8-block culling test (hlgs_math.h foot_touches) never rejects a
block holding a pixel with alpha >= 1/255 (float32 test vs float64 pixel oracle, 4e5 random splats),
and the key scatter's band form of it (splat_bands / row_quad_mask): `python tools/cull_check.py`, or run(N) from
tests/test_cull_check.py."""
import numpy as np


def run(N=400000, seed=0, size=8):
    """size = 8: the 8x8 quadrant blocks (foot_touches, the key scatter's bands); 4: the blend backward's 4x4
    sub-blocks (sub_block_mask: the same band form with 4-row bands and 4-column blocks)."""
    e = float(size - 1)
    rng = np.random.default_rng(seed)
    f32 = np.float32
    x = rng.uniform(-20, 28, N).astype(f32); y = rng.uniform(-20, 28, N).astype(f32)
    # random PD covariance -> conic (dilated like the renderer)
    s1 = np.exp(rng.uniform(np.log(0.3), np.log(30), N)); s2 = np.exp(rng.uniform(np.log(0.3), np.log(30), N))
    th = rng.uniform(0, np.pi, N)
    c, s = np.cos(th), np.sin(th)
    cxx = c*c*s1**2 + s*s*s2**2 + 0.3; cyy = s*s*s1**2 + c*c*s2**2 + 0.3; cxy = c*s*(s1**2 - s2**2)
    det = cxx*cyy - cxy*cxy
    a = (cyy/det).astype(f32); b = (-cxy/det).astype(f32); cc = (cxx/det).astype(f32)
    o = rng.uniform(0.0, 1.0, N).astype(f32)
    # brute force over the 8x8 block at (0,0): any pixel with alpha >= 1/255 (float64 reference)
    px, py = np.meshgrid(np.arange(size), np.arange(size))
    px = px.ravel(); py = py.ravel()
    dx = x[:, None].astype(np.float64) - px; dy = y[:, None].astype(np.float64) - py
    power = -0.5*(a[:, None]*dx*dx + cc[:, None]*dy*dy) - b[:, None]*dx*dy
    alpha = np.minimum(0.99, o[:, None]*np.exp(power))
    truth = ((power <= 0) & (alpha >= 1/255)).any(1)
    # the float32 test
    # the kernels take the bound from the splat's e2 threshold: the smallest float32 at or above -log2(255 o)
    thr_exact = -np.log2(255.0 * o.astype(np.float64))
    thr = thr_exact.astype(f32)
    thr = np.where(thr.astype(np.float64) < thr_exact, np.nextafter(thr, f32(np.inf)), thr).astype(f32)
    t = (np.maximum(f32(-1.3862944)*thr, f32(0)).astype(f32)*f32(1.002) + f32(2e-3)).astype(f32)
    kv = (-b/cc).astype(f32); ku = (-b/a).astype(f32)
    u0 = (0 - x).astype(f32); u1 = u0 + f32(e); v0 = (0 - y).astype(f32); v1 = v0 + f32(e)
    def qu(U):
        v = np.clip(kv*U, v0, v1); return U*(a*U + 2*b*v) + cc*v*v
    def qv(V):
        u = np.clip(ku*V, u0, u1); return V*(cc*V + 2*b*u) + a*u*u
    m = np.minimum(np.minimum(qu(u0), qu(u1)), np.minimum(qv(v0), qv(v1)))
    inside = (u0 <= 0) & (u1 >= 0) & (v0 <= 0) & (v1 >= 0)
    test = np.where(o < f32(1/255*0.999), False, inside | (m <= t))
    res = dict(true=int(truth.sum()), foot_missed=int((truth & ~test).sum()), foot_test=int(test.sum()))

    # ---- the key scatter's band form of the same test (hlgs_math.h splat_bands / quad_mask_bands), checked the same way:
    # per 8-row band, the footprint's exact x-extent, widened by the rounding tolerance; block hit = extent overlaps it
    f64 = np.float64
    def fma32(p, q, r):
        return (p.astype(f64)*q.astype(f64) + r.astype(f64)).astype(f32)
    bb = (b*b).astype(f32); eb = fma32(-b, b, bb)
    det = (fma32(a, cc, -bb) + eb).astype(f32)
    idet = (f32(1)/det).astype(f32); s_ia = (f32(1)/a).astype(f32)
    vmax = np.sqrt((a*t).astype(f32)*idet).astype(f32)
    s_nb = -b; s_det = det; s_at = (a*t).astype(f32)
    s_vmax = (fma32(vmax, np.full_like(vmax, 1e-4), vmax) + f32(1e-3)).astype(f32)
    s_vr = (-b*np.sqrt((t*idet).astype(f32)*(f32(1)/cc).astype(f32)).astype(f32)).astype(f32)
    s_tol = (f32(2e-3)*(np.sqrt(s_at).astype(f32) + np.abs(b)*vmax)*s_ia + f32(2e-3)).astype(f32)
    lo = np.maximum(v0, -s_vmax); hi = np.minimum(v1, s_vmax)
    vR = np.clip(s_vr, lo, hi); vL = np.clip(-s_vr, lo, hi)
    sq = lambda v: np.sqrt(np.maximum(fma32((-s_det*v).astype(f32), v, s_at), f32(0))).astype(f32)
    umax = (fma32(s_nb, vR, sq(vR))*s_ia).astype(f32) + s_tol
    umin = (fma32(s_nb, vL, -sq(vL))*s_ia).astype(f32) - s_tol
    band = (lo <= hi) & (umax >= u0) & (umin <= u1)
    test_b = np.where(o < f32(1/255*0.999), False, band)
    res.update(band_missed=int((truth & ~test_b).sum()), band_test=int(test_b.sum()))
    return res


if __name__ == "__main__":
    r4 = run(size=4)
    print("4x4 sub-blocks, band form: missed (must be 0):", r4["band_missed"], " true:", r4["true"], " test:", r4["band_test"])
    r = run()
    print("missed (must be 0):", r["foot_missed"], " true:", r["true"], " test:", r["foot_test"])
    print("band form: missed (must be 0):", r["band_missed"], " test:", r["band_test"], " (foot form:", r["foot_test"], ")")

"""Deterministic synthetic scenes, cameras and dynamic hierarchies.

The camera follows the reference's conventions exactly:
  world_view_transform = getWorld2View2(R, T).T, projection = getProjectionMatrix(...).T,
  full_proj = world_view @ projection, campos = inverse(world_view)[3, :3]
(scene/cameras.py:96-107, utils/graphics_utils.py:38-77).  The Gaussian
distribution is the one SURVEY.md section 8(d) / BASELINE.md fixes for the
benchmark configs (seeded PCG64).  There is no dataset here: everything is
synthetic and says so.
"""
import math

import numpy as np
import torch


def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


def _world2view2(R, t):
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def _projection(znear, zfar, fovX, fovY, primx=0.5, primy=0.5):
    tanHalfFovY = math.tan((fovY / 2))
    tanHalfFovX = math.tan((fovX / 2))
    top = tanHalfFovY * znear
    bottom = (1 - primy) * 2 * -top
    top = primy * 2 * top
    right = tanHalfFovX * znear
    left = (1 - primx) * 2 * -right
    right = primx * 2 * right
    P = torch.zeros(4, 4)
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def make_camera(W, H, R=None, T=None, focal_scale=0.9, znear=0.01, zfar=100.0, bg=(0.0, 0.0, 0.0), fx=None, fy=None,
                fovx=None, fovy=None, primx=0.5, primy=0.5):
    """Camera dict with float32 CPU tensors laid out exactly as the reference passes them.

    R is the camera-to-world rotation and T the world-to-camera translation (the reference's Camera.R / Camera.T,
    scene/dataset_readers.py).  The field of view comes from fovx / fovy when given (a camera kept at its own FoV and
    rendered at another resolution, as the reference's Camera does when its image is resized), else from the focal
    lengths fx / fy (default focal_scale * W for both): FoVx = focal2fov(fx, W), FoVy = focal2fov(fy, H)
    (scene/dataset_readers.py:87-101).  primx / primy: the principal point as a fraction of the image size
    (getProjectionMatrix, utils/graphics_utils.py:51-77)."""
    R = np.eye(3) if R is None else np.asarray(R, dtype=np.float64)
    T = np.zeros(3) if T is None else np.asarray(T, dtype=np.float64)
    fx = focal_scale * W if fx is None else float(fx)
    fy = focal_scale * W if fy is None else float(fy)
    if fovx is None:
        fovx = focal2fov(fx, W)
    else:  # the focal length the rasterizer derives from the FoV at this width (rasterizer_impl.cu:246-247)
        fovx, fx = float(fovx), W / (2 * math.tan(float(fovx) * 0.5))
    if fovy is None:
        fovy = focal2fov(fy, H)
    else:
        fovy, fy = float(fovy), H / (2 * math.tan(float(fovy) * 0.5))
    wv_t = torch.tensor(_world2view2(R, T)).transpose(0, 1)  # a transposed view, as scene/cameras.py:102 holds it
    wv = wv_t.contiguous()
    pr = _projection(znear, zfar, fovx, fovy, primx, primy).transpose(0, 1)
    full = wv.unsqueeze(0).bmm(pr.unsqueeze(0)).squeeze(0).contiguous()
    campos = wv_t.inverse()[3, :3].contiguous()  # :107 (the float32 inverse rounds by the operand's layout)
    return dict(W=int(W), H=int(H), tanfovx=math.tan(fovx * 0.5), tanfovy=math.tan(fovy * 0.5), fx=fx, fy=fy,
                viewmatrix=wv, projmatrix=full, campos=campos, bg=torch.tensor(bg, dtype=torch.float32), R=R, T=T,
                fovx=fovx, fovy=fovy)


def real_camera(entry, W=None, H=None, **kw):
    """A camera of the reference's own dataset from one cameras.json entry (utils/camera_utils.py:91-111 writes it:
    `position` is the camera centre and `rotation` the camera-to-world rotation, i.e. Camera.R; fx / fy the focal
    lengths at width x height).  T = -R^T position undoes camera_to_JSON's inversion.  W, H: render at another
    resolution with the camera's own field of view (the reference's Camera keeps FoVx / FoVy when it resizes)."""
    R = np.asarray(entry["rotation"], np.float64)
    T = -R.T @ np.asarray(entry["position"], np.float64)
    w0, h0 = int(entry["width"]), int(entry["height"])
    fovx, fovy = focal2fov(float(entry["fx"]), w0), focal2fov(float(entry["fy"]), h0)
    return make_camera(w0 if W is None else W, h0 if H is None else H, R=R, T=T, fovx=fovx, fovy=fovy, **kw)


def load_real_cameras(path=None):
    """The cameras.json entries committed in tests/golden/golden_realcam.npz (tests/golden/make_golden.py), as dicts
    real_camera accepts."""
    import os
    path = path or os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "tests", "golden", "golden_realcam.npz")
    z = np.load(path)
    out = []
    for i in range(int(z["count"])):
        out.append(dict(id=int(z[f"id_{i}"]), rotation=z[f"rotation_{i}"], position=z[f"position_{i}"],
                        fx=float(z[f"fxfy_{i}"][0]), fy=float(z[f"fxfy_{i}"][1]), width=int(z[f"WH_{i}"][0]),
                        height=int(z[f"WH_{i}"][1])))
    return out


def ring_camera(W, H, k, n, radius=0.4, yaw_deg=3.0, **kw):
    """k-th of n cameras on a small ring around the origin, all looking roughly down +z."""
    a = 2 * math.pi * k / max(n, 1)
    yaw = math.radians(yaw_deg) * math.sin(a)
    c, s = math.cos(yaw), math.sin(yaw)
    Rc2w = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])  # camera-to-world rotation
    C = np.array([radius * math.cos(a), radius * math.sin(a) * 0.5, 0.0])
    T = -Rc2w.T @ C  # world-to-camera translation
    return make_camera(W, H, R=Rc2w, T=T, **kw)


def cam_numpy(cam):
    return {k: (v.numpy() if isinstance(v, torch.Tensor) else v) for k, v in cam.items()}


def make_gaussians(P, sh_degree, cam, seed=0, zmin=2.0, zmax=30.0, xy_spread=1.1, sigma_px=(0.3, 3.0),
                   opacity_std=1.5):
    """P Gaussians inside 1.1x the frustum of `cam`; activated parameters, numpy float32."""
    rng = np.random.Generator(np.random.PCG64(seed))
    z = rng.uniform(zmin, zmax, P)
    x = rng.uniform(-xy_spread, xy_spread, P) * z * cam["tanfovx"]
    y = rng.uniform(-xy_spread, xy_spread, P) * z * cam["tanfovy"]
    means = np.stack([x, y, z], 1)
    base = rng.uniform(sigma_px[0], sigma_px[1], P) * z / cam["fx"]
    log_scales = np.log(base)[:, None] + rng.normal(0, 0.2, (P, 3))
    q = rng.normal(0, 1, (P, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    opac = 1 / (1 + np.exp(-rng.normal(0, opacity_std, P)))
    M = (sh_degree + 1) ** 2
    shs = np.empty((P, M, 3))
    shs[:, 0, :] = rng.normal(0, 0.5, (P, 3))
    if M > 1:
        shs[:, 1:, :] = rng.normal(0, 0.1, (P, M - 1, 3))
    # express in world space if the camera is not at the origin (means were drawn in camera space)
    Rc2w, T = np.asarray(cam.get("R", np.eye(3))), np.asarray(cam.get("T", np.zeros(3)))
    C = -Rc2w @ T
    means = means @ Rc2w.T + C
    f = np.float32
    return dict(means3D=means.astype(f), scales=np.exp(log_scales).astype(f), rotations=q.astype(f),
                opacities=opac.astype(f)[:, None], shs=shs.astype(f), sh_degree=sh_degree)


def upstream_grads(W, H, seed=1, depth=True):
    rng = np.random.Generator(np.random.PCG64(seed))
    g = rng.normal(0, 1, (3, H, W)).astype(np.float32)
    gd = rng.normal(0, 0.1, (1, H, W)).astype(np.float32) if depth else None
    return g, gd


# ----------------------------------------------------------------------------------------------------
# Synthetic dynamic hierarchy (.dhier layout)
# ----------------------------------------------------------------------------------------------------

def _morton3(p):
    lo, hi = p.min(0), p.max(0)
    q = ((p - lo) / np.maximum(hi - lo, 1e-9) * 1023).astype(np.uint64)

    def spread(v):
        v = v & np.uint64(0x3FF)
        v = (v | (v << np.uint64(16))) & np.uint64(0x30000FF)
        v = (v | (v << np.uint64(8))) & np.uint64(0x300F00F)
        v = (v | (v << np.uint64(4))) & np.uint64(0x30C30C3)
        v = (v | (v << np.uint64(2))) & np.uint64(0x9249249)
        return v

    return spread(q[:, 0]) | (spread(q[:, 1]) << np.uint64(1)) | (spread(q[:, 2]) << np.uint64(2))


def _quat_to_mat(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        np.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        np.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -2)


def _mat_to_quat(Rm):
    # robust per-element conversion (Shepperd)
    out = np.empty((Rm.shape[0], 4))
    tr = Rm[:, 0, 0] + Rm[:, 1, 1] + Rm[:, 2, 2]
    for i in range(Rm.shape[0]):
        m = Rm[i]
        if tr[i] > 0:
            s = math.sqrt(tr[i] + 1.0) * 2
            out[i] = [0.25 * s, (m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s]
        elif m[0, 0] > m[1, 1] and m[0, 0] > m[2, 2]:
            s = math.sqrt(1.0 + m[0, 0] - m[1, 1] - m[2, 2]) * 2
            out[i] = [(m[2, 1] - m[1, 2]) / s, 0.25 * s, (m[0, 1] + m[1, 0]) / s, (m[0, 2] + m[2, 0]) / s]
        elif m[1, 1] > m[2, 2]:
            s = math.sqrt(1.0 + m[1, 1] - m[0, 0] - m[2, 2]) * 2
            out[i] = [(m[0, 2] - m[2, 0]) / s, (m[0, 1] + m[1, 0]) / s, 0.25 * s, (m[1, 2] + m[2, 1]) / s]
        else:
            s = math.sqrt(1.0 + m[2, 2] - m[0, 0] - m[1, 1]) * 2
            out[i] = [(m[1, 0] - m[0, 1]) / s, (m[0, 2] + m[2, 0]) / s, (m[1, 2] + m[2, 1]) / s, 0.25 * s]
    return out / np.linalg.norm(out, axis=1, keepdims=True)


def make_dynamic_hierarchy(leaves, skybox_points=0, seed=0):
    """Binary hierarchy over `leaves` (a make_gaussians dict), built bottom-up by pairing Morton
    neighbours; parents are moment-matched.  Returns arrays in pre-order DFS with the node layout
    {depth, parent, child_count, first_child, next_sibling, max_side_length} (GH/types.h:60-67), node id ==
    Gaussian id, skybox rows (node fields -99) prepended as create_from_hier does
    (scene/gaussian_model.py:990-1095)."""
    means = leaves["means3D"].astype(np.float64)
    scales = leaves["scales"].astype(np.float64)
    rots = leaves["rotations"].astype(np.float64)
    opac = leaves["opacities"].reshape(-1).astype(np.float64)
    shs = leaves["shs"].astype(np.float64)
    n = means.shape[0]
    order = np.argsort(_morton3(means), kind="stable")
    # per-node arrays, appended level by level (index = build id)
    mu, cov, op, sh = [means[order]], [], [opac[order]], [shs[order]]
    Rm = _quat_to_mat(rots[order])
    S2 = scales[order] ** 2
    cov.append(np.einsum("nij,nj,nkj->nik", Rm, S2, Rm))
    children = [np.full((n, 2), -1, np.int64)]
    leaf_src = [order.astype(np.int64)]
    level = np.arange(n)
    offset = n
    while len(level) > 1:
        m_ = len(level) // 2
        a, b = level[0:2 * m_:2], level[1:2 * m_:2]
        MU, COV, OP, SH = np.concatenate(mu), np.concatenate(cov), np.concatenate(op), np.concatenate(sh)
        wa, wb = OP[a], OP[b]
        w = (wa + wb)[:, None]
        pm = (wa[:, None] * MU[a] + wb[:, None] * MU[b]) / w
        da, db = MU[a] - pm, MU[b] - pm
        pc = (wa[:, None, None] * (COV[a] + np.einsum("ni,nj->nij", da, da)) +
              wb[:, None, None] * (COV[b] + np.einsum("ni,nj->nij", db, db))) / w[:, :, None]
        mu.append(pm)
        cov.append(pc)
        op.append(np.maximum(wa, wb))
        sh.append(0.5 * (SH[a] + SH[b]))
        children.append(np.stack([a, b], 1))
        leaf_src.append(np.full(m_, -1, np.int64))
        new = np.arange(offset, offset + m_)
        offset += m_
        level = np.concatenate([new, level[2 * m_:]])
    MU, COV, OP, SH = np.concatenate(mu), np.concatenate(cov), np.concatenate(op), np.concatenate(sh)
    CH, SRC = np.concatenate(children), np.concatenate(leaf_src)
    G = MU.shape[0]
    root = int(level[0])
    # subtree sizes bottom-up (build order is topological: children have smaller ids)
    size = np.ones(G, np.int64)
    for i in range(n, G):
        size[i] = 1 + size[CH[i, 0]] + size[CH[i, 1]]
    # pre-order ids top-down
    pre = np.zeros(G, np.int64)
    depth = np.zeros(G, np.int64)
    parent = np.full(G, -1, np.int64)
    stack = [root]
    pre[root] = 0
    while stack:
        v = stack.pop()
        c0, c1 = CH[v]
        if c0 < 0:
            continue
        pre[c0] = pre[v] + 1
        pre[c1] = pre[v] + 1 + size[c0]
        depth[c0] = depth[c1] = depth[v] + 1
        parent[c0] = parent[c1] = v
        stack.extend([c0, c1])
    inv = np.empty(G, np.int64)
    inv[pre] = np.arange(G)
    ev, evec = np.linalg.eigh(COV)
    ev = np.maximum(ev, 1e-12)
    evec = evec * np.sign(np.linalg.det(evec))[:, None, None]
    q = _mat_to_quat(evec) if G <= 200000 else _mat_to_quat_fast(evec)
    nodes = np.zeros((G, 6), np.int64)
    nodes[pre, 0] = depth
    nodes[pre, 1] = np.where(parent >= 0, pre[np.maximum(parent, 0)], -1)
    nodes[pre, 2] = np.where(CH[:, 0] >= 0, 2, 0)
    nodes[pre, 3] = pre + 1
    nxt = np.zeros(G, np.int64)
    internal = np.where(CH[:, 0] >= 0)[0]
    nxt[CH[internal, 0]] = pre[CH[internal, 1]]
    nodes[pre, 4] = nxt
    nodes[pre, 5] = np.where(SRC >= 0, SRC, -1)
    out = dict(
        means3D=MU[inv].astype(np.float32), scales=np.sqrt(ev)[inv].astype(np.float32),
        rotations=q[inv].astype(np.float32), opacities=OP[inv].astype(np.float32)[:, None],
        shs=SH[inv].astype(np.float32), nodes=nodes.astype(np.int32), sh_degree=leaves.get("sh_degree", 0))
    if skybox_points:
        rng = np.random.Generator(np.random.PCG64(seed + 7))
        S = skybox_points
        d = rng.normal(0, 1, (S, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        sky = dict(means3D=(d * 80).astype(np.float32), scales=np.full((S, 3), 2.0, np.float32),
                   rotations=np.tile(np.array([1, 0, 0, 0], np.float32), (S, 1)),
                   opacities=np.full((S, 1), 0.9, np.float32),
                   shs=np.zeros((S,) + out["shs"].shape[1:], np.float32))
        # scene/gaussian_model.py:1059-1065
        nodes = out["nodes"].copy()
        nodes[:, 3] += S
        nodes[:, 1] += S
        nodes[nodes[:, 4] > 0, 4] += S
        nodes[0, 1] = -1
        nodes[:, 3] = np.where(nodes[:, 2] == 2, nodes[:, 3], 0)
        out = {k: (np.concatenate([sky[k], out[k]]) if k in sky else out[k]) for k in out}
        out["nodes"] = np.concatenate([np.full((S, 6), -99, np.int32), nodes.astype(np.int32)])
    out["skybox_points"] = skybox_points
    return out


def chunk_weight(pos, chunk_id, centers, falloff=0.05):
    """Per-Gaussian weight of chunk `chunk_id` (hierarchy_explicit_loader.cpp:22-52): 1 well inside the chunk's
    Voronoi cell, 0 beyond (1 + falloff) x the distance to the nearest other chunk centre, linear in between.
    pos (n,3), centers (C,3); float32 arithmetic as the loader's."""
    pos = np.asarray(pos, np.float32)
    c = np.asarray(centers, np.float32)
    d_cur = np.linalg.norm(pos - c[chunk_id], axis=1).astype(np.float32)
    others = [np.linalg.norm(pos - c[k], axis=1).astype(np.float32) for k in range(len(c)) if k != chunk_id]
    d_oth = np.min(np.stack(others), 0) if others else np.full(len(pos), 1e12, np.float32)
    f = np.float32(falloff)
    a = np.float32(-1.0) / (np.float32(2.0) * f * d_oth)
    b = (np.float32(1.0) + f) / (np.float32(2.0) * f)
    w = np.where(d_cur <= (1 - f) * d_oth, np.float32(1.0),
                 np.where(d_cur > (1 + f) * d_oth, np.float32(0.0), a * d_cur + b))
    return w.astype(np.float32)


def make_merged_hierarchy(chunks, centers, seed=0, root_scale=1e4):
    """A multi-chunk hierarchy merged under one root, as mainHierarchyMerger.cpp:94-140 builds it, in the dynamic
    (.dhier) node layout of make_dynamic_hierarchy.  chunks: one make_gaussians dict per chunk (its leaves);
    centers (C,3): the chunk centres (center.txt).

    Per chunk (HierarchyExplicitLoader::loadExplicit, hierarchy_explicit_loader.cpp:54-150): every Gaussian is
    weighted by chunk_weight, dropped at weight 0, and its opacity scaled by the weight; the chunk's tree is built
    over what is left (make_dynamic_hierarchy) and its root moved to the chunk centre (pos[0] = chunk_center).
    The merge (mainHierarchyMerger.cpp:111-134) hangs the chunk roots under a new root whose size is set so that
    no cut ever selects it (bounds[3] = 1e9 there; here its scales are `root_scale`, so max(scale)/distance exceeds
    any threshold and the chunk roots get interpolation weight 1).  Node ids are pre-order: the root, then chunk
    0's subtree, then chunk 1's, ..."""
    subs = []
    for k, leaves in enumerate(chunks):
        w = chunk_weight(leaves["means3D"], k, centers)
        keep = w > 0
        kept = {key: (v[keep] if isinstance(v, np.ndarray) and v.shape[:1] == w.shape else v)
                for key, v in leaves.items()}
        kept["opacities"] = (kept["opacities"].reshape(-1) * w[keep]).astype(np.float32)[:, None]
        h = make_dynamic_hierarchy(kept, seed=seed + k)
        h["means3D"] = h["means3D"].copy()
        h["means3D"][0] = np.asarray(centers[k], np.float32)
        subs.append(h)
    sizes = [h["nodes"].shape[0] for h in subs]
    G = 1 + sum(sizes)
    nodes = np.zeros((G, 6), np.int32)
    nodes[0] = (0, -1, len(subs), 1, 0, -1)
    out = {k: [] for k in ("means3D", "scales", "rotations", "opacities", "shs")}
    roots = []
    off = 1
    for k, h in enumerate(subs):
        n = h["nodes"].copy()
        n[:, 0] += 1
        n[:, 1] = np.where(n[:, 1] >= 0, n[:, 1] + off, 0)
        n[:, 3] = np.where(n[:, 2] > 0, n[:, 3] + off, 0)
        n[:, 4] = np.where(n[:, 4] > 0, n[:, 4] + off, 0)
        n[0, 4] = off + sizes[k] if k + 1 < len(subs) else 0
        nodes[off:off + sizes[k]] = n
        roots.append(off)
        for key in out:
            out[key].append(h[key])
        off += sizes[k]
    cat = {key: np.concatenate(v) for key, v in out.items()}
    w = np.array([float(cat["opacities"][r - 1, 0]) for r in roots])
    cm = (w[:, None] * np.stack([cat["means3D"][r - 1] for r in roots])).sum(0) / max(w.sum(), 1e-12)
    root = dict(means3D=cm.astype(np.float32)[None], scales=np.full((1, 3), root_scale, np.float32),
                rotations=np.array([[1, 0, 0, 0]], np.float32), opacities=np.array([[w.max()]], np.float32),
                shs=np.mean(np.stack([cat["shs"][r - 1] for r in roots]), 0, keepdims=True).astype(np.float32))
    res = {key: np.concatenate([root[key], cat[key]]) for key in out}
    res["nodes"] = nodes
    res["sh_degree"] = chunks[0].get("sh_degree", 0)
    res["skybox_points"] = 0
    res["chunk_roots"] = np.array(roots, np.int32)
    return res


def _mat_to_quat_fast(Rm):
    """Vectorised branch-free variant for large trees (same convention as _mat_to_quat)."""
    m = Rm
    w = np.sqrt(np.maximum(0, 1 + m[:, 0, 0] + m[:, 1, 1] + m[:, 2, 2])) / 2
    x = np.sqrt(np.maximum(0, 1 + m[:, 0, 0] - m[:, 1, 1] - m[:, 2, 2])) / 2
    y = np.sqrt(np.maximum(0, 1 - m[:, 0, 0] + m[:, 1, 1] - m[:, 2, 2])) / 2
    z = np.sqrt(np.maximum(0, 1 - m[:, 0, 0] - m[:, 1, 1] + m[:, 2, 2])) / 2
    x = np.copysign(x, m[:, 2, 1] - m[:, 1, 2])
    y = np.copysign(y, m[:, 0, 2] - m[:, 2, 0])
    z = np.copysign(z, m[:, 1, 0] - m[:, 0, 1])
    q = np.stack([w, x, y, z], 1)
    return q / np.linalg.norm(q, axis=1, keepdims=True)

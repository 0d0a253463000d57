"""train_post.py's SPT cache (Cache_SPTs=True) on the HIP path.

The reference keeps every Gaussian in host storage (GaussianModel.move_storage_to, scene/gaussian_model.py
:430-460) and, per training view, keeps on the GPU only the Gaussians of the SPTs the view cuts:

  setup                  train_post.py:208-231  (skybox resident, empty SPT state)
  coarse cut             :326-343  -> hlgs_upper_tree_cut_device (k_upper_cut + k_cut_level), its length read
                                      on the device by the plan
  bookkeeping            :346-430  -> hlgs_spt_cache_plan (k_cache_lists + two scans + k_cache_split), with
                                      get_spt_cut_cuda on the SPTs to load
  write-back and load    :439-479  -> three launches move all six parameters and their twelve Adam moments:
                                      write-back with hlgs_copy_rows_packed, resident compaction with
                                      hlgs_copy_rows, load with hlgs_load_rows_packed (rows the write-back has
                                      just stored and the step loads again come from their resident rows).  The host side is pinned memory the GPU reads and writes
                                      directly, one packed row per Gaussian (all eighteen rows back to back,
                                      padded to whole 64-byte lines), so the host link carries whole lines
  optimizer step         :786-812  -> hlgs_adam_step (one launch over the six tensors, skybox gradients zeroed)

  occlusion cull         :344-351  -> optional (occlusion_culling=True, train_post.py's Use_Occlusion_Culling, off by
                                      default there, :83): the coarse cut's upper-tree Gaussians are read from host
                                      storage and rendered, and the cut keeps the ones the render reports (below)

Differences from the reference: when the Gaussian budget forces a second pass, each pass
starts again from the step's initial state with the larger distance multiplier (the reference's second pass
reads state its first pass already replaced and then fails on mismatched masks).

Occlusion culling as the reference runs it (gaussian_renderer/__init__.py:24-33, render_on_disk :163-232): the
Gaussians of the coarse cut's nodes (upper_tree_nodes[:, 5]) are taken from storage with the activations applied
(sigmoid opacity clamped to [0, 1], exp scale, normalised rotation, SH degree 3), rendered without depth on a black
background, and the cut keeps the nodes whose `seen` is set -- where `seen` is the second value the reference's
GaussianRasterizer returns, i.e. the radii (render_on_disk unpacks `rendered_image, seen, depth`): a node stays when
its Gaussian has a non-zero screen radius (in front of the near plane, on screen).  With a batch of views a node
stays when any view keeps it.
"""
import ctypes as C
import math

import torch

from hlgs_core import _lib as L
from hlgs_core import spt as _spt

NAMES = ("xyz", "f_dc", "opacity", "scaling", "rotation", "f_rest")


def _p(t):
    return t.data_ptr() if t is not None and t.numel() else None


def _row_bytes(t):
    return t.element_size() * math.prod(t.shape[1:])


def copy_rows(pairs, n, src_rows=None, dst_rows=None):
    """dst[dst_rows[i]] = src[src_rows[i]] for every (src, dst) pair, one launch (hlgs_copy_rows)."""
    lib = L.load()
    if n == 0 or not pairs:
        return
    tabs = (L.RowCopy * len(pairs))()
    for k, (src, dst) in enumerate(pairs):
        for t in (src, dst):
            if not t.is_contiguous():
                raise RuntimeError("row storage must be contiguous")
            if t.device.type == "cpu" and not t.is_pinned():
                raise RuntimeError("host storage must be pinned (tensor.pin_memory()) for direct GPU access")
        rb = _row_bytes(src)
        if rb != _row_bytes(dst) or src.dtype != dst.dtype:
            raise RuntimeError("source and destination rows differ")
        tabs[k] = L.RowCopy(src.data_ptr(), dst.data_ptr(), rb)
    L.check(lib.hlgs_copy_rows(len(pairs), tabs, int(n), _p(src_rows), _p(dst_rows), L.stream()))


def copy_rows_packed(dev_tables, n, dev_rows, host_rows, host, to_host):
    """Host legs with packed host storage (hlgs_copy_rows_packed): host[host_rows[i]] holds the rows of every
    device table back to back; to_host writes whole host rows from dev_t[dev_rows[i]], else the tables' parts are
    read back into dev_t[dev_rows[i]].  None row lists are the identity."""
    lib = L.load()
    if n == 0 or not dev_tables:
        return
    if host.device.type != "cpu" or not host.is_pinned() or not host.is_contiguous():
        raise RuntimeError("packed host storage must be a contiguous pinned tensor")
    tabs = (L.RowCopy * len(dev_tables))()
    for k, d in enumerate(dev_tables):
        if not d.is_contiguous() or d.dtype != torch.float32:
            raise RuntimeError("device tables must be contiguous float32")
        L.require_gpu(d)
        tabs[k] = L.RowCopy(d.data_ptr(), None, _row_bytes(d))
    L.check(lib.hlgs_copy_rows_packed(len(dev_tables), tabs, int(n), _p(dev_rows), _p(host_rows), host.data_ptr(),
                                      host.stride(0) * host.element_size(), 1 if to_host else 0, L.stream()))


def load_rows_packed(dst_tables, n, host_rows, host, resident_tables=None, resident_of=None):
    """Load leg (hlgs_load_rows_packed): dst_t[i] = the table's part of host[host_rows[i]], except rows with
    resident_of[host_rows[i]] = r >= 0, which are copied from resident_tables[t][r] on the device."""
    lib = L.load()
    if n == 0 or not dst_tables:
        return
    if host.device.type != "cpu" or not host.is_pinned() or not host.is_contiguous():
        raise RuntimeError("packed host storage must be a contiguous pinned tensor")
    tabs = (L.RowCopy * len(dst_tables))()
    res = resident_tables if resident_of is not None else [None] * len(dst_tables)
    for k, (d, r) in enumerate(zip(dst_tables, res)):
        for t in (d,) if r is None else (d, r):
            if not t.is_contiguous() or t.dtype != torch.float32:
                raise RuntimeError("device tables must be contiguous float32")
            L.require_gpu(t)
        tabs[k] = L.RowCopy(_p(r) if r is not None else None, d.data_ptr(), _row_bytes(d))
    L.check(lib.hlgs_load_rows_packed(len(dst_tables), tabs, int(n), _p(host_rows), _p(resident_of), host.data_ptr(),
                                      host.stride(0) * host.element_size(), L.stream()))


def adam_step(params, grads, exp_avgs, exp_avg_sqs, lrs, step, skybox_points=0, beta1=0.9, beta2=0.999, eps=1e-8):
    """The dense Adam of train_post.py:786-812 over a list of float32 tensors (in place, one launch): grads of
    the first skybox_points rows are zeroed, then OurAdam._single_tensor_adam2 with state step `step` (the
    reference passes torch.tensor(iteration) and increments it, so step = iteration + 1)."""
    lib = L.load()
    ts = (L.AdamTensor * len(params))()
    for k, (p, g, m, v, lr) in enumerate(zip(params, grads, exp_avgs, exp_avg_sqs, lrs)):
        for t in (p, g, m, v):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != p.numel():
                raise RuntimeError("Adam tensors must be contiguous float32 of the parameter's size")
        L.require_gpu(p, g, m, v)
        rows = p.size(0) if p.dim() else 1
        ts[k] = L.AdamTensor(_p(p), _p(g), _p(m), _p(v), p.numel(), p.numel() // rows if rows else 0, float(lr))
    L.check(lib.hlgs_adam_step(len(params), ts, int(step), int(skybox_points), float(beta1), float(beta2), float(eps),
                               L.stream()))


def gather_views(full_proj_transform, camera_center, group=None):
    """Every rank's training view, in rank order: (G, 4, 4) projection matrices and (G, 3) camera centres.

    The view-data-parallel config #5 step: each rank trains its own view, and every rank passes the
    gathered batch to SPTCache.step, so all ranks compute the same union cut from the same inputs and hold the same
    resident set in the same order -- the gradient all-reduce over SPTCache.params is then elementwise, and the
    replicated Adam step keeps the replicas identical.  One small all_gather (19 floats per rank)."""
    import torch.distributed as dist
    fpt = full_proj_transform.detach().reshape(-1)[:16].float()
    cam = camera_center.detach().reshape(-1)[:3].float()
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return fpt.reshape(1, 4, 4), cam.reshape(1, 3)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else \
        torch.device("cpu")
    v = torch.cat([fpt, cam]).to(dev)
    out = [torch.empty_like(v) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, v, group=group)
    st = torch.stack(out)
    return st[:, :16].reshape(-1, 4, 4).contiguous(), st[:, 16:19].contiguous()


class SPTCache:
    """Resident set of a cached training run.  storage: dict name -> host tensor of all Gaussians (rows), for
    the names in NAMES; opt_storage: dict name -> {"exp_avgs", "exp_avgs_sqs"} of the same shapes (zero-filled
    when None).  Host tensors are pinned here if they are not already.  spt: build_hierarchical_spt's dict.

    After step(), `params`, `exp_avgs` and `exp_avg_sqs` (dicts of device tensors) hold the resident rows in
    render_indices order, as the reference's parameter list does."""

    def __init__(self, storage, spt, skybox_points, opt_storage=None, reuse_tolerance=0.9,
                 max_gaussian_budget=100_000_000, distance_multiplier_until_budget=1.5, use_frustum_culling=True,
                 use_bounding_spheres=True, device="cuda", occlusion_culling=False, flat_cut=True):
        # packed pinned host storage: one row per Gaussian holding its six parameter rows, then the six exp_avgs and
        # the six exp_avg_sqs rows, padded to whole 64-byte lines; self.storage / self.opt_storage are views of it
        G = int(storage[NAMES[0]].shape[0])
        shapes = {k: tuple(storage[k].shape[1:]) for k in NAMES}
        widths = [math.prod(shapes[k]) for k in NAMES] * 3
        hw = -(-sum(widths) // 16) * 16
        self.host = torch.zeros((G, hw), dtype=torch.float32, pin_memory=True)  # pinned at allocation: no pageable copy
        offs = [sum(widths[:i]) for i in range(len(widths))]
        view = lambda i, k: self.host[:, offs[i]:offs[i] + widths[i]].view((G,) + shapes[k])  # noqa: E731
        self.storage = {k: view(i, k) for i, k in enumerate(NAMES)}
        self.opt_storage = {k: {"exp_avgs": view(len(NAMES) + i, k), "exp_avgs_sqs": view(2 * len(NAMES) + i, k)}
                            for i, k in enumerate(NAMES)}
        for k in NAMES:
            self.storage[k].copy_(storage[k].reshape((G,) + shapes[k]))
            if opt_storage is not None:
                self.opt_storage[k]["exp_avgs"].copy_(opt_storage[k]["exp_avgs"].reshape((G,) + shapes[k]))
                self.opt_storage[k]["exp_avgs_sqs"].copy_(opt_storage[k]["exp_avgs_sqs"].reshape((G,) + shapes[k]))
        self.device = torch.device(device)
        dev = self.device
        self.nodes = spt["upper_tree_nodes"].to(dev, torch.int32).contiguous()
        # the upper tree's walk order for the flat coarse cut (hlgs_upper_tree_order), or None for the level walk
        self.cut_order = _spt.upper_tree_order(spt["upper_tree_nodes"], dev) if flat_cut else None
        self.xyz = spt["upper_tree_xyz"].to(dev, torch.float32).contiguous()
        self.min_distance_squared = spt["min_distance_squared"].to(dev, torch.float32).contiguous()
        if use_bounding_spheres:
            self.bounds = spt["bounding_sphere_radii"].to(dev, torch.float32).contiguous()
        else:  # scaling_activation(max(upper_tree_scaling)) * 3.0 (train_post.py:330)
            self.bounds = (torch.exp(torch.max(spt["upper_tree_scaling"].to(dev, torch.float32), dim=-1)[0]) * 3.0)
        self.spt_starts = spt["SPT_starts"].to(dev, torch.int32).contiguous()
        self.spt_max = spt["SPT_max"].to(dev, torch.float32).contiguous()
        self.spt_min = spt["SPT_min"].to(dev, torch.float32).contiguous()
        self.spt_gidx = spt["SPT_gaussian_indices"].to(dev, torch.int32).contiguous()
        self.num_spts = int(self.spt_starts.numel()) - 1
        self.sky = int(skybox_points)
        self.rtol, self.atol = float(reuse_tolerance), 0.05
        self.budget = max_gaussian_budget
        self.dm_step = distance_multiplier_until_budget
        self.use_frustum = use_frustum_culling
        self.occlusion = bool(occlusion_culling)
        self.last_occlusion = None  # the last occlusion cull's inputs and mask (tests)
        # setup, train_post.py:208-231
        self.render_indices = torch.arange(0, self.sky, device=dev, dtype=torch.int32)
        head = torch.arange(0, self.sky, device=dev, dtype=torch.int32)
        self.params = {k: self._alloc(k, self.sky) for k in NAMES}
        copy_rows_packed([self.params[k] for k in NAMES], self.sky, None, head, self.host, to_host=False)
        self.exp_avgs = {k: torch.zeros_like(self.params[k]) for k in NAMES}
        self.exp_avg_sqs = {k: torch.zeros_like(self.params[k]) for k in NAMES}
        # per storage row: the resident row holding it while a step's write-back and load run, else -1
        self.resident_of = torch.full((G,), -1, dtype=torch.int32, device=dev)
        # the write-back crosses the host link on its own stream, beside the compaction, the load and the rest of
        # the training step; the next step's load waits for it (wb_done)
        self.wb_stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self.wb_done = None
        self._wb_hold = None
        self._wb_pending = None  # this step's write-back, launched when the next step starts (_flush_write_back)
        self._row_shapes = self._widths = None  # per resident tensor: row shape and floats per row (fixed)
        self._cut = self._cut_scratch = self._cut_count = None
        self.prev_SPT_indices = torch.empty(0, dtype=torch.int32, device=dev)
        self.prev_SPT_distances = torch.empty(0, dtype=torch.float32, device=dev)
        self.prev_SPT_counts = torch.empty(0, dtype=torch.int32, device=dev)
        self.n_loaded = 0
        self.last_plan = None

    def _alloc(self, k, rows):
        return torch.empty((rows,) + tuple(self.storage[k].shape[1:]), dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------ bookkeeping (:326-430)
    def _occlusion_cull(self, views):
        """Filter the device coarse cut (self._cut, length in self._cut_count[0]) as train_post.py:344-351 does."""
        from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
        dev = self.device
        n = int(self._cut_count[0].item())
        cut = self._cut[:n]
        gid = self.nodes[cut.long(), 5].contiguous()
        if self.wb_done is not None:  # storage as the previous steps' write-backs left it
            torch.cuda.current_stream(dev).wait_event(self.wb_done)
        rows = {k: self._alloc(k, n) for k in NAMES}
        load_rows_packed([rows[k] for k in NAMES], n, gid, self.host)
        means = rows["xyz"]
        opac = torch.clamp(torch.sigmoid(rows["opacity"]), 0, 1)
        scales = torch.exp(rows["scaling"])
        rots = torch.nn.functional.normalize(rows["rotation"])
        shs = torch.cat((rows["f_dc"], rows["f_rest"]), dim=1).contiguous()
        keep = torch.zeros(n, dtype=torch.bool, device=dev)
        with torch.no_grad():
            for v in views:
                rs = GaussianRasterizationSettings(
                    image_height=int(v["H"]), image_width=int(v["W"]), tanfovx=float(v["tanfovx"]),
                    tanfovy=float(v["tanfovy"]), bg=torch.zeros(3, device=dev), scale_modifier=1.0,
                    viewmatrix=v["viewmatrix"].to(dev), projmatrix=v["projmatrix"].to(dev), sh_degree=3,
                    campos=v["campos"].to(dev), prefiltered=False, debug=True,
                    render_indices=torch.empty(0, dtype=torch.int32, device=dev),
                    parent_indices=torch.empty(0, dtype=torch.int32, device=dev),
                    interpolation_weights=torch.empty(0, device=dev),
                    num_node_kids=torch.empty(0, dtype=torch.int32, device=dev), do_depth=False)
                _, radii, _ = GaussianRasterizer(rs)(means3D=means, means2D=torch.zeros_like(means), opacities=opac,
                                                     shs=shs, scales=scales, rotations=rots)
                keep |= radii > 0
        kept = cut[keep]
        self._cut[:kept.numel()] = kept
        self._cut_count[0] = kept.numel()
        self.last_occlusion = dict(indices=gid, means3D=means, opacities=opac, scales=scales, rotations=rots, shs=shs,
                                   keep=keep, n_before=n, n_after=int(kept.numel()))

    def plan(self, full_proj_transform, camera_center, distance_multiplier=1.0, views=None):
        """One bookkeeping pass for a view; no parameter moves.  Returns the reference's per-pass variables.

        A batch of G views (full_proj_transform G x 4 x 4, camera_center G x 3; one view per rank of a
        view-data-parallel step) gives the union cut: visible in any frustum, each LOD decision and SPT
        distance taken from the nearest camera.  With one view it is the reference's cut, bit for bit."""
        lib = L.load()
        dev = self.device
        fpt = full_proj_transform.detach().to(dev, torch.float32)
        G = fpt.shape[0] if fpt.dim() == 3 else 1
        fpt = fpt.reshape(G, 4, 4)
        cam = camera_center.detach().to(dev, torch.float32).reshape(G, -1)[:, :3].contiguous()
        planes = (torch.stack([_spt.extract_frustum_planes(fpt[g]) for g in range(G)]).contiguous()
                  if self.use_frustum else None)
        # coarse cut with its length left on the device (hlgs_upper_tree_cut_device): the plan reads it, so the step
        # has one host synchronisation, the plan's
        N = self.nodes.size(0)
        if self._cut is None:
            self._cut = torch.empty((max(N, 1),), dtype=torch.int32, device=dev)
            self._cut_scratch = torch.empty(lib.hlgs_upper_cut_scratch_size(N), dtype=torch.uint8, device=dev)
            self._cut_count = torch.zeros((2,), dtype=torch.int32, device=dev)
        L.check(lib.hlgs_upper_tree_cut_views_ordered_device(
            N, _p(self.nodes), _p(self.cut_order), _p(self.xyz), _p(self.bounds), _p(self.min_distance_squared), G,
            _p(planes), _p(cam), float(distance_multiplier), int(bool(self.use_frustum)), 1, _p(self._cut_scratch),
            _p(self._cut), _p(self._cut_count), L.stream()))
        if self.occlusion:
            if views is None:
                raise ValueError("occlusion culling renders the cut: pass the view(s) (W, H, tanfovx, tanfovy, "
                                 "viewmatrix, projmatrix, campos) to step()")
            self._occlusion_cull(views if isinstance(views, (list, tuple)) else [views])
        coarse = self._cut
        n_cut, m, R = N, self.prev_SPT_indices.numel(), self.render_indices.numel()
        # the ten output lists carved from one int32 allocation (the distances as float32 views of it)
        sizes = dict(keep_spt_indices=m, keep_spt_distances=m, keep_spt_counts=m, load_spt_indices=n_cut,
                     load_spt_distances=n_cut, upper_render=n_cut, keep_rows=R, render_kept=R, write_back_rows=R,
                     write_back_indices=R)
        lens = [(max(n, 1) + 63) // 64 * 64 for n in sizes.values()]
        flat = torch.empty(sum(lens), dtype=torch.int32, device=dev)
        out = {}
        for (k, n), part in zip(sizes.items(), flat.split(lens)):
            out[k] = part[:max(n, 1)].view(torch.float32) if k.endswith("distances") else part[:max(n, 1)]
        a = L.CacheArgs(n_cut, _p(coarse), _p(self.nodes), _p(self.xyz), _p(cam), float(distance_multiplier),
                        self.num_spts, m, _p(self.prev_SPT_indices), _p(self.prev_SPT_distances),
                        _p(self.prev_SPT_counts), R, _p(self.render_indices), int(self.n_loaded), self.sky,
                        self.rtol, self.atol, _p(self._cut_count), G)
        pl = L.CachePlan(*[out[f].data_ptr() for f, _ in L.CachePlan._fields_[:10]])
        scratch = torch.empty(lib.hlgs_spt_cache_scratch_size(n_cut, m, R, self.num_spts), dtype=torch.uint8,
                              device=dev)
        L.check(lib.hlgs_spt_cache_plan(C.byref(a), C.byref(pl), scratch.data_ptr(), L.stream()))
        nk, nl, nu, nkr, prefix = pl.n_kept, pl.n_load, pl.n_upper, pl.n_keep_rows, pl.prefix
        load_idx, load_dist = out["load_spt_indices"][:nl], out["load_spt_distances"][:nl]
        if nl > 0:
            import gaussian_hierarchy._C as GHC
            cut_spts, spt_counts = GHC.get_spt_cut_cuda(nl, self.spt_gidx, self.spt_starts, self.spt_max,
                                                        self.spt_min, load_idx, load_dist)
        else:
            cut_spts = torch.empty(0, dtype=torch.int32, device=dev)
            spt_counts = torch.empty(0, dtype=torch.int32, device=dev)
        load_from_disk = torch.cat([cut_spts, out["upper_render"][:nu]])
        return dict(
            SPT_indices=torch.cat([out["keep_spt_indices"][:nk], load_idx]),
            SPT_distances=torch.cat([out["keep_spt_distances"][:nk], load_dist]),
            SPT_counts=torch.cat([out["keep_spt_counts"][:nk], spt_counts + (self.sky + prefix)]),
            keep_rows=out["keep_rows"][:nkr], write_back_rows=out["write_back_rows"][:R - nkr],
            write_back_indices=out["write_back_indices"][:R - nkr], load_from_disk_indices=load_from_disk,
            render_indices=torch.cat([out["render_kept"][:nkr], load_from_disk]), n_kept=nk,
            load_SPT_indices=load_idx, upper_tree_nodes_to_render=out["upper_render"][:nu], prefix=prefix,
            distance_multiplier=distance_multiplier)

    # ------------------------------------------------------------ one view (:326-483), or a batch of views
    def step(self, full_proj_transform, camera_center, views=None):
        """views: the camera(s) of this step as dicts (W, H, tanfovx, tanfovy, viewmatrix, projmatrix, campos), needed
        only with occlusion_culling (the cull renders the cut's upper-tree Gaussians)."""
        # the previous step's write-back crosses the host link now, beside this step's coarse cut and bookkeeping (the
        # GPU is mostly idle there, waiting on host work); its rows are read again at the earliest by this step's load
        self._flush_write_back()
        dm = 1.0
        while True:
            pl = self.plan(full_proj_transform, camera_center, dm, views)
            if pl["render_indices"].numel() <= self.budget:
                break
            dm *= self.dm_step
        self._move(pl)
        self.prev_SPT_indices = pl["SPT_indices"]
        self.prev_SPT_distances = pl["SPT_distances"]
        self.prev_SPT_counts = pl["SPT_counts"]
        self.render_indices = pl["render_indices"]
        self.n_loaded = pl["load_from_disk_indices"].numel()
        self.last_plan = pl
        return self.render_indices

    def _move(self, pl):
        dev_t = [self.params[k] for k in NAMES] + [self.exp_avgs[k] for k in NAMES] + \
                [self.exp_avg_sqs[k] for k in NAMES]
        wb = pl["write_back_rows"]
        cur = torch.cuda.current_stream(self.device)
        prev_wb, prev_hold = self.wb_done, self._wb_hold
        nk = pl["keep_rows"].numel()
        load = pl["load_from_disk_indices"]
        rows = nk + load.numel()
        # the eighteen new resident tensors carved from one allocation (each 256-byte aligned).  The compaction of the
        # rows that stay (:446-479) is launched from the raw addresses first, and the eighteen tensor views are made
        # while it runs: the views cost ~50 torch calls of host time, which the GPU otherwise waited through.
        if self._row_shapes is None:
            self._row_shapes = [tuple(d.shape[1:]) for d in dev_t]
            self._widths = [math.prod(sh) for sh in self._row_shapes]
        widths = self._widths
        lens = [(rows * w + 63) // 64 * 64 for w in widths]
        flat = torch.empty(sum(lens), dtype=torch.float32, device=self.device)
        if nk:
            base, off = flat.data_ptr(), 0
            tabs = (L.RowCopy * len(dev_t))()
            for k, (d, w, ln) in enumerate(zip(dev_t, widths, lens)):
                tabs[k] = L.RowCopy(d.data_ptr(), base + 4 * off, 4 * w)
                off += ln
            L.check(L.load().hlgs_copy_rows(len(dev_t), tabs, nk, _p(pl["keep_rows"]), None, L.stream()))
        new_t = [part[:rows * w].view((rows,) + sh) for part, w, sh in zip(flat.split(lens), widths, self._row_shapes)]
        # rows written back above and loaded again (the upper-tree Gaussians, every step) come from their resident
        # rows, the rest over the host link once the previous step's write-back has landed
        if prev_wb is not None:
            cur.wait_event(prev_wb)
            del prev_hold
        if wb.numel():
            wbi = pl["write_back_indices"].long()
            self.resident_of[wbi] = wb
            load_rows_packed([n[nk:] for n in new_t], load.numel(), load, self.host, [d.detach() for d in dev_t],
                             self.resident_of)
            # index_fill_ takes the scalar as a kernel argument; `resident_of[wbi] = -1` copied a CPU scalar tensor
            # to the device first, a synchronous copy that waited for the compaction and the load (~100 us per step)
            self.resident_of.index_fill_(0, wbi, -1)
        else:
            load_rows_packed([n[nk:] for n in new_t], load.numel(), load, self.host)
        # the evicted rows go back to storage (:439-444, :473-474) on the write-back stream when the next step starts
        # (_flush_write_back), or earlier where the training loop calls flush_write_back().  Their values are final:
        # these tensors are no longer trained.  A write-back writing over the host link slows whatever kernel runs
        # beside it (at 128 workgroups: the compaction 185 -> 280 us, the rasterizer's preprocess 73 -> 190-240 us),
        # so it runs on a small grid (csrc/stream.hip) and not beside the compaction.  Nothing in this step reads
        # those host rows (the rows it loads again came from their resident rows, above); the next step's load waits
        # for it (wb_done).
        if wb.numel():
            self._wb_pending = (dev_t, wb, pl["write_back_indices"])
        k6 = len(NAMES)
        self.params = {k: new_t[i].requires_grad_(True) for i, k in enumerate(NAMES)}
        self.exp_avgs = {k: new_t[k6 + i] for i, k in enumerate(NAMES)}
        self.exp_avg_sqs = {k: new_t[2 * k6 + i] for i, k in enumerate(NAMES)}

    def flush_write_back(self):
        """Launch the pending write-back of the last step() on the write-back stream, behind everything queued on the
        current stream so far (wb_done marks its end).  Optional: the next step() (or sync_storage()) launches it
        otherwise.  A training loop can call it where the GPU runs compute-bound work, e.g. just before
        loss.backward(), whose blend backward is bound by VALU issue rather than by memory."""
        self._flush_write_back()

    def _flush_write_back(self):
        """Launch the pending write-back of the last step on the write-back stream (behind everything queued on the
        current stream so far); wb_done marks its end."""
        if self._wb_pending is None:
            return
        dev_t, wb, idx = self._wb_pending
        self._wb_pending = None
        cur = torch.cuda.current_stream(self.device)
        self.wb_stream.wait_stream(cur)
        with torch.cuda.stream(self.wb_stream):
            copy_rows_packed([d.detach() for d in dev_t], wb.numel(), wb, idx, self.host, to_host=True)
            self.wb_done = torch.cuda.Event()
            self.wb_done.record(self.wb_stream)
        # the write-back's inputs stay referenced until a later step has waited for it (then their memory may go
        # back to this stream's allocations)
        self._wb_hold = (dev_t, wb, idx)

    def sync_storage(self):
        """Wait until the last write-back has landed in host storage.  Call before reading self.storage /
        self.opt_storage on the host (the reference's write-back is a synchronous .cpu() copy)."""
        self._flush_write_back()
        if self.wb_done is not None:
            self.wb_done.synchronize()

    # ------------------------------------------------------------ optimizer step (:786-812)
    def optimizer_step(self, iteration, lrs):
        """lrs: dict name -> learning rate.  Uses the gradients autograd left on self.params."""
        ps = [self.params[k] for k in NAMES]
        for p in ps:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        with torch.no_grad():
            adam_step([p.data for p in ps], [p.grad for p in ps], [self.exp_avgs[k] for k in NAMES],
                      [self.exp_avg_sqs[k] for k in NAMES], [lrs[k] for k in NAMES], int(iteration) + 1, self.sky)

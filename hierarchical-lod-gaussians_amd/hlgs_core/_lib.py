"""ctypes binding of libhlgs.so (include/hlgs.h).

The library is the only compute path: if it is missing, or no GPU is present, calls raise -- there is
no CPU fallback.  Tensors cross the boundary as raw device pointers taken from torch; work runs on
torch's current HIP stream.
"""
import ctypes as C
import os

import torch

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("HLGS_LIBRARY") or os.path.join(PKG_DIR, "lib", "libhlgs.so")  # HLGS_LIBRARY: an alternative in-tree build (experiments)
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "hlgs.h")

_vp = C.c_void_p
_i = C.c_int
_f = C.c_float
_sz = C.c_size_t


class RasterArgs(C.Structure):
    _fields_ = [("P", _i), ("P_full", _i), ("D", _i), ("M", _i), ("W", _i), ("H", _i),
                ("bg", _vp), ("means3D", _vp), ("shs", _vp), ("colors_precomp", _vp), ("opacities", _vp),
                ("scales", _vp), ("rotations", _vp), ("cov3D_precomp", _vp), ("viewmatrix", _vp),
                ("projmatrix", _vp), ("campos", _vp), ("scale_modifier", _f), ("tanfovx", _f), ("tanfovy", _f),
                ("indices", _vp), ("parent_indices", _vp), ("ts", _vp), ("kids", _vp), ("prefiltered", _i),
                ("debug", _i), ("dc", _vp), ("antialiasing", _i), ("variant", _i)]


VARIANT_HIERARCHY = 0
VARIANT_ALT = 1


class Grads(C.Structure):
    _fields_ = [("dmean2D", _vp), ("dcolor", _vp), ("dopacity", _vp), ("dmean3D", _vp), ("dcov3D", _vp),
                ("dsh", _vp), ("dscale", _vp), ("drot", _vp), ("ddc", _vp), ("drgb", _vp)]


class HierInfo(C.Structure):
    _fields_ = [("format", _i), ("G", _i), ("N", _i), ("sh_degree", _i)]


class FrameInfo(C.Structure):
    _fields_ = [("num_rendered", _i), ("max_tile_count", _i), ("rendered", _i), ("num_binned", _i),
                ("entry_shift", _i), ("drops_empty", _i)]


class CacheArgs(C.Structure):
    _fields_ = [("n_cut", _i), ("cut", _vp), ("upper_nodes", _vp), ("upper_xyz", _vp), ("campos", _vp),
                ("distance_multiplier", _f), ("num_spts", _i), ("m", _i), ("prev_spt_indices", _vp),
                ("prev_spt_distances", _vp), ("prev_spt_counts", _vp), ("R", _i), ("render_indices", _vp),
                ("n_loaded_prev", _i), ("skybox_points", _i), ("rtol", _f), ("atol", _f), ("n_cut_device", _vp),
                ("n_views", _i)]


class CachePlan(C.Structure):
    _fields_ = [("keep_spt_indices", _vp), ("keep_spt_distances", _vp), ("keep_spt_counts", _vp),
                ("load_spt_indices", _vp), ("load_spt_distances", _vp), ("upper_render", _vp), ("keep_rows", _vp),
                ("render_kept", _vp), ("write_back_rows", _vp), ("write_back_indices", _vp), ("n_kept", _i),
                ("n_load", _i), ("n_upper", _i), ("n_keep_rows", _i), ("prefix", _i)]


class RowCopy(C.Structure):
    _fields_ = [("src", _vp), ("dst", _vp), ("row_bytes", C.c_int64)]


class AdamTensor(C.Structure):
    _fields_ = [("param", _vp), ("grad", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp), ("numel", C.c_int64),
                ("row_elems", C.c_int64), ("lr", C.c_double)]


_SIGS = {
    "hlgs_last_error": (C.c_char_p, []),
    "hlgs_version": (C.c_char_p, []),
    "hlgs_geom_buffer_size": (_sz, [_i]),
    "hlgs_image_buffer_size": (_sz, [_i, _i]),
    "hlgs_binning_buffer_size": (_sz, [_i]),
    "hlgs_backward_scratch_size": (_sz, [_i, _i]),
    "hlgs_rasterize_forward_prepare": (_i, [C.POINTER(RasterArgs), _vp, _vp, _vp, C.POINTER(FrameInfo), _vp]),
    "hlgs_rasterize_forward_render": (_i, [C.POINTER(RasterArgs), _vp, _vp, _vp, _vp, C.POINTER(FrameInfo), _vp,
                                           _vp, _vp, _vp]),
    "hlgs_rasterize_forward": (_i, [C.POINTER(RasterArgs), _vp, _vp, _vp, _vp, _sz, C.POINTER(FrameInfo), _vp, _vp,
                                    _vp, _vp]),
    "hlgs_rasterize_backward": (_i, [C.POINTER(RasterArgs), _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp,
                                     C.POINTER(Grads), _vp]),
    "hlgs_rasterize_backward_split": (_i, [C.POINTER(RasterArgs), _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp,
                                           C.POINTER(Grads), _vp, _vp]),
    "hlgs_sh_grad_from_colour": (_i, [_i, _i, _i, _i, _i, _vp, _vp, _vp, C.c_int64, _f, _vp, _vp, _vp]),
    "hlgs_mark_visible": (_i, [_i, _vp, _vp, _vp, _vp, _vp]),
    "hlgs_compute_relocation": (_i, [_i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    "hlgs_adam_update": (_i, [_vp, _vp, _vp, _vp, _vp, _f, _f, _f, _f, C.c_uint32, C.c_uint32, _vp]),
    "hlgs_morton_codes": (_i, [_i, _vp, _vp, _vp, _vp, _vp]),
    "hlgs_upper_cut_scratch_size": (_sz, [_i]),
    "hlgs_upper_tree_cut": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _f, _i, _i, _vp, _vp, C.POINTER(_i), _vp]),
    "hlgs_upper_tree_cut_device": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _vp, _f, _i, _i, _vp, _vp, _vp, _vp]),
    "hlgs_upper_tree_cut_views_device": (_i, [_i, _vp, _vp, _vp, _vp, _i, _vp, _vp, _f, _i, _i, _vp, _vp, _vp,
                                              _vp]),
    "hlgs_upper_tree_cut_views_ordered_device": (_i, [_i, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _f, _i, _i, _vp, _vp,
                                                      _vp, _vp]),
    "hlgs_upper_tree_order_size": (_sz, [_i]),
    "hlgs_upper_tree_order": (_i, [_i, _vp, _vp]),
    "hlgs_gather_rows": (_i, [C.c_int64, _i, _vp, _vp, _vp, _vp]),
    "hlgs_spt_cache_scratch_size": (_sz, [_i, _i, _i, _i]),
    "hlgs_spt_cache_plan": (_i, [C.POINTER(CacheArgs), C.POINTER(CachePlan), _vp, _vp]),
    "hlgs_copy_rows": (_i, [_i, C.POINTER(RowCopy), C.c_int64, _vp, _vp, _vp]),
    "hlgs_copy_rows_packed": (_i, [_i, C.POINTER(RowCopy), C.c_int64, _vp, _vp, _vp, C.c_int64, _i, _vp]),
    "hlgs_load_rows_packed": (_i, [_i, C.POINTER(RowCopy), C.c_int64, _vp, _vp, _vp, C.c_int64, _vp]),
    "hlgs_activate_forward": (_i, [C.c_int64] + [_vp] * 7),
    "hlgs_activate_backward": (_i, [C.c_int64] + [_vp] * 10),
    "hlgs_adam_step": (_i, [_i, C.POINTER(AdamTensor), C.c_int64, _i, C.c_double, C.c_double, C.c_double, _vp]),
    "hlgs_spt_build": (_i, [_i, _vp, _vp, _vp, _i, _f, _f, _i, _i, C.POINTER(_vp)]),
    "hlgs_spt_result_sizes": (_i, [_vp, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i)]),
    "hlgs_spt_result_copy": (_i, [_vp] * 11),
    "hlgs_spt_result_free": (None, [_vp]),
    "hlgs_scatter_rows": (_i, [C.c_int64, _i, _vp, _vp, _vp, _vp]),
    "hlgs_ssim_scratch_size": (_sz, [_i, _i, _i]),
    "hlgs_ssim_forward": (_i, [_i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp]),
    "hlgs_ssim_backward": (_i, [_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "hlgs_ssim_forward_ex": (_i, [_i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp]),
    "hlgs_ssim_backward_ex": (_i, [_i, _i, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp]),
    "hlgs_depth_l1_scratch_size": (_sz, [C.c_int64]),
    "hlgs_depth_l1_forward": (_i, [C.c_int64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "hlgs_depth_l1_backward": (_i, [C.c_int64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "hlgs_hier_info_read": (_i, [C.c_char_p, _i, C.POINTER(HierInfo)]),
    "hlgs_hier_load": (_i, [C.c_char_p] + [_vp] * 7),
    "hlgs_hier_write": (_i, [C.c_char_p, _i, _i] + [_vp] * 7 + [_i]),
    "hlgs_dhier_load": (_i, [C.c_char_p] + [_vp] * 6),
    "hlgs_dhier_write": (_i, [C.c_char_p, _i, _i] + [_vp] * 6 + [_i]),
    "hlgs_expand_to_target": (_i, [_i, _vp, _i, _vp, _i, C.POINTER(_i)]),
    "hlgs_lod_scratch_size": (_sz, [_i]),
    "hlgs_expand_to_size_dynamic": (_i, [_i, _f, _vp, _vp, _vp, _vp, C.POINTER(_f), _vp, _vp, _vp, _vp,
                                         C.POINTER(_i), _vp]),
    "hlgs_get_interpolation_weights_dynamic": (_i, [_i, _vp, _f, _vp, _vp, _vp, C.POINTER(_f), C.POINTER(_f), _vp,
                                                    _vp, _vp]),
    "hlgs_expand_to_size": (_i, [_i, _f, _vp, _vp, _vp, C.POINTER(_f), _vp, _vp, _vp, _vp, C.POINTER(_i), _vp]),
    "hlgs_get_interpolation_weights": (_i, [_i, _vp, _f, _vp, _vp, C.POINTER(_f), C.POINTER(_f), _vp, _vp, _vp]),
    "hlgs_spt_scratch_size": (_sz, [_i]),
    "hlgs_spt_work_size": (_sz, [_i]),
    "hlgs_spt_cut_prepare": (_i, [_i, _vp, _vp, _vp, _vp, _vp, C.POINTER(_i), _vp]),
    "hlgs_spt_cut_finish": (_i, [_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, C.POINTER(_i), _vp]),
    "hlgs_lod_interp_forward": (_i, [_i, _i, _i] + [_vp] * 14),
    "hlgs_lod_interp_scratch_size": (_sz, [_i, _i]),
    "hlgs_lod_interp_backward": (_i, [_i, _i, _i, _i] + [_vp] * 16),
    "hlgs_binning_point_list_offset": (_sz, [_i]),
    "hlgs_point_list_entry_shift": (_i, [_i]),
    "hlgs_point_list_drops_empty": (_i, [_i]),
    "hlgs_set_entry_packing": (None, [_i]),
    "hlgs_set_drop_empty": (None, [_i]),
    "hlgs_set_plan_polls": (None, [C.c_uint]),
    "hlgs_image_ranges_offset": (_sz, [_i, _i]),
    "hlgs_image_misc_offset": (_sz, [_i, _i]),
    "hlgs_geom_splat_offset": (_sz, [_i]),
    "hlgs_set_stage_timing": (None, [_i]),
    "hlgs_stage_count": (_i, []),
    "hlgs_stage_name": (C.c_char_p, [_i]),
    "hlgs_stage_stats": (_i, [C.POINTER(_f), C.POINTER(_i), _i]),
}

_lib = None


def load():
    """Load libhlgs.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libhlgs.so not found at {LIB_PATH}; run `python __graft_entry__.py build` "
                               "(hipcc --offload-arch=gfx950) first -- there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            # every header function is exported by libhlgs.so (tests/test_abi_cpu.py, __graft_entry__.build()); a
            # host-only build (tests/sanitize/build.py) exports the host functions, and the others raise when called
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        msg = load().hlgs_last_error().decode(errors="replace")
        raise RuntimeError(f"libhlgs error {rc}: {msg}")


_GPU = []  # torch.cuda.is_available(), asked once per process (it costs a few us per call on every launch path)


def require_gpu(*tensors):
    if not _GPU:
        _GPU.append(torch.cuda.is_available())
    if not _GPU[0]:
        raise RuntimeError("libhlgs needs a HIP device (MI355X); torch.cuda.is_available() is False")
    for t in tensors:
        if t is not None and t.numel() and not t.is_cuda:
            raise RuntimeError("libhlgs expects device tensors")


def ptr(t):
    """Device pointer of a tensor, or NULL for None / empty tensors (the reference's data_ptr() of an
    empty tensor is nullptr as well)."""
    if t is None or t.numel() == 0:
        return None
    return _vp(t.data_ptr())


def stream():
    return _vp(torch.cuda.current_stream().cuda_stream)


def f3(values):
    arr = (_f * 3)(*[float(v) for v in values])
    return arr


def header_functions():
    """Names of the functions declared in include/hlgs.h (used by the ABI test)."""
    import re
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hlgs_[a-z0-9_]+)\s*\(", txt)))


def stage_stats():
    """{stage name: (mean ms per launch, launches)} since the last set_stage_timing()."""
    lib = load()
    n = lib.hlgs_stage_count()
    ms, calls = (_f * n)(), (_i * n)()
    lib.hlgs_stage_stats(ms, calls, n)
    return {lib.hlgs_stage_name(i).decode(): (float(ms[i]), int(calls[i])) for i in range(n)}


def set_stage_timing(enable, stages=None):
    """Time every stage (enable=True), only the named stages, or none (enable=False)."""
    lib = load()
    if not enable:
        mask = 0
    elif stages is None:
        mask = -1
    else:
        names = [lib.hlgs_stage_name(i).decode() for i in range(lib.hlgs_stage_count())]
        mask = sum(1 << names.index(n) for n in stages)
    lib.hlgs_set_stage_timing(mask)

"""CPU-side checks of the boundary: libhlgs.so loads, exports every function include/hlgs.h declares,
its host-only sizing queries are sane, and the Python API mirrors the reference's surface and errors.
No compute call is made here (there is no GPU in this container)."""
import ctypes as C
import inspect

import pytest
import torch

from hlgs_core import _lib as L


def test_library_exports_every_header_symbol():
    lib = L.load()
    names = L.header_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.hlgs_version().startswith(b"hlgs")


def test_buffer_sizes_are_monotone_and_aligned():
    lib = L.load()
    for P in (0, 1, 1000, 1_000_000):
        s = lib.hlgs_geom_buffer_size(P)
        assert s >= P * (4 + 4 + 8 + 24 + 16 + 12 + 4 + 4 + 8)
    assert lib.hlgs_image_buffer_size(1920, 1080) >= 1920 * 1080 * 8 + 8160 * 16
    assert lib.hlgs_binning_buffer_size(2_500_000) >= 2_500_000 * 20
    assert lib.hlgs_backward_scratch_size(1000, 5000) >= 5000 * 40
    assert lib.hlgs_lod_scratch_size(10) > 0 and lib.hlgs_spt_work_size(10) > 0


def _c_layout(struct, fields):
    """sizeof and field offsets of a header struct, as gcc lays it out from include/hlgs.h itself."""
    import os
    import subprocess
    import tempfile
    body = "".join(f'printf("%zu\\n", offsetof({struct}, {f}));' for f in fields)
    src = ('#include <stdio.h>\n#include <stddef.h>\n#include "hlgs.h"\n'
           f'int main(void) {{ printf("%zu\\n", sizeof({struct})); {body} return 0; }}\n')
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "t.c"), os.path.join(d, "t")
        open(c, "w").write(src)
        subprocess.check_call(["gcc", "-I", os.path.dirname(L.HEADER), c, "-o", exe])
        vals = [int(v) for v in subprocess.check_output([exe]).split()]
    return vals[0], vals[1:]


@pytest.mark.parametrize("cls,struct", [(L.RasterArgs, "hlgs_raster_args"), (L.Grads, "hlgs_grads"),
                                        (L.FrameInfo, "hlgs_frame_info"), (L.HierInfo, "hlgs_hier_info"),
                                        (L.CacheArgs, "hlgs_cache_args"), (L.CachePlan, "hlgs_cache_plan"),
                                        (L.RowCopy, "hlgs_row_copy"), (L.AdamTensor, "hlgs_adam_tensor")])
def test_ctypes_structs_match_header_layout(cls, struct):
    names = [f[0] for f in cls._fields_]
    size, offs = _c_layout(struct, names)
    assert C.sizeof(cls) == size
    assert [getattr(cls, n).offset for n in names] == offs


def test_stage_names():
    lib = L.load()
    names = [lib.hlgs_stage_name(i).decode() for i in range(lib.hlgs_stage_count())]
    assert names == ["preprocess", "scan", "tile_ranges", "scatter", "tile_sort", "blend_fwd", "blend_bwd",
                     "gauss_bwd", "count_tiles"]


def test_settings_fields_match_reference_order():
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    assert GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug", "render_indices", "parent_indices", "interpolation_weights",
        "num_node_kids", "do_depth")


def test_public_signatures_match_reference():
    import diff_gaussian_rasterization as D
    import gaussian_hierarchy as G
    # positional parameters (keyword-only extensions such as _C.rasterize_gaussians(..., need_seen=) are ours)
    sig = lambda f: [k for k, v in inspect.signature(f).parameters.items()  # noqa: E731
                     if v.kind != inspect.Parameter.KEYWORD_ONLY]
    assert sig(D.GaussianRasterizer.forward) == ["self", "means3D", "means2D", "opacities", "shs", "colors_precomp",
                                                  "scales", "rotations", "cov3D_precomp"]
    assert sig(D.rasterize_gaussians) == ["means3D", "means2D", "sh", "colors_precomp", "opacities", "scales",
                                          "rotations", "cov3Ds_precomp", "raster_settings"]
    assert sig(D.compute_relocation) == ["opacity_old", "scale_old", "N", "binoms", "n_max"]
    assert len(sig(D._C.rasterize_gaussians)) == 24 and len(sig(D._C.rasterize_gaussians_backward)) == 27
    assert sig(G.expand_to_size_dynamic)[:9] == ["nodes", "positions", "scales", "size", "viewpoint", "viewdir",
                                                 "render_indices", "parent_indices", "nodes_for_render_indices"]
    assert sig(G.get_interpolation_weights_dynamic) == ["indices", "size", "nodes", "positions", "scales",
                                                        "viewpoint", "viewdir", "ts", "num_kids"]
    assert sig(G.get_spt_cut_cuda)[:7] == ["number_of_SPTs", "gaussian_indices", "SPT_starts", "SPT_max", "SPT_min",
                                           "SPT_indices", "SPT_distances"]


def test_argument_errors_match_reference():
    from diff_gaussian_rasterization import GaussianRasterizer
    r = GaussianRasterizer(None)
    x = torch.zeros(4, 3)
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(x, x, torch.zeros(4, 1), shs=torch.zeros(4, 1, 3), colors_precomp=torch.zeros(4, 3), scales=x, rotations=x)
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(x, x, torch.zeros(4, 1), shs=torch.zeros(4, 1, 3), scales=x)
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(x, x, torch.zeros(4, 1), shs=torch.zeros(4, 1, 3), scales=x, rotations=x, cov3D_precomp=x)


def test_no_cpu_fallback():
    """Without a HIP device every compute entry point raises instead of silently running elsewhere."""
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from diff_gaussian_rasterization import _C
    e = torch.empty(0)
    with pytest.raises(RuntimeError, match="HIP device"):
        _C.rasterize_gaussians(torch.zeros(3), e, e, e, e, torch.zeros(4, 3), e, torch.zeros(4, 1), torch.ones(4, 3),
                               torch.ones(4, 4), 1.0, e, torch.eye(4), torch.eye(4), 0.5, 0.5, 16, 16,
                               torch.zeros(4, 1, 3), 0, torch.zeros(3), False, False, True)
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        _C.rasterize_gaussians(torch.zeros(3), e, e, e, e, torch.zeros(4, 2), e, e, e, e, 1.0, e, torch.eye(4),
                               torch.eye(4), 0.5, 0.5, 16, 16, e, 0, torch.zeros(3), False, False, True)


def test_product_sources_have_no_variant_switches():
    """libhlgs.so is exactly the tested configuration: no `#if HLGS_...` switch (diagnostic or measured loser) in the
    product sources -- variants are patches under tools/variants/ (or files in git history), built by
    tools/build_variant.py only."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "hlgs_build", os.path.join(root, "hierarchical-lod-gaussians_amd", "hlgs_core", "build.py"))
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)
    assert B.variant_switches() == []


def test_variants_are_patches_that_apply():
    """tools/variants/ holds no full-file kernel copies: only patches against the product sources,
    and each of them still applies to the current tree (so an A/B build cannot silently measure stale code)."""
    import glob
    import importlib.util
    import os
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    vdir = os.path.join(root, "tools", "variants")
    assert not glob.glob(os.path.join(vdir, "*.hip")) and not glob.glob(os.path.join(vdir, "*.cpp"))
    spec = importlib.util.spec_from_file_location("build_variant", os.path.join(root, "tools", "build_variant.py"))
    V = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(V)
    for patch in sorted(glob.glob(os.path.join(vdir, "*.patch"))):
        V.touched_files(patch)  # product sources only
        with tempfile.TemporaryDirectory() as tree:
            import shutil
            shutil.copytree(os.path.join(root, V.CSRC_REL), os.path.join(tree, V.CSRC_REL))
            shutil.copytree(os.path.join(root, "include"), os.path.join(tree, "include"))
            V.apply_patch(patch, tree, check_only=True)

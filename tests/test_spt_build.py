"""SPT construction in the library's host code (csrc/spt_build.cpp) against the CPU torch restatement of
GaussianModel.build_hierarchical_SPT (oracle/spt_ref.py), on synthetic dynamic hierarchies with a skybox prefix
(the layout create_from_hier produces).  Integer outputs bit-exact; distances within float32 rounding (the
restatement uses torch's exp/sqrt, the library libm's)."""
import numpy as np
import pytest
import torch

from hlgs_core import synthetic as S
from oracle import spt_ref as SR


@pytest.mark.parametrize("n,sky,volume,min_size", [(3000, 5, 5.0, 20), (6000, 0, 2.0, 50), (2000, 3, 20.0, 10)])
def test_spt_build_matches_restatement(n, sky, volume, min_size):
    from hlgs_core import spt
    cam = S.make_camera(256, 192)
    h = S.make_dynamic_hierarchy(S.make_gaussians(n, 0, cam, seed=n), skybox_points=sky, seed=n)
    nodes = torch.tensor(h["nodes"])
    nodes[:, 3] = torch.where(nodes[:, 2] == 2, nodes[:, 3], torch.zeros_like(nodes[:, 3]))  # create_from_hier :1065
    xyz = torch.tensor(h["means3D"])
    scaling = torch.log(torch.tensor(h["scales"]))
    got = spt.build_hierarchical_spt(nodes, xyz, scaling, sky, volume, 0.02, min_size)
    want = SR.build_spt(nodes, xyz, scaling, sky, volume, 0.02, min_size)
    assert len(want["SPT_root_hierarchy_indices"]) > 3, "the case should build several SPTs"
    for k in ("SPT_starts", "SPT_gaussian_indices", "SPT_root_hierarchy_indices", "upper_tree_nodes"):
        np.testing.assert_array_equal(got[k].numpy(), want[k].numpy(), err_msg=k)
    for k in ("upper_tree_xyz", "upper_tree_scaling"):
        np.testing.assert_array_equal(got[k].numpy(), want[k].numpy(), err_msg=k)
    for k in ("SPT_max", "SPT_min", "min_distance_squared", "bounding_sphere_radii"):
        np.testing.assert_allclose(got[k].numpy(), want[k].numpy(), rtol=2e-6, atol=0, err_msg=k)

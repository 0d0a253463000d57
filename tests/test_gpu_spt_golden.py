"""The HIP SPT streaming kernels against fixtures produced by the reference's OWN Python (tests/golden/make_golden.py
spt_fixture): train_post.py's coarse cut (:330-343, GaussianModel.cut_hierarchy_on_condition with
frustum_cull_spheres, scene/gaussian_model.py:55-103, 364-404) run from scene/gaussian_model.py, and
OurAdam._single_tensor_adam2 (scene/OurAdam.py:357-457) run from its file.  The cut is bit-exact; Adam is the same
float32 operation order (the scalars formed in double, as torch does)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_spt.npz"))
CASES = sorted({int(k.split("_")[-1]) for k in G.files if k.startswith("params_")})
CAMS = sorted({int(k.split("_")[-1]) for k in G.files if k.startswith("campos_")})


@pytest.mark.parametrize("i", CASES)
@pytest.mark.parametrize("c", CAMS)
def test_upper_tree_cut_matches_reference_run(i, c):
    from hlgs_core import spt
    d = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda")  # noqa: E731
    for k, dm in enumerate((1.0, 2.25)):
        cut = spt.upper_tree_cut(d(G[f"upper_tree_nodes_{i}"]), d(G[f"upper_tree_xyz_{i}"]), d(G[f"bounds_{i}"]),
                                 d(G[f"min_distance_squared_{i}"]), d(G[f"planes_{i}_{c}"]), d(G[f"campos_{c}"]), dm)
        np.testing.assert_array_equal(cut.cpu().numpy(), G[f"coarse_cut_{i}_{c}_{k}"], err_msg=f"multiplier {dm}")


def test_dense_adam_matches_reference_run():
    from hlgs_core.spt_cache import adam_step
    js = sorted({int(k.split("_")[-1]) for k in G.files if k.startswith("adam_in_")})
    for j in js:
        p, g, m, v = (torch.tensor(a.copy(), device="cuda").contiguous() for a in G[f"adam_in_{j}"])
        lr, it = G[f"adam_lr_it_{j}"]
        adam_step([p], [g], [m], [v], [float(lr)], int(it) + 1, 0)
        want = G[f"adam_out_{j}"]
        for got, w, name in zip((p, m, v), want, ("param", "exp_avg", "exp_avg_sq")):
            np.testing.assert_allclose(got.cpu().numpy(), w, rtol=2e-6, atol=1e-12, err_msg=f"{name} case {j}")

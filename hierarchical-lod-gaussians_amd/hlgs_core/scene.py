"""Scene assembly around a loaded dynamic hierarchy: the tensor bookkeeping of GaussianModel.create_from_hier
(scene/gaussian_model.py:990-1095) and sort_morton (:570-589), without the training state around them.

assemble_hierarchy() takes what gaussian_hierarchy.load_dynamic_hierarchy returns plus an optional scaffold
(skybox) point set and produces the model tensors the renderers read: skybox rows prepended, node indices
shifted past them, their node rows set to -99 (never selected by expand_to_size_dynamic,
runtime_switching.cu:557-560), first_child zeroed unless child_count == 2, and the last node column zeroed.
"""
import torch

# HierarchyNode columns (submodules/gaussianhierarchy/types.h:60-67)
NODE_DEPTH, NODE_PARENT, NODE_CHILD_COUNT, NODE_FIRST_CHILD, NODE_NEXT_SIBLING, NODE_MAX_SIDE = range(6)


def assemble_hierarchy(xyz, shs_all, alpha, scales, rots, nodes, sky=None, max_sh_degree=3):
    """xyz (P,3), shs_all (P,16,3), alpha (P,1) activated, scales / rots as stored, nodes (P,6) int32.
    sky: None, or dict(xyz, features_dc (S,1,3), features_rest (S,3,3), opacity_logits (S,1), scales, rotations)
    -- the scaffold's first S points (gaussian_model.py:1030-1049), whose opacity is sigmoid-activated here.
    Returns a dict of CPU tensors: xyz, features_dc, features_rest, opacity, scaling, rotation, nodes,
    skybox_points."""
    nodes = nodes.clone().to(torch.int32)
    S = 0
    if sky is not None:  # gaussian_model.py:1050-1066 (the `if scaffold_file:` branch)
        S = int(sky["xyz"].shape[0])
        if S > 0:
            xyz = torch.cat((sky["xyz"], xyz))
            alpha = torch.cat((torch.sigmoid(sky["opacity_logits"]), alpha))
            scales = torch.cat((sky["scales"], scales))
            rots = torch.cat((sky["rotations"], rots))
            filler = torch.zeros(S, 16, 3)
            filler[:, :1, :] = sky["features_dc"]
            filler[:, 1:4, :] = sky["features_rest"]
            shs_all = torch.cat((filler, shs_all))
        nodes[:, NODE_FIRST_CHILD] += S
        nodes[:, NODE_PARENT] += S
        nodes[nodes[:, NODE_NEXT_SIBLING] > 0, NODE_NEXT_SIBLING] += S
        nodes[0, NODE_PARENT] = -1
        nodes = torch.cat((torch.full((S, 6), -99, dtype=torch.int32), nodes))
        nodes[S:, 3] = torch.where(nodes[S:, 2] == 2, nodes[S:, 3], torch.zeros_like(nodes[S:, 3]))
    n_rest = {3: 15, 2: 8, 1: 3}.get(int(max_sh_degree), 0)
    nodes[:, -1] = 0  # gaussian_model.py:1092-1093
    return dict(xyz=xyz, features_dc=shs_all[:, :1, :], features_rest=shs_all[:, 1:1 + n_rest, :], opacity=alpha,
                scaling=scales, rotation=rots, nodes=nodes, skybox_points=S)


def morton_order(xyz, skybox_points=0):
    """sort_morton's permutation (gaussian_model.py:570-589): Morton codes of the non-skybox points on the
    device (gaussian_hierarchy.get_morton_indices), argsort, the root kept at position 0, shifted past the
    skybox.  Returns the int32 index tensor `indices` with model[indices] = model[skybox_points:]."""
    import gaussian_hierarchy as GH
    pts = xyz[skybox_points:]
    codes = torch.zeros_like(pts[:, 0], dtype=torch.int64)
    GH.get_morton_indices(pts, torch.min(pts, dim=0)[0], torch.max(pts, dim=0)[0], codes)
    indices = torch.argsort(codes).to(torch.int32)
    root_index = torch.where(indices == 0)[0][0]
    indices[root_index] = indices[0]
    indices[0] = 0
    return indices + skybox_points

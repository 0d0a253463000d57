"""A plain alt-rasterizer render of SPT-cache parameter rows (config #5's activations: sigmoid opacity, exp scale,
normalised rotation, SH degree 1, antialiasing), for tests that compare resident sets."""
import torch


def render_alt(p, cam, dev):
    from alt_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    s = GaussianRasterizationSettings(image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanfovx"],
                                      tanfovy=cam["tanfovy"], bg=torch.zeros(3, device=dev), scale_modifier=1.0,
                                      viewmatrix=cam["viewmatrix"].to(dev), projmatrix=cam["projmatrix"].to(dev),
                                      sh_degree=1, campos=cam["campos"].to(dev), prefiltered=False, debug=False,
                                      antialiasing=True)
    with torch.no_grad():
        img, _, _ = GaussianRasterizer(s)(
            means3D=p["xyz"], means2D=torch.zeros_like(p["xyz"]), dc=p["f_dc"], shs=p["f_rest"],
            opacities=torch.sigmoid(p["opacity"]), scales=torch.exp(p["scaling"]),
            rotations=torch.nn.functional.normalize(p["rotation"]))
    return img

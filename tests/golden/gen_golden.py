"""Generate the committed golden fixtures tests/golden/*.npz (container-only tool).

    python tests/golden/gen_golden.py

Each fixture holds the rasterizer's inputs (synthetic scene + camera) and
the outputs of the independent dense torch restatement (dense_reference.py): rendered
image, final transmittance, last contributor, radii (float32 geometry) and float64
autograd gradients of every input.  Loaded with ``numpy.load(allow_pickle=False)``.
The reference repository has no rasterizer and no fixtures for one, so
these vectors pin the hand-written backward of the CPU oracle and of the HIP kernels.
"""
from __future__ import annotations

import hashlib
import importlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
import dense_reference as dref  # noqa: E402

graphics = importlib.import_module("3d_gaussian_splatting_amd.graphics")
scene = importlib.import_module("3d_gaussian_splatting_amd.scene")

CASES = [
    # name, P, W, H, active D, max deg, bg, scale_mod, precomp, seed
    ("sh3_64x48", 256, 64, 48, 3, 3, (0.0, 0.0, 0.0), 1.0, False, 0),
    ("sh1_white_72x56", 300, 72, 56, 1, 3, (1.0, 1.0, 1.0), 1.0, False, 3),
    ("sh2_mod_64x64", 200, 64, 64, 2, 2, (0.25, 0.5, 0.75), 0.8, False, 5),
    ("sh0_40x40", 120, 40, 40, 0, 0, (0.0, 0.0, 0.0), 1.0, False, 7),
    ("precomp_48x40", 200, 48, 40, 0, 0, (0.1, 0.2, 0.3), 1.0, True, 9),
]


def run_case(name, P, W, H, D, maxdeg, bg, smod, precomp, seed):
    cam = graphics.synthetic_camera(W, H)
    s = scene.make_scene(cam, P, max_sh_degree=maxdeg, seed=seed)
    dpix = scene.make_dL_dpix(cam, seed=seed + 1)
    dt = torch.float64
    leaf = lambda a: torch.tensor(np.asarray(a), dtype=dt, requires_grad=True)
    means = leaf(s.means3D)
    opac = leaf(s.opacities)
    inputs = dict(means3D=s.means3D, opacities=s.opacities, dL_dpix=dpix,
                  bg=np.asarray(bg, np.float32))
    if precomp:
        rng = np.random.default_rng(seed)
        colors_np = rng.uniform(0.0, 1.0, (P, 3)).astype(np.float32)
        # cov3D from the scene's (scale, rotation) so it is a valid SPD matrix
        cov_np = np.stack([_cov6(s.scales[i], s.rotations[i]) for i in range(P)]).astype(np.float32)
        colors, cov = leaf(colors_np), leaf(cov_np)
        pre = dref.preprocess(cam, means, opac, colors=colors, cov3D=cov, dtype=dt)
        geom = dref.geometry_f32(cam, s.means3D, s.opacities, cov3D=cov_np)
        inputs.update(colors_precomp=colors_np, cov3D_precomp=cov_np)
        leaves = dict(means3D=means, opacities=opac, colors=colors, cov3D=cov)
    else:
        scales, rots = leaf(s.scales), leaf(s.rotations)
        dc, rest = leaf(s.sh_dc), leaf(s.sh_rest)
        pre = dref.preprocess(cam, means, opac, scales=scales, rots=rots, sh_dc=dc, sh_rest=rest, D=D,
                              scale_mod=smod, dtype=dt)
        geom = dref.geometry_f32(cam, s.means3D, s.opacities, scales=s.scales, rots=s.rotations,
                                 scale_mod=smod)
        inputs.update(scales=s.scales, rotations=s.rotations, sh_dc=s.sh_dc, sh_rest=s.sh_rest)
        leaves = dict(means3D=means, opacities=opac, scales=scales, rotations=rots, sh_dc=dc, sh_rest=rest)
    img, T, last = dref.render(cam, pre, geom, bg)
    loss = (img * torch.tensor(dpix, dtype=dt)).sum()
    loss.backward()
    out = dict(color=img.detach().numpy(), final_T=T.detach().numpy(), n_contrib=last.numpy().astype(np.uint32),
               radii=geom["radius"].numpy().astype(np.int32),
               grad_means2D=pre["hook"].grad.numpy())
    for k, v in leaves.items():
        out["grad_" + k] = v.grad.numpy() if v.grad is not None else np.zeros(v.shape)
    meta = dict(name=name, P=P, W=W, H=H, sh_degree=D, max_sh_degree=maxdeg, scale_modifier=smod,
                precomp=precomp, seed=seed, viewmatrix=cam.viewmatrix.tolist(),
                projmatrix=cam.projmatrix.tolist(), campos=cam.campos.tolist(),
                tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
                visible=int(geom["visible"].sum()))
    return inputs, out, meta


def _cov6(sv, q):
    r, x, y, z = [float(v) for v in q]
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)],
                  [2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)],
                  [2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)]])
    L = R * np.asarray(sv, np.float64)[None, :]
    S = L @ L.T
    return np.array([S[0, 0], S[0, 1], S[0, 2], S[1, 1], S[1, 2], S[2, 2]])


def main():
    manifest = {}
    for case in CASES:
        inputs, out, meta = run_case(*case)
        path = os.path.join(HERE, f"{meta['name']}.npz")
        arrays = {"in_" + k: v for k, v in inputs.items()}
        arrays.update({"out_" + k: v for k, v in out.items()})
        arrays["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        np.savez_compressed(path, **arrays)
        with open(path, "rb") as fh:
            manifest[os.path.basename(path)] = dict(sha256=hashlib.sha256(fh.read()).hexdigest(),
                                                   visible=meta["visible"], P=meta["P"])
        print(meta["name"], "visible", meta["visible"], "img mean", float(out["color"].mean()))
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

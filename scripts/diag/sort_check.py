"""Diagnostic: the per-tile sorted (tile, gid) lists of the HIP forward against the oracle's for a
few small scenes; prints the first tile that differs (its length and both lists' heads)."""
import os, sys, glob
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from conftest import pkg, load_fixture
import gsr_oracle
gsr_oracle.build()
rast = pkg("rasterizer").CAbiRasterizer("cuda")
native = pkg("native")

def check(name, cam, args, kw):
    st = rast.forward(cam, *args, **kw)
    f = gsr_oracle.forward(cam, *args, **kw)
    K = st.num_rendered
    t_ref, d_ref, g_ref = f.state.sorted()
    gid = st.view(native.VIEW_SORTED_GID, torch.int32, K).cpu().numpy().view(np.uint32)
    rng = f.state.ranges()
    bad = 0
    for t, (a, b) in enumerate(rng):
        if not np.array_equal(gid[a:b], g_ref[a:b]):
            if bad < 3:
                dk = f.state.preprocess()["depth"].view(np.uint32)
                i = int(np.nonzero(gid[a:b] != g_ref[a:b])[0][0])
                print(name, "tile", t, "n", b - a, "first diff at", i, "gpu", gid[a + i:a + i + 4], "ref", g_ref[a + i:a + i + 4],
                      "dk gpu", dk[gid[a + i:a + i + 4]], "dk ref", dk[g_ref[a + i:a + i + 4]])
            bad += 1
    print(name, "K", K, "tiles", len(rng), "bad tiles", bad, flush=True)

for path in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.npz")))[:3]:
    meta, cam, inp, out = load_fixture(path)
    g = inp.get
    check(os.path.basename(path), cam, (g("means3D"), g("opacities"), g("scales"), g("rotations"), g("sh_dc"), g("sh_rest")),
          dict(sh_degree=meta["sh_degree"], colors_precomp=g("colors_precomp"), cov3D_precomp=g("cov3D_precomp"),
               scale_modifier=meta["scale_modifier"], bg=g("bg")))
gr, sc = pkg("graphics"), pkg("scene")
for P, W, H in [(1000, 256, 256), (5000, 300, 200)]:
    cam = gr.synthetic_camera(W, H)
    s = sc.make_scene(cam, P, max_sh_degree=1, seed=1)
    check(f"{P}_{W}x{H}", cam, (s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest), dict(sh_degree=1))

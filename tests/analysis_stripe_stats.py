#!/usr/bin/env python3
"""CPU emulation of the blend kernels' stripe culling at 1M/1080p (analysis tool; uses the
oracle): visited records, stripe evaluations and mask popcounts per (tile, record).  The
live-stripe test approximates the kernels' termination check by the oracle's n_contrib."""
import numpy as np, sys, importlib, time
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle import gsr_oracle as O
scene = importlib.import_module("3d_gaussian_splatting_amd.scene"); gr = importlib.import_module("3d_gaussian_splatting_amd.graphics")
cam = gr.synthetic_camera(1920,1080)
s = scene.make_scene(cam, 1_000_000, 3, seed=0)
f = O.forward(cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, sh_degree=3)
st = f.state
pre = st.preprocess()
tkey, dep, gid = st.sorted()
ranges = st.ranges()
T, ncon = st.pixel_state()
W, H = 1920, 1080
ncon = ncon.reshape(H, W)
xy = pre["xy"]; co = pre["conic_o"]
A, B, C, o = co[:,0], co[:,1], co[:,2], co[:,3]
det = A*C - B*B
det = np.where(det == 0, 1, det)
ca, cc = C/det, A/det   # cov2D a, c
with np.errstate(invalid='ignore', divide='ignore'):
    tthr = 2*np.log(255*o)
    ex = np.where(tthr > 0, np.sqrt(np.maximum(tthr*ca,0))*1.02+0.5, -1)
    ey = np.where(tthr > 0, np.sqrt(np.maximum(tthr*cc,0))*1.02+0.5, -1)
gx = (W+15)//16
ranges = ranges.reshape(-1, 2)
R = S = Rall = 0; pc = np.zeros(5, np.int64); pairs3 = 0
for t in range(ranges.shape[0]):
    a, b = ranges[t]
    if b <= a: continue
    tx, ty = t % gx, t // gx
    bx0, by0 = tx*16, ty*16
    g = gid[a:b]
    x, y = xy[g,0], xy[g,1]
    exg, eyg = ex[g], ey[g]
    okx = (exg >= 0) & (x + exg >= bx0) & (x - exg <= bx0 + 15)
    m = np.zeros(len(g), np.int64)
    for p in range(4):
        s0 = by0 + 4*p
        m |= (okx & (y + eyg >= s0) & (y - eyg <= s0 + 3)).astype(np.int64) << p
    # live per stripe: pixel alive at record e if e < its termination (approx n_contrib)
    tile_n = ncon[by0:by0+16, bx0:bx0+16]
    e = np.arange(len(g))
    live = np.zeros(len(g), np.int64)
    for p in range(4):
        rows = tile_n[4*p:4*p+4]
        mx = rows.max() if rows.size else 0
        live |= (e < mx).astype(np.int64) << p
    mm = m & live
    vis = mm != 0
    R += vis.sum(); Rall += len(g)
    cnt = np.array([bin(v).count('1') for v in mm[vis]]) if vis.any() else np.zeros(0,int)
    S += cnt.sum()
    pc += np.bincount(cnt, minlength=5)[:5]
    pairs3 += (((mm & 3) == 3) | ((mm & 12) == 12)).sum()
print(f"instances {Rall}  visited records R={R} ({R/Rall:.2f})  stripe evals S={S}  S/R={S/R:.2f}")
print("popcount hist (records):", pc)
print("records with a full pair (0,1) or (2,3):", pairs3)

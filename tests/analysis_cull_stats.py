#!/usr/bin/env python3
"""CPU emulation (oracle outputs, 1M/1080p) of the blend kernels' culling options: stripe (16x4)
vs quadrant (8x8) units, footprint box vs exact ellipse test; counts unit evaluations and
visited records.  Analysis tool for DESIGN.md §5.1."""
import numpy as np, sys, importlib
_R = __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))); sys.path.insert(0, _R); sys.path.insert(0, _R + '/oracle')
import gsr_oracle as O
scene = importlib.import_module("3d_gaussian_splatting_amd.scene"); gr = importlib.import_module("3d_gaussian_splatting_amd.graphics")
cam = gr.synthetic_camera(1920,1080)
s = scene.make_scene(cam, 1_000_000, 3, seed=0)
f = O.forward(cam, s.means3D, s.opacities, s.scales, s.rotations, s.sh_dc, s.sh_rest, sh_degree=3)
st = f.state
pre = st.preprocess()
tkey, dep, gid = st.sorted()
ranges = st.ranges().reshape(-1,2)
T, ncon = st.pixel_state()
W, H = 1920, 1080
ncon = ncon.reshape(H, W)
xy = pre["xy"]; co = pre["conic_o"].astype(np.float64)
A, B, C, o = co[:,0], co[:,1], co[:,2], co[:,3]
det = A*C - B*B; det = np.where(det == 0, 1, det)
ca, cc = C/det, A/det
with np.errstate(invalid='ignore', divide='ignore'):
    tthr = 2*np.log(255*o)
ex = np.where(tthr > 0, np.sqrt(np.maximum(tthr*ca,0))*1.02+0.5, -1)
ey = np.where(tthr > 0, np.sqrt(np.maximum(tthr*cc,0))*1.02+0.5, -1)
gx = (W+15)//16

def rect_min_q(x, y, a, b, c, x0, x1, y0, y1):
    # min over rect [x0,x1]x[y0,y1] of q = a dx^2 + 2b dx dy + c dy^2, dx = X - x, dy = Y - y (vectorised over records)
    best = np.full(x.shape, np.inf)
    inside = (x >= x0) & (x <= x1) & (y >= y0) & (y <= y1)
    for X in (x0, x1):   # vertical edges: minimise over Y in [y0,y1]
        dx = X - x
        ystar = np.clip(y - b*dx/np.where(c==0,1e-30,c), y0, y1)
        dy = ystar - y
        best = np.minimum(best, a*dx*dx + 2*b*dx*dy + c*dy*dy)
    for Y in (y0, y1):
        dy = Y - y
        xstar = np.clip(x - b*dy/np.where(a==0,1e-30,a), x0, x1)
        dx = xstar - x
        best = np.minimum(best, a*dx*dx + 2*b*dx*dy + c*dy*dy)
    return np.where(inside, 0.0, best)

tot = dict(stripe_box=0, quad_box=0, stripe_ell=0, quad_ell=0, recs=0, recs_ell=0)
for t in range(ranges.shape[0]):
    a0, b0 = ranges[t]
    if b0 <= a0: continue
    tx, ty = t % gx, t // gx
    bx0, by0 = tx*16, ty*16
    g = gid[a0:b0]
    x, y = xy[g,0].astype(np.float64), xy[g,1].astype(np.float64)
    exg, eyg = ex[g], ey[g]
    tile_n = ncon[by0:by0+16, bx0:bx0+16]
    e = np.arange(len(g))
    # live approx: region alive while e < max n_contrib of the region
    def live(r0, r1, c0, c1):
        sub = tile_n[r0:r1, c0:c1]
        return e < (sub.max() if sub.size else 0)
    okx = (exg >= 0) & (x + exg >= bx0) & (x - exg <= bx0 + 15)
    thr = np.maximum(tthr[g], 0)  # q <= thr  <=> alpha >= 1/255 (q = d^T conic d)
    aa, bb, cc2 = A[g], B[g], C[g]
    any_s = np.zeros(len(g), bool); any_e = np.zeros(len(g), bool)
    for p in range(4):
        s0 = by0 + 4*p
        m = okx & (y + eyg >= s0) & (y - eyg <= s0 + 3) & live(4*p, 4*p+4, 0, 16)
        tot['stripe_box'] += m.sum()
        me = m & (rect_min_q(x, y, aa, bb, cc2, bx0, bx0+15, s0, s0+3) <= thr)
        tot['stripe_ell'] += me.sum()
        any_s |= m; any_e |= me
    for qy in range(2):
        for qx in range(2):
            X0, Y0 = bx0 + 8*qx, by0 + 8*qy
            m = (exg >= 0) & (x + exg >= X0) & (x - exg <= X0 + 7) & (y + eyg >= Y0) & (y - eyg <= Y0 + 7) & live(8*qy, 8*qy+8, 8*qx, 8*qx+8)
            tot['quad_box'] += m.sum()
            me = m & (rect_min_q(x, y, aa, bb, cc2, X0, X0+7, Y0, Y0+7) <= thr)
            tot['quad_ell'] += me.sum()
    tot['recs'] += any_s.sum(); tot['recs_ell'] += any_e.sum()
print(tot)
print("pairs fwd (oracle)", st.forward_pairs() if hasattr(st,'forward_pairs') else None)

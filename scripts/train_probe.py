import sys, time, os, importlib
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
bench = importlib.import_module("bench")
gr, sc = bench.gr, bench.sc
Tr = importlib.import_module("3d_gaussian_splatting_amd.trainer")
dev = torch.device("cuda", 0)
cam = gr.synthetic_camera(1920, 1080)
s = sc.make_scene(cam, 1_000_000, max_sh_degree=3, seed=0)
tr = Tr.GaussianTrainer(s.means3D, s.sh_dc, s.sh_rest, s.raw_opacities, s.raw_scales, s.raw_rotations, max_sh_degree=3, device=dev)
tr.active_sh_degree = 3
gt = torch.rand(3, 1080, 1920, device=dev)
for i in range(3): tr.step(i + 1, cam, gt, densify=False)
torch.cuda.synchronize()
def timed(label, fn, n=10):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for i in range(n): fn(i)
    torch.cuda.synchronize(); print(label, (time.perf_counter() - t0) / n * 1e3, "ms", flush=True)
timed("step nosync", lambda i: tr.step(10 + i, cam, gt, densify=False))
timed("step sync", lambda i: (tr.step(30 + i, cam, gt, densify=False), torch.cuda.synchronize()))
def parts(i):
    t = [time.perf_counter()]
    st = tr.render(cam); t.append(time.perf_counter())
    stats, maps = tr.k.loss_forward(st.color, gt, 0.2); d = tr.k.loss_backward(st.color, gt, 0.2, maps); t.append(time.perf_counter())
    g = tr.rast.backward(st, d); t.append(time.perf_counter())
    grads = {"xyz": g["means3D"], "f_dc": g["sh_dc"], "f_rest": g["sh_rest"], "opacity": g["opacities"], "scaling": g["scales"], "rotation": g["rotations"]}
    tr.optimizer_step(grads); t.append(time.perf_counter())
    torch.cuda.synchronize(); t.append(time.perf_counter())
    print("host ms", [round((b - a) * 1e3, 3) for a, b in zip(t, t[1:])], flush=True)
for i in range(4): parts(i)
print(torch.cuda.memory_stats()["num_alloc_retries"], torch.cuda.memory_allocated() / 1e9, torch.cuda.memory_reserved() / 1e9)

def detail(it):
    opt = tr.opt
    t = [time.perf_counter()]
    tr.update_learning_rate(it); t.append(time.perf_counter())
    st = tr.render(cam); torch.cuda.synchronize(); t.append(time.perf_counter())
    stats, maps = tr.k.loss_forward(st.color, gt, opt.lambda_dssim)
    dimg = tr.k.loss_backward(st.color, gt, opt.lambda_dssim, maps); torch.cuda.synchronize(); t.append(time.perf_counter())
    g = tr.rast.backward(st, dimg); torch.cuda.synchronize(); t.append(time.perf_counter())
    tr.k.densify_stats(st.radii, g["means2D"], tr.max_radii2D, tr.xyz_gradient_accum, tr.denom); torch.cuda.synchronize(); t.append(time.perf_counter())
    grads = {"xyz": g["means3D"], "f_dc": g["sh_dc"], "opacity": g["opacities"], "scaling": g["scales"], "rotation": g["rotations"], "f_rest": g["sh_rest"]}
    tr.optimizer_step(grads); torch.cuda.synchronize(); t.append(time.perf_counter())
    print("detail ms", [round((b - a) * 1e3, 3) for a, b in zip(t, t[1:])], flush=True)
for i in range(4): detail(100 + i)

"""The C-ABI shared library loads and exports every symbol include/gsr/gsr.h declares; size
queries and argument validation work without a GPU (no kernel launches here)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT, pkg

HEADER = os.path.join(ROOT, "include", "gsr", "gsr.h")
TRAIN_HEADER = os.path.join(ROOT, "include", "gsr", "gsr_train.h")
COMM_HEADER = os.path.join(ROOT, "include", "gsr", "gsr_comm.h")


def declared_functions(header=None):
    headers = [header] if header else [HEADER, TRAIN_HEADER, COMM_HEADER]
    out = set()
    for h in headers:
        text = open(h).read()
        out |= set(re.findall(r"^\s*(?:const\s+)?[\w\*\s]+?\b(gsr_\w+)\s*\(", text, re.M))
    return sorted(out - {"gsr_alloc_fn"})


def test_header_declares_expected_entry_points():
    native = pkg("native")
    assert set(native.EXPORTS) == set(declared_functions(HEADER)), declared_functions(HEADER)
    assert set(native.TRAIN_EXPORTS) == set(declared_functions(TRAIN_HEADER)), declared_functions(TRAIN_HEADER)
    assert set(native.COMM_EXPORTS) == set(declared_functions(COMM_HEADER)), declared_functions(COMM_HEADER)


def test_comm_abi_validation_without_gpu():
    """gsr_comm.h: the RCCL transport's entry points reject bad arguments before touching a
    device; the unique-id size matches the header."""
    native = pkg("native")
    L = native.load_hip()
    text = open(COMM_HEADER).read()
    assert int(re.search(r"#define GSR_COMM_ID_BYTES (\d+)", text).group(1)) == native.COMM_ID_BYTES
    comm = ctypes.c_void_p()
    id_ = (ctypes.c_uint8 * native.COMM_ID_BYTES)()
    L.gsr_comm_init.restype = ctypes.c_int
    assert L.gsr_comm_init(ctypes.byref(comm), id_, 2, 5) < 0 and "rank" in native.last_error()
    assert L.gsr_comm_init(None, id_, 1, 0) < 0
    assert L.gsr_comm_all_to_all(None, None, None, ctypes.c_size_t(0), None) < 0
    assert L.gsr_comm_destroy(None) == 0


def test_train_abi_validation_without_gpu():
    """gsr_train.h entry points load, size their scratch and reject bad arguments (no launch)."""
    native = pkg("native")
    L = native.load_hip()
    assert L.gsr_loss_scratch_bytes(3, 1080, 1920) >= 3 * 3 * 1080 * 1920 * 4
    assert L.gsr_compact_scratch_bytes(1 << 20) >= 1024 * 4
    assert L.gsr_loss_forward(None, None, 3, 8, 8, 0.2, None, None, None) < 0
    assert "loss" in native.last_error()
    g = (native.AdamGroup * 1)()
    g[0].n, g[0].step, g[0].act = 8, 0, native.ACT_NONE
    g[0].param = g[0].grad = g[0].exp_avg = g[0].exp_avg_sq = 256
    assert L.gsr_adam_step(g, 1, 0.9, 0.999, 1e-8, None) < 0 and "step" in native.last_error()
    g[0].step, g[0].act, g[0].n = 1, native.ACT_NORMALIZE4, 6
    assert L.gsr_adam_step(g, 1, 0.9, 0.999, 1e-8, None) < 0 and "rows of 4" in native.last_error()
    assert L.gsr_adam_step(g, 9, 0.9, 0.999, 1e-8, None) < 0
    c = (native.RowCopy * 1)()
    c[0].src, c[0].dst, c[0].width = 256, 256, 3
    assert L.gsr_gather_rows(c, 1, ctypes.c_void_p(512), 4, None) < 0 and "alias" in native.last_error()
    assert L.gsr_densify_stats(None, None, 4, None, None, None, None) < 0


def test_header_constants_match_the_python_mirror():
    """#define constants of gsr.h that the Python mirror restates (native.py)."""
    native = pkg("native")
    text = open(HEADER).read()
    val = lambda name: int(re.search(rf"#define {name} (\d+)", text).group(1))
    assert val("GSR_TERM_STRIDE") == native.TERM_STRIDE
    assert val("GSR_VIEW_TERM") == native.VIEW_TERM
    assert val("GSR_VIEW_CK_LIVE") == native.VIEW_CK_LIVE


def test_library_exports_every_symbol():
    native = pkg("native")
    so = native.hip_library_path()
    assert os.path.exists(so), "run __graft_entry__.build()"
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [f for f in declared_functions() if f not in syms]
    assert not missing, missing


def test_library_loads_and_reports_sizes():
    native = pkg("native")
    L = native.load_hip()
    assert L.gsr_abi_version() == native.ABI_VERSION == 4
    assert L.gsr_geom_bytes(1000) > 1000 * 64
    assert L.gsr_binning_bytes(10, 64, 64) >= 10 * 24
    assert L.gsr_image_bytes(1920, 1080) >= 1920 * 1080 * 8
    # the B1 checkpoint slots (binning buffer): capacity / 48 + tiles + 1, at most the 31 per tile
    # a fixed array would hold -- 1080p, 7.2M instances: 0.63 GB, not 1.0; 4K: 1.3 GB, not 4.1
    tiles = 120 * 68
    assert L.gsr_ck_pool_slots(7_200_000, 1920, 1080) == 7_200_000 // 48 + tiles + 1
    assert L.gsr_ck_pool_slots(2**31 - 1, 1920, 1080) == 31 * tiles
    assert L.gsr_binning_bytes(7_200_000, 1920, 1080) < 16 * 7_200_000 + 4100 * (7_200_000 // 48 + tiles + 1) + (64 << 20)
    assert L.gsr_image_bytes(1920, 1080) < 64 << 20  # no per-tile checkpoint array any more
    assert L.gsr_scratch_bytes(100) >= 100 * 37  # 36-B partial + 1 flag byte per instance
    assert L.gsr_scratch_bytes(1 << 20) == (32 << 20) + (4 << 20) + (1 << 20)
    assert L.gsr_exchange_block_bytes(100) == 64 * 101
    assert L.gsr_shard_state_bytes(1000, 8, 100) > L.gsr_geom_bytes(1000) + 8 * 1000 * 4


def _c_sizes():
    """sizeof / offsetof of the gsr.h structs as the C compiler lays them out."""
    import tempfile
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "gsr/gsr.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(gsr_camera), sizeof(gsr_gaussians), sizeof(gsr_raster_settings),
         sizeof(gsr_grads), sizeof(gsr_buffers), offsetof(gsr_buffers, capacity));
  printf("%zu %zu\n", offsetof(gsr_raster_settings, max_rendered), offsetof(gsr_buffers, n_local));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "s.c"), os.path.join(d, "s")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        return [int(v) for v in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]


def test_ctypes_structs_match_the_c_layout():
    """The ctypes mirror (native.py) and the stub INTEGRATION.md hands to FFI callers have the
    exact sizes and field offsets of include/gsr/gsr.h."""
    native = pkg("native")
    sz = _c_sizes()
    assert [ctypes.sizeof(t) for t in (native.Camera, native.Gaussians, native.Settings, native.Grads,
                                       native.Buffers)] == sz[:5]
    assert native.Buffers.capacity.offset == sz[5]
    assert native.Settings.max_rendered.offset == sz[6] and native.Buffers.n_local.offset == sz[7]
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    stub = re.search(r"```python\n(# ctypes binding stub.*?)```", text, re.S)
    assert stub, "INTEGRATION.md must carry the ctypes binding stub"
    ns = {}
    exec(stub.group(1), ns)
    for name, mine in (("Camera", native.Camera), ("Gaussians", native.Gaussians), ("Settings", native.Settings),
                       ("Grads", native.Grads), ("Buffers", native.Buffers)):
        assert ctypes.sizeof(ns[name]) == ctypes.sizeof(mine), name
        assert [f[0] for f in ns[name]._fields_] == [f[0] for f in mine._fields_], name


def test_validation_rejects_bad_arguments_without_gpu():
    native = pkg("native")
    L = native.load_hip()
    c = native.Camera()
    c.width, c.height = 0, 10
    g = native.Gaussians()
    s = native.Settings()
    b = native.Buffers()
    rc = L.gsr_forward(ctypes.byref(c), ctypes.byref(g), ctypes.byref(s), None, None,
                       native.ALLOC_FN(lambda *_: 0), native.ALLOC_FN(lambda *_: 0), native.ALLOC_FN(lambda *_: 0),
                       None, ctypes.byref(b), None)
    assert rc < 0
    assert "image size" in native.last_error()
    c.width = 10
    g.P, g.sh_degree = 5, 4
    rc = L.gsr_forward(ctypes.byref(c), ctypes.byref(g), ctypes.byref(s), ctypes.c_void_p(16), ctypes.c_void_p(16),
                       native.ALLOC_FN(lambda *_: 0), native.ALLOC_FN(lambda *_: 0), native.ALLOC_FN(lambda *_: 0),
                       None, ctypes.byref(b), None)
    assert rc < 0
    # multi-GPU entry points validate before touching the device
    c.width, c.height = 64, 48
    g.P, g.sh_degree = 0, 0
    rows = (ctypes.c_int32 * 3)(0, 2, 2)
    rc = L.gsr_shard_forward(ctypes.byref(c), ctypes.byref(g), ctypes.byref(s), 2, rows, 16, ctypes.c_void_p(256),
                             None, ctypes.c_void_p(256), None, None)
    assert rc < 0 and "band_rows" in native.last_error()
    rc = L.gsr_band_forward(ctypes.byref(c), ctypes.byref(s), 2, 16, ctypes.c_void_p(256), ctypes.c_void_p(256),
                            native.ALLOC_FN(lambda *_: 0), native.ALLOC_FN(lambda *_: 0), native.ALLOC_FN(lambda *_: 0),
                            None, ctypes.byref(b), None)
    assert rc < 0 and "max_rendered" in native.last_error()
    s.max_rendered = -1
    rc = L.gsr_forward(ctypes.byref(c), ctypes.byref(g), ctypes.byref(s), ctypes.c_void_p(16), None,
                       native.ALLOC_FN(lambda *_: 0), native.ALLOC_FN(lambda *_: 0), native.ALLOC_FN(lambda *_: 0),
                       None, ctypes.byref(b), None)
    assert rc < 0 and "max_rendered" in native.last_error()


def test_torch_extension_loads():
    native = pkg("native")
    ext = native.load_torch_ext()
    assert ext.abi_version() == 4
    cam = ext.RasterCamera(16, 16, 0.5, 0.5, [0.0] * 16, [0.0] * 16, [0.0] * 3)
    assert cam.width == 16


def test_product_does_not_reference_oracle():
    """The product package never imports / links the oracle (test infrastructure only)."""
    pkg_dir = os.path.join(ROOT, "3d_gaussian_splatting_amd")
    for dirpath, _, files in os.walk(pkg_dir):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                text = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(import|from)\s+gsr_oracle|#include[^\n]*oracle|libgsr_oracle|"
                                     r"sys\.path[^\n]*oracle", text, re.M), f


@pytest.mark.parametrize("name", ["gsr_dropin", "gsr_train_loop", "gsr_shard_step"])
def test_dropin_executable_has_one_hip_runtime(name):
    """The C++ executables (lib/gsr_dropin: render(); lib/gsr_train_loop: the training loop)
    must resolve libgsr_hip.so's libamdhip64.so.7 to the torch wheel's bundled runtime, not load
    /opt/rocm's as a second one (_build._exe_flags: libtorch_hip ahead of libgsr_hip in NEEDED
    order, and no direct libamdhip64 dependency of their own)."""
    import shutil
    import subprocess
    exe = os.path.join(ROOT, "3d_gaussian_splatting_amd", "lib", name)
    if not os.path.exists(exe) or not shutil.which("ldd"):
        pytest.skip("drop-in executable not built")
    out = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    hip = [l.split("=>")[1].split("(")[0].strip() for l in out.splitlines() if "libamdhip64" in l and "=>" in l]
    hsa = [l for l in out.splitlines() if "libhsa-runtime64" in l]
    assert len(hip) == 1 and len(hsa) == 1, out


def test_bench_metric_names():
    """bench.py reports BASELINE.json's metric string verbatim for the headline config, and a
    workload-named one for every other config (no mislabelled lines)."""
    import json
    import bench
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)["metric"]
    assert bench.config_metric("1m_1080p") == base
    names = {bench.config_metric(k) for k in bench.CONFIGS}
    assert len(names) == len(bench.CONFIGS)
    assert "5M Gaussians" in bench.config_metric("5m_1080p")


def test_backward_refuses_bad_layout_word():
    """ABI 4: gsr_buffers.layout carries the forward's binning choice; a
    backward handed a struct whose word is zeroed (rebuilt without the field) or disagrees with
    what a forward of these buffers chooses returns GSR_ERR_LAYOUT with the reason, before any
    allocation or launch -- it never reads the other binning's arrays.  gsr_view returns NULL."""
    native = pkg("native")
    L = native.load_hip()
    text = open(HEADER).read()
    hexval = lambda name: int(re.search(rf"#define {name} (0x[0-9A-Fa-f]+|\d+)u?", text).group(1), 0)
    TAG, RB = hexval("GSR_LAYOUT_TAG"), hexval("GSR_LAYOUT_ROW_BUCKETED")
    err = int(re.search(r"#define GSR_ERR_LAYOUT \((-\d+)\)", text).group(1))
    c = native.Camera()
    c.width, c.height = 64, 48
    g = native.Gaussians()
    g.P, g.sh_degree = 5, 0
    fake = ctypes.c_void_p(1 << 20)  # never dereferenced: the check comes first
    g.means3D = g.opacities = g.sh_dc = g.scales = g.rotations = fake
    s = native.Settings()
    s.tile_y1 = 2**31 - 1
    gr = native.Grads()
    gr.dL_dmeans2D = gr.dL_dopacity = gr.dL_dmeans3D = gr.dL_dsh_dc = gr.dL_dscales = gr.dL_drotations = fake
    calls = []
    alloc = native.ALLOC_FN(lambda _c, n: calls.append(n) or 0)

    def backward(layout, capacity):
        b = native.Buffers()
        b.geom = b.binning = b.image = fake
        b.n_local, b.capacity, b.num_rendered, b.layout = 5, capacity, capacity, layout
        return L.gsr_backward(ctypes.byref(c), ctypes.byref(g), ctypes.byref(s), ctypes.byref(b), fake, alloc, None,
                              ctypes.byref(gr), None), b

    rc, b = backward(0, 64)  # a struct rebuilt with the word zeroed
    assert rc == err and "not a forward's" in native.last_error(), native.last_error()
    rc, _ = backward(TAG, 64)  # tagged, but a 4 x 3-tile image of 5 Gaussians takes the row-bucketed binning
    assert rc == err and "disagrees" in native.last_error(), native.last_error()
    rc, _ = backward(TAG | RB, 0)  # an empty binning never takes it
    assert rc == err and "disagrees" in native.last_error(), native.last_error()
    assert calls == [], "nothing may be allocated before the layout check"
    b.layout = 0
    L.gsr_view.restype = ctypes.c_void_p
    assert L.gsr_view(ctypes.byref(c), 5, ctypes.byref(b), 1) is None
    assert "layout" in native.last_error()
    # gsr_backward_blend / gsr_band_backward share the check (blend_backward)
    grad2d = fake
    rc = L.gsr_backward_blend(ctypes.byref(c), ctypes.byref(g), ctypes.byref(s), ctypes.byref(b), fake, alloc, None,
                              grad2d, None)
    assert rc == err and calls == []

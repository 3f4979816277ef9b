"""In-tree build of the native libraries (gfx950 only).

  lib/libgsr_hip.so      hipcc --offload-arch=gfx950: the CDNA4 kernels + the C ABI
  lib/_gsr_torch*.so     libtorch render() + autograd Function (C++), links libgsr_hip.so

Per-file flags: gsr_preprocess.hip is compiled with -ffp-contract=off so its key-feeding
arithmetic is bit-identical to the CPU oracle; the blend and preprocess-backward files too
(B1 replays the forward's alpha / T bit for bit; B2 recomputes clamp bits like F1); the
training kernels keep hipcc's default FMA contraction (compared within tolerance).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
ROOT = os.path.dirname(PKG)
ARCH = "gfx950"

HIP_SOURCES = {
    "gsr_preprocess.hip": ["-ffp-contract=off"],
    "gsr_sort.hip": [],
    # F6 and B1 must evaluate alpha / T identically; no SLP packing (it splits DPP-fused adds)
    "gsr_blend.hip": ["-ffp-contract=off", "-fno-slp-vectorize"],
    # recomputes the forward's SH clamp bits: must round exactly like gsr_preprocess.hip
    "gsr_preprocess_bwd.hip": ["-ffp-contract=off"],
    # training-step kernels (loss, fused Adam, densification): tolerance-compared, default flags
    "gsr_train.hip": [],
    # point-cloud initialisation (exact k-NN): box and point distances must round alike
    "gsr_init.hip": ["-ffp-contract=off"],
    # multi-GPU splat pack / unpack / gradient sum (copies and integer work)
    "gsr_shard.hip": [],
    "gsr_api.cpp": [],
    # RCCL transport of the multi-GPU step (include/gsr/gsr_comm.h)
    "gsr_comm.cpp": [],
}
LINK_LIBS = ["-lrccl"]
COMMON = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fno-fast-math",
          "-Wall", "-Wno-unused-function", "-I" + os.path.join(ROOT, "include")]


def _hipcc() -> str:
    p = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found")
    return p


def _stamp(paths, extra=""):
    h = hashlib.sha256(extra.encode())
    for p in sorted(paths):
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _headers():
    out = [os.path.join(ROOT, "include", "gsr", h) for h in ("gsr.h", "gsr_train.h", "gsr_comm.h")]
    out += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return out


def build_hip(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(LIB, exist_ok=True)
    so = os.path.join(LIB, "libgsr_hip.so")
    srcs = [os.path.join(CSRC, f) for f in HIP_SOURCES]
    stamp = _stamp(srcs + _headers(), " ".join(COMMON))
    stamp_file = so + ".stamp"
    if not force and os.path.exists(so) and os.path.exists(stamp_file) and open(stamp_file).read() == stamp:
        return so
    hipcc = _hipcc()
    obj_dir = os.path.join(LIB, "obj_hip")
    os.makedirs(obj_dir, exist_ok=True)

    def compile_one(name):
        # per-object content stamp (its source, the shared headers, its flags): an edit of one
        # kernel file recompiles that file only
        src = os.path.join(CSRC, name)
        obj = os.path.join(obj_dir, name + ".o")
        lang = ["-x", "hip"] if name.endswith(".cpp") else []
        cmd = [hipcc] + COMMON + HIP_SOURCES[name] + lang + ["-c", src, "-o", obj]
        ostamp = _stamp([src] + _headers(), " ".join(cmd))
        if not force and os.path.exists(obj) and os.path.exists(obj + ".stamp") and open(obj + ".stamp").read() == ostamp:
            return obj
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {name}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr)
        with open(obj + ".stamp", "w") as fh:
            fh.write(ostamp)
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, len(HIP_SOURCES))) as ex:
        objs = list(ex.map(compile_one, HIP_SOURCES))
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so] + objs + LINK_LIBS
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    with open(stamp_file, "w") as fh:
        fh.write(stamp)
    return so


def torch_ext_name() -> str:
    return "_gsr_torch" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so")


def build_torch_ext(verbose: bool = False, force: bool = False) -> str:
    """Compile csrc/torch/gsr_torch.cpp against libtorch (host C++, no device code) and link
    it to libgsr_hip.so with an $ORIGIN rpath, into lib/."""
    import torch
    from torch.utils import cpp_extension

    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, torch_ext_name())
    srcs = [os.path.join(CSRC, "torch", f) for f in ("gsr_torch.cpp", "gsr_shard.cpp")]
    tinc = cpp_extension.include_paths()
    flags = ["-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__=1",
             "-DTORCH_EXTENSION_NAME=_gsr_torch", "-DTORCH_API_INCLUDE_EXTENSION_H",
             f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
             "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include",
             "-I" + sysconfig.get_paths()["include"]] + ["-I" + p for p in tinc]
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    libs = ["-L" + LIB, "-lgsr_hip", "-Wl,-rpath,$ORIGIN", "-L" + tlib, "-lc10", "-ltorch",
            "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-Wl,-rpath," + tlib]
    stamp = _stamp(srcs + _headers() + EXE_HEADERS, " ".join(flags))
    stamp_file = out + ".stamp"
    if not force and os.path.exists(out) and os.path.exists(stamp_file) and open(stamp_file).read() == stamp:
        return out
    cxx = shutil.which("g++") or "c++"
    cmd = [cxx] + flags + ["-I" + os.path.join(CSRC, "torch")] + srcs + ["-o", out] + libs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch extension build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp_file, "w") as fh:
        fh.write(stamp)
    return out


def build_variant(name: str, defines: list, verbose: bool = False, csrc: str | None = None) -> str:
    """An experimental build of libgsr_hip.so with extra -D flags into lib/variants/<name>/ (for
    A/B timing with `bench.py --lib`; the product library is build_hip's).  `csrc`: build from
    another copy of the kernel sources (e.g. an earlier commit's, for a before / after A/B)."""
    src_dir = csrc or CSRC
    out_dir = os.path.join(LIB, "variants", name)
    os.makedirs(out_dir, exist_ok=True)
    so = os.path.join(out_dir, "libgsr_hip.so")
    hipcc = _hipcc()

    def one(src_name):
        flags = HIP_SOURCES[src_name]
        obj = os.path.join(out_dir, src_name + ".o")
        lang = ["-x", "hip"] if src_name.endswith(".cpp") else []
        cmd = [hipcc] + COMMON + flags + ["-D" + d for d in defines] + lang + ["-I" + src_dir, "-c",
                                                                              os.path.join(src_dir, src_name), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src_name}:\n{r.stderr}")
        return obj

    names = [n for n in HIP_SOURCES if os.path.exists(os.path.join(src_dir, n))]  # an older commit's sources
    with cf.ThreadPoolExecutor(max_workers=min(8, len(names))) as ex:
        objs = list(ex.map(one, names))
    r = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so] + objs + LINK_LIBS,
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    for o in objs:
        os.remove(o)
    return so


def _exe_flags():
    import torch
    from torch.utils import cpp_extension

    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    flags = ["-O2", "-std=c++17", "-DGSR_NO_PYBIND", "-D__HIP_PLATFORM_AMD__=1",
             f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
             "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(CSRC, "torch"), "-I/opt/rocm/include"]
    flags += ["-I" + p for p in cpp_extension.include_paths()]
    # One HIP runtime per process: the torch wheel bundles its own libamdhip64 (soname
    # libamdhip64.so.7, file libamdhip64.so) and libtorch_hip names it by file name, while
    # libgsr_hip.so asks for libamdhip64.so.7.  The loader resolves dependencies breadth-first
    # in NEEDED order, so libtorch_hip goes ahead of libgsr_hip: the wheel's runtime is loaded
    # first and libgsr_hip's request is then satisfied by soname with that same copy.  With
    # libgsr_hip first, /opt/rocm's runtime is loaded as a second one (two HIP and HSA runtimes,
    # torch's streams handed to the other, a double free at exit).
    # RCCL: the wheel's own librccl.so (the one libtorch_hip loads), so the process has one RCCL
    libs = ["-L" + tlib, "-Wl,--no-as-needed", "-ltorch_hip", "-lc10_hip",
            "-Wl,--as-needed", "-ltorch", "-ltorch_cpu", "-lc10", "-L" + LIB, "-lgsr_hip",
            "-Wl,-rpath," + tlib, "-Wl,-rpath,$ORIGIN"]
    return flags, libs


# the libtorch layer shared by the C++ executables (compiled once, -DGSR_NO_PYBIND)
EXE_LIB_SOURCES = [os.path.join(CSRC, "torch", f) for f in ("gsr_torch.cpp", "gsr_trainer.cpp", "gsr_shard.cpp")]
EXE_HEADERS = [os.path.join(CSRC, "torch", h) for h in ("gsr_render.h", "gsr_trainer.h", "gsr_shard.h")]


def _compile_exe_objs(flags, force: bool) -> list:
    """gsr_torch.cpp + gsr_trainer.cpp -> lib/obj/*.o (content-stamped)."""
    obj_dir = os.path.join(LIB, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    cxx = shutil.which("g++") or "c++"

    def one(src):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        stamp = _stamp([src] + _headers() + EXE_HEADERS, " ".join(flags))
        if not force and os.path.exists(obj) and os.path.exists(obj + ".stamp") and open(obj + ".stamp").read() == stamp:
            return obj
        cmd = [cxx] + flags + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        with open(obj + ".stamp", "w") as fh:
            fh.write(stamp)
        return obj

    with cf.ThreadPoolExecutor(max_workers=len(EXE_LIB_SOURCES)) as ex:
        return list(ex.map(one, EXE_LIB_SOURCES))


def _build_exe(name: str, main_src: str, force: bool = False) -> str:
    flags, libs = _exe_flags()
    objs = _compile_exe_objs(flags, force)
    out = os.path.join(LIB, name)
    stamp = _stamp([main_src] + EXE_LIB_SOURCES + _headers() + EXE_HEADERS, " ".join(flags + libs))
    stamp_file = out + ".stamp"
    if not force and os.path.exists(out) and os.path.exists(stamp_file) and open(stamp_file).read() == stamp:
        return out
    cxx = shutil.which("g++") or "c++"
    cmd = [cxx] + flags + [main_src] + objs + ["-o", out] + libs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{name} build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp_file, "w") as fh:
        fh.write(stamp)
    return out


def build_dropin(verbose: bool = False, force: bool = False) -> str:
    """tests/cpp/dropin_main.cpp + the libtorch layer into the C++ executable lib/gsr_dropin:
    gsr::render() compiled against the reference's call surface (tests/test_gpu_dropin.py)."""
    return _build_exe("gsr_dropin", os.path.join(ROOT, "tests", "cpp", "dropin_main.cpp"), force)


def build_train_loop(verbose: bool = False, force: bool = False) -> str:
    """tests/cpp/train_main.cpp + the libtorch layer into lib/gsr_train_loop: the reference's
    train() loop (train_utils.cpp:128-145) over gsr::Trainer (tests/test_gpu_train_loop.py,
    bench.py --mode loop)."""
    return _build_exe("gsr_train_loop", os.path.join(ROOT, "tests", "cpp", "train_main.cpp"), force)


def build_shard_step(verbose: bool = False, force: bool = False) -> str:
    """tests/cpp/shard_main.cpp + the libtorch layer into lib/gsr_shard_step: one rank of the
    C++ multi-GPU step (gsr::ShardStep over RCCL or a store exchange; tests/test_gpu_shard_cpp.py)."""
    return _build_exe("gsr_shard_step", os.path.join(ROOT, "tests", "cpp", "shard_main.cpp"), force)


def build_all(verbose: bool = False, force: bool = False):
    so = build_hip(verbose, force)
    ext = build_torch_ext(verbose, force)
    build_dropin(verbose, force)
    build_train_loop(verbose, force)
    build_shard_step(verbose, force)
    return so, ext


if __name__ == "__main__":
    print(build_all(verbose=True, force="--force" in sys.argv))

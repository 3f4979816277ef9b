"""Scene I/O: COLMAP binary models, point-cloud and Gaussian PLY files,
training checkpoints.

Host-side byte parsing with numpy / struct (little-endian, packed, as COLMAP writes them);
nothing here is on the GPU hot path.  What each function restates:

  - ``read_intrinsics_binary``   src/scene/colmap_loader.cpp:222-249 (cameras.bin: "Q" count,
    then per camera "iiQQ" + num_params doubles; model table :194-206)
  - ``read_extrinsics_binary``   src/scene/colmap_loader.cpp:120-170 (images.bin: "Q" count,
    then "idddddddi", a NUL-terminated name, "Q" + num_points2D x "ddq")
  - ``qvec2rotmat``              src/scene/colmap_loader.cpp:265-279
  - ``read_colmap_cameras``      src/scene/dataset_readers.cpp:40-95 (PINHOLE / SIMPLE_PINHOLE
    only, R = qvec2rotmat(q)^T, FoV from focal2fov, uid = the intrinsics id)
  - ``get_center_and_diag`` / ``get_nerfpp_norm``  dataset_readers.cpp:100-137
  - ``read_colmap_scene_info``   dataset_readers.cpp:140-196: cameras sorted by image name,
    llffhold train/test split.  The reference stops there -- its points3D / PLY branch is
    commented out (:198-219) and the function returns void; this build
    finishes the upstream behaviour that comment sketches: points3D.bin -> points3D.ply on
    first open, then the point cloud from the PLY, returned in a SceneInfo.
  - ``read_points3D_binary``, ``store_ply``, ``fetch_ply``: the upstream formats that comment
    names (points3D.bin: "Q" count, then "QdddBBBd" + "Q" track length + track x "ii").
  - ``save_gaussians_ply`` / ``load_gaussians_ply``: the upstream 3DGS point-cloud layout
    (x y z nx ny nz f_dc_* f_rest_* opacity scale_* rot_*, raw pre-activation values, SH
    coefficients channel-major), which the usual splat viewers read.
  - ``save_checkpoint`` / ``load_checkpoint``: GaussianModel::capture / restore
    (src/scene/gaussian_model.cpp:76-202): the CoreParams tensor list in the reference's order
    plus each parameter group's Adam state, loadable with torch.load(weights_only=True).

Images are not decoded (OpenCV is absent here and out of scope): ``CameraInfo`` carries the
path and ``image`` stays None unless the caller fills it.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass

import numpy as np

from .graphics import RasterCamera, focal2fov, get_world2view_2, make_camera

# colmap_loader.cpp:194-206: model_id -> (name, num_params)
CAMERA_MODELS = {
    0: ("SIMPLE_PINHOLE", 3),
    1: ("PINHOLE", 4),
    2: ("SIMPLE_RADIAL", 4),
    3: ("RADIAL", 5),
    4: ("OPENCV", 8),
    5: ("OPENCV_FISHEYE", 8),
    6: ("FULL_OPENCV", 12),
    7: ("FOV", 5),
    8: ("SIMPLE_RADIAL_FISHEYE", 4),
    9: ("RADIAL_FISHEYE", 5),
    10: ("THIN_PRISM_FISHEYE", 12),
}
_MODEL_IDS = {name: (mid, n) for mid, (name, n) in CAMERA_MODELS.items()}


@dataclass
class ColmapCamera:
    """colmap_loader.h Camera: id, model name, width, height, params."""
    id: int
    model: str
    width: int
    height: int
    params: np.ndarray


@dataclass
class ColmapImage:
    """colmap_loader.h Image: id, qvec (w, x, y, z), tvec, camera_id, name, xys, point3D_ids."""
    id: int
    qvec: np.ndarray
    tvec: np.ndarray
    camera_id: int
    name: str
    xys: np.ndarray
    point3D_ids: np.ndarray


@dataclass
class CameraInfo:
    """dataset_readers.h CameraInfo (dataset_readers.cpp:14-36)."""
    uid: int
    R: np.ndarray
    T: np.ndarray
    FovY: float
    FovX: float
    image_path: str
    image_name: str
    width: int
    height: int
    image: object = None


@dataclass
class BasicPointCloud:
    points: np.ndarray   # (N, 3)
    colors: np.ndarray   # (N, 3) in [0, 1]
    normals: np.ndarray  # (N, 3)


@dataclass
class SceneInfo:
    point_cloud: BasicPointCloud | None
    train_cameras: list
    test_cameras: list
    nerf_normalization: dict
    ply_path: str = ""


class _Reader:
    """Sequential little-endian reader over a whole file, bounds-checked."""

    def __init__(self, path: str):
        with open(path, "rb") as f:
            self.buf = f.read()
        self.pos = 0
        self.path = path

    def _need(self, n: int):
        if self.pos + n > len(self.buf):
            raise ValueError(f"{self.path}: truncated at byte {self.pos} (need {n} more)")

    def take(self, fmt: str):
        n = struct.calcsize("<" + fmt)
        self._need(n)
        v = struct.unpack_from("<" + fmt, self.buf, self.pos)
        self.pos += n
        return v

    def array(self, dtype, count: int) -> np.ndarray:
        dt = np.dtype(dtype)
        self._need(dt.itemsize * count)
        a = np.frombuffer(self.buf, dtype=dt, count=count, offset=self.pos).copy()
        self.pos += dt.itemsize * count
        return a

    def cstring(self) -> str:
        end = self.buf.find(b"\0", self.pos)
        if end < 0:
            raise ValueError(f"{self.path}: unterminated name at byte {self.pos}")
        s = self.buf[self.pos:end].decode("utf-8")
        self.pos = end + 1
        return s


def _open_check(path: str):
    if not os.path.isfile(path):
        raise RuntimeError("Unable to open file: " + path)  # colmap_loader.cpp:123-126


def read_intrinsics_binary(path: str) -> dict[int, ColmapCamera]:
    """cameras.bin -> {camera_id: ColmapCamera} (colmap_loader.cpp:222-249)."""
    _open_check(path)
    r = _Reader(path)
    (n,) = r.take("Q")
    cams = {}
    for _ in range(n):
        cid, mid, w, h = r.take("iiQQ")
        if mid not in CAMERA_MODELS:  # CAMERA_MODEL_IDS.at() throws
            raise KeyError(f"{path}: unknown COLMAP camera model id {mid}")
        name, npar = CAMERA_MODELS[mid]
        cams[cid] = ColmapCamera(cid, name, int(w), int(h), r.array("<f8", npar))
    return cams


_XYID = np.dtype([("x", "<f8"), ("y", "<f8"), ("id", "<i8")])


def read_extrinsics_binary(path: str) -> dict[int, ColmapImage]:
    """images.bin -> {image_id: ColmapImage} (colmap_loader.cpp:120-170)."""
    _open_check(path)
    r = _Reader(path)
    (n,) = r.take("Q")
    images = {}
    for _ in range(n):
        props = r.take("idddddddi")
        iid, cam_id = props[0], props[8]
        name = r.cstring()
        (npts,) = r.take("Q")
        rec = r.array(_XYID, npts)
        xys = np.stack([rec["x"], rec["y"]], axis=1) if npts else np.zeros((0, 2))
        images[iid] = ColmapImage(iid, np.array(props[1:5], np.float64), np.array(props[5:8], np.float64), cam_id,
                                  name, xys, rec["id"].astype(np.int64))
    return images


def read_points3D_binary(path: str):
    """points3D.bin -> (xyz (N,3) f64, rgb (N,3) u8, error (N,) f64): the upstream reader the
    reference's commented branch calls (dataset_readers.cpp:204)."""
    _open_check(path)
    r = _Reader(path)
    (n,) = r.take("Q")
    xyz = np.empty((n, 3), np.float64)
    rgb = np.empty((n, 3), np.uint8)
    err = np.empty(n, np.float64)
    for i in range(n):
        v = r.take("QdddBBBd")
        xyz[i] = v[1:4]
        rgb[i] = v[4:7]
        err[i] = v[7]
        (track_len,) = r.take("Q")
        r._need(8 * track_len)  # track: (image_id i32, point2D_idx i32) pairs, skipped
        r.pos += 8 * track_len
    return xyz, rgb, err


def write_intrinsics_binary(path: str, cams: dict[int, ColmapCamera]) -> None:
    """Inverse of read_intrinsics_binary (dataset tooling, test fixtures)."""
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(cams)))
        for cid, c in cams.items():
            mid, npar = _MODEL_IDS[c.model]
            p = np.asarray(c.params, dtype="<f8").reshape(-1)
            if p.size != npar:
                raise ValueError(f"{c.model} takes {npar} params, got {p.size}")
            f.write(struct.pack("<iiQQ", cid, mid, c.width, c.height) + p.tobytes())


def write_extrinsics_binary(path: str, images: dict[int, ColmapImage]) -> None:
    """Inverse of read_extrinsics_binary."""
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(images)))
        for iid, im in images.items():
            f.write(struct.pack("<idddddddi", iid, *map(float, im.qvec), *map(float, im.tvec), im.camera_id))
            f.write(im.name.encode("utf-8") + b"\0")
            xys = np.asarray(im.xys, np.float64).reshape(-1, 2)
            rec = np.empty(len(xys), _XYID)
            rec["x"], rec["y"] = xys[:, 0], xys[:, 1]
            rec["id"] = np.asarray(im.point3D_ids, np.int64).reshape(-1)
            f.write(struct.pack("<Q", len(xys)) + rec.tobytes())


def write_points3D_binary(path: str, xyz, rgb, err=None, tracks=None) -> None:
    """Inverse of read_points3D_binary (ids 1..N; tracks: per point a list of (image, idx))."""
    xyz = np.asarray(xyz, np.float64).reshape(-1, 3)
    rgb = np.asarray(rgb, np.uint8).reshape(-1, 3)
    n = len(xyz)
    err = np.zeros(n) if err is None else np.asarray(err, np.float64)
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", n))
        for i in range(n):
            f.write(struct.pack("<QdddBBBd", i + 1, *xyz[i], *map(int, rgb[i]), err[i]))
            tr = np.zeros((0, 2), "<i4") if tracks is None else np.asarray(tracks[i], "<i4").reshape(-1, 2)
            f.write(struct.pack("<Q", len(tr)) + tr.tobytes())


def qvec2rotmat(q) -> np.ndarray:
    """colmap_loader.cpp:265-279 (q = (w, x, y, z), not normalised)."""
    w, x, y, z = (float(v) for v in q)
    return np.array([
        [1 - 2 * y * y - 2 * z * z, 2 * x * y - 2 * w * z, 2 * z * x + 2 * w * y],
        [2 * x * y + 2 * w * z, 1 - 2 * x * x - 2 * z * z, 2 * y * z - 2 * w * x],
        [2 * z * x - 2 * w * y, 2 * y * z + 2 * w * x, 1 - 2 * x * x - 2 * y * y],
    ])


def read_colmap_cameras(extr: dict[int, ColmapImage], intr: dict[int, ColmapCamera],
                        images_folder: str) -> list[CameraInfo]:
    """dataset_readers.cpp:40-95."""
    out = []
    for e in extr.values():
        c = intr[e.camera_id]
        if c.model == "SIMPLE_PINHOLE":
            fovy, fovx = focal2fov(c.params[0], c.height), focal2fov(c.params[0], c.width)
        elif c.model == "PINHOLE":
            fovy, fovx = focal2fov(c.params[1], c.height), focal2fov(c.params[0], c.width)
        else:
            raise RuntimeError("Colmap camera model not handled: only undistorted datasets "
                               "(PINHOLE or SIMPLE_PINHOLE cameras) supported!")
        base = os.path.basename(e.name)
        out.append(CameraInfo(uid=c.id, R=qvec2rotmat(e.qvec).T, T=np.array(e.tvec, np.float64), FovY=fovy,
                              FovX=fovx, image_path=os.path.join(images_folder, base),
                              image_name=os.path.splitext(base)[0], width=c.width, height=c.height))
    return out


def get_center_and_diag(cam_centers) -> tuple[np.ndarray, float]:
    """dataset_readers.cpp:101-120: the mean centre and the largest distance to it."""
    c = np.asarray(cam_centers, np.float64).reshape(-1, 3)
    avg = c.sum(axis=0) / len(c)
    return avg, float(np.max(np.linalg.norm(c - avg, axis=1)))


def get_nerfpp_norm(cam_infos: list[CameraInfo]) -> dict:
    """dataset_readers.cpp:122-137: translate = -centre, radius = 1.1 x diagonal."""
    centers = [np.linalg.inv(get_world2view_2(ci.R, ci.T))[:3, 3] for ci in cam_infos]
    center, diag = get_center_and_diag(centers)
    return {"translate": -center, "radius": diag * 1.1}


def camera_from_info(ci: CameraInfo, trans=(0.0, 0.0, 0.0), scale: float = 1.0) -> RasterCamera:
    """Camera (camera.cpp:66-71) of a CameraInfo, as the rasterizer consumes it."""
    return make_camera(ci.R, ci.T, ci.FovX, ci.FovY, ci.width, ci.height, trans, scale)


# ---- PLY ----
_PLY_TYPES = {"float": "f4", "float32": "f4", "double": "f8", "float64": "f8", "uchar": "u1",
              "uint8": "u1", "char": "i1", "int8": "i1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4"}
_PLY_NAMES = {"f4": "float", "f8": "double", "u1": "uchar", "i1": "char", "i2": "short",
              "u2": "ushort", "i4": "int", "u4": "uint"}


def write_ply(path: str, columns: dict[str, np.ndarray]) -> None:
    """Binary little-endian PLY with one 'vertex' element, columns in the given order."""
    names = list(columns)
    n = len(next(iter(columns.values()))) if names else 0
    dt = np.dtype([(k, "<" + np.asarray(columns[k]).dtype.str[1:]) for k in names])
    rec = np.empty(n, dt)
    for k in names:
        rec[k] = columns[k]
    head = ["ply", "format binary_little_endian 1.0", f"element vertex {n}"]
    head += [f"property {_PLY_NAMES[dt[k].str[1:]]} {k}" for k in names]
    head.append("end_header")
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode("ascii"))
        f.write(rec.tobytes())


def read_ply(path: str) -> dict[str, np.ndarray]:
    """The 'vertex' element of a binary (either endianness) or ASCII PLY, as columns."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.find(b"end_header")
    if not data.startswith(b"ply") or end < 0:
        raise ValueError(f"{path}: not a PLY file")
    body = data[data.find(b"\n", end) + 1:]
    fmt, elems, cur = None, [], None
    for line in data[:end].decode("ascii").splitlines():
        t = line.split()
        if not t:
            continue
        if t[0] == "format":
            fmt = t[1]
        elif t[0] == "element":
            cur = [t[1], int(t[2]), []]
            elems.append(cur)
        elif t[0] == "property":
            if t[1] == "list":
                raise ValueError(f"{path}: list properties are not supported")
            cur[2].append((t[2], _PLY_TYPES[t[1]]))
    if fmt not in ("binary_little_endian", "binary_big_endian", "ascii"):
        raise ValueError(f"{path}: unsupported PLY format {fmt}")
    off = 0
    for name, count, props in elems:
        if fmt == "ascii":
            if name != "vertex":
                raise ValueError(f"{path}: ASCII PLY with elements before 'vertex'")
            rows = [r.split() for r in body.decode("ascii").splitlines()[:count]]
            arr = np.array(rows, dtype=np.float64).reshape(count, len(props))
            return {p: arr[:, i].astype(t) for i, (p, t) in enumerate(props)}
        e = "<" if fmt == "binary_little_endian" else ">"
        dt = np.dtype([(p, e + t) for p, t in props])
        if name == "vertex":
            rec = np.frombuffer(body, dtype=dt, count=count, offset=off)
            return {p: rec[p].astype(t) for p, t in props}
        off += dt.itemsize * count
    raise ValueError(f"{path}: no vertex element")


def store_ply(path: str, xyz, rgb) -> None:
    """Upstream storePly: x y z (f32), nx ny nz (zeros), red green blue (u8)."""
    xyz = np.asarray(xyz, np.float32).reshape(-1, 3)
    rgb = np.asarray(rgb, np.uint8).reshape(-1, 3)
    z = np.zeros(len(xyz), np.float32)
    write_ply(path, {"x": xyz[:, 0], "y": xyz[:, 1], "z": xyz[:, 2], "nx": z, "ny": z, "nz": z,
                     "red": rgb[:, 0], "green": rgb[:, 1], "blue": rgb[:, 2]})


def fetch_ply(path: str) -> BasicPointCloud:
    """Upstream fetchPly: positions, colours / 255, normals (zeros when absent)."""
    c = read_ply(path)
    pts = np.stack([c["x"], c["y"], c["z"]], 1)
    col = np.stack([c["red"], c["green"], c["blue"]], 1).astype(np.float64) / 255.0
    nrm = np.stack([c["nx"], c["ny"], c["nz"]], 1) if "nx" in c else np.zeros_like(pts)
    return BasicPointCloud(pts, col, nrm)


def read_colmap_scene_info(path: str, images: str = "", eval: bool = False, llffhold: int = 8) -> SceneInfo:
    """dataset_readers.cpp:140-196, plus the upstream point-cloud tail it leaves commented."""
    sparse = os.path.join(path, "sparse", "0")
    try:
        extr = read_extrinsics_binary(os.path.join(sparse, "images.bin"))
        intr = read_intrinsics_binary(os.path.join(sparse, "cameras.bin"))
    except (RuntimeError, ValueError, KeyError) as exc:
        # the reference's text readers are stubs and it throws here (Appendix A.8)
        raise RuntimeError("Not implemented: COLMAP text models (sparse/0/*.txt)") from exc
    cams = sorted(read_colmap_cameras(extr, intr, os.path.join(path, images or "images")),
                  key=lambda c: c.image_name)
    if eval:
        train = [c for i, c in enumerate(cams) if i % llffhold != 0]
        test = [c for i, c in enumerate(cams) if i % llffhold == 0]
    else:
        train, test = cams, []
    norm = get_nerfpp_norm(train) if train else {"translate": np.zeros(3), "radius": 0.0}
    ply_path = os.path.join(sparse, "points3D.ply")
    bin_path = os.path.join(sparse, "points3D.bin")
    if not os.path.exists(ply_path) and os.path.exists(bin_path):
        xyz, rgb, _ = read_points3D_binary(bin_path)
        store_ply(ply_path, xyz, rgb)
    try:
        pcd = fetch_ply(ply_path)
    except (OSError, ValueError, KeyError):
        pcd = None
    return SceneInfo(pcd, train, test, norm, ply_path)


# ---- Gaussians in the upstream PLY layout ----
def gaussian_ply_attributes(n_rest_coeffs: int) -> list[str]:
    """Upstream construct_list_of_attributes order for n_rest_coeffs SH-rest coefficients."""
    names = ["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(3)]
    names += [f"f_rest_{i}" for i in range(3 * n_rest_coeffs)]
    return names + ["opacity"] + [f"scale_{i}" for i in range(3)] + [f"rot_{i}" for i in range(4)]


def _host(a) -> np.ndarray:
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.asarray(a, np.float32)


def save_gaussians_ply(path: str, xyz, f_dc, f_rest, opacity, scaling, rotation) -> None:
    """Raw (pre-activation) leaves -> PLY.  f_dc (N,1,3) and f_rest (N,M,3) are stored
    channel-major (transpose(1,2).flatten, the upstream save_ply layout)."""
    xyz = _host(xyz).reshape(-1, 3)
    n = len(xyz)
    dc = _host(f_dc).reshape(n, -1, 3).transpose(0, 2, 1).reshape(n, -1)
    rest = _host(f_rest).reshape(n, -1, 3).transpose(0, 2, 1).reshape(n, -1)
    cols = np.concatenate([xyz, np.zeros_like(xyz), dc, rest, _host(opacity).reshape(n, 1),
                           _host(scaling).reshape(n, 3), _host(rotation).reshape(n, 4)], axis=1)
    names = gaussian_ply_attributes(rest.shape[1] // 3)
    write_ply(path, {k: np.ascontiguousarray(cols[:, i]) for i, k in enumerate(names)})


def load_gaussians_ply(path: str, max_sh_degree: int = 3) -> dict[str, np.ndarray]:
    """PLY -> raw leaves {xyz (N,3), f_dc (N,1,3), f_rest (N,M,3), opacity (N,1), scaling (N,3),
    rotation (N,4)}; the file must hold 3 M = 3 ((max_sh_degree+1)^2 - 1) f_rest columns (the
    upstream load_ply assertion)."""
    c = read_ply(path)
    n = len(c["x"])

    def group(prefix):
        ks = sorted((k for k in c if k.startswith(prefix)), key=lambda k: int(k.rsplit("_", 1)[1]))
        return np.stack([c[k] for k in ks], 1).astype(np.float32) if ks else np.zeros((n, 0), np.float32)
    m = (max_sh_degree + 1) ** 2 - 1
    rest = group("f_rest_")
    if rest.shape[1] != 3 * m:
        raise ValueError(f"{path}: {rest.shape[1]} f_rest columns, expected {3 * m} for SH degree {max_sh_degree}")
    return {"xyz": np.stack([c["x"], c["y"], c["z"]], 1).astype(np.float32),
            "f_dc": np.ascontiguousarray(group("f_dc_").reshape(n, 3, 1).transpose(0, 2, 1)),
            "f_rest": np.ascontiguousarray(rest.reshape(n, 3, m).transpose(0, 2, 1)),
            "opacity": c["opacity"].astype(np.float32).reshape(n, 1),
            "scaling": group("scale_"), "rotation": group("rot_")}


# ---- training checkpoints (GaussianModel::capture / restore) ----
_CORE = ("xyz", "f_dc", "f_rest", "scaling", "rotation", "opacity")  # gaussian_model.cpp:85-97
_STATS = ("max_radii2D", "xyz_gradient_accum", "denom")


def save_checkpoint(path: str, state: dict) -> None:
    """One file holding the reference's CoreParams tensor list in its order -- [active_sh_degree,
    xyz, f_dc, f_rest, scaling, rotation, opacity, max_radii2D, xyz_gradient_accum, denom,
    spatial_lr_scale] (gaussian_model.cpp:85-98) -- and, in place of its six per-group
    torch::optim::Adam archives (:100-130), each group's exp_avg / exp_avg_sq / step.
    spatial_lr_scale is a float32 scalar, as the reference's CoreParams::spatial_lr_scale_ is a
    float; the densification extent (cameras_extent, not a reference field) rides along in
    float64."""
    import torch
    cpu = lambda t: t.detach().to("cpu").contiguous()
    p = state["params"]
    core = [torch.tensor(int(state["active_sh_degree"]))] + [cpu(p[k]) for k in _CORE]
    core += [cpu(state[k]) for k in _STATS] + [torch.tensor(float(state["spatial_lr_scale"]))]
    optim = {k: {"exp_avg": cpu(state["exp_avg"][k]), "exp_avg_sq": cpu(state["exp_avg_sq"][k]),
                 "step": torch.tensor(int(state["steps"][k]))} for k in p if k in state["exp_avg"]}
    extra = {}
    if "cameras_extent" in state:
        extra["cameras_extent"] = torch.tensor(float(state["cameras_extent"]), dtype=torch.float64)
    torch.save({"core": core, "optim": optim, "extra": extra}, path)


def load_checkpoint(path: str, device="cpu") -> dict:
    """Inverse of save_checkpoint (torch.load with weights_only=True: nothing executes)."""
    import torch
    raw = torch.load(path, map_location=device, weights_only=True)
    core = raw["core"]
    st = {"active_sh_degree": int(core[0].item()), "params": dict(zip(_CORE, core[1:7])),
          "spatial_lr_scale": float(core[10].item())}
    st.update(zip(_STATS, core[7:10]))
    st["exp_avg"] = {k: v["exp_avg"] for k, v in raw["optim"].items()}
    st["exp_avg_sq"] = {k: v["exp_avg_sq"] for k, v in raw["optim"].items()}
    st["steps"] = {k: int(v["step"].item()) for k, v in raw["optim"].items()}
    for k, v in raw.get("extra", {}).items():
        st[k] = float(v.item())
    return st


# ---- point-cloud initialisation constants (upstream sh_utils / general_utils) ----
SH_C0 = 0.28209479177387814


def rgb2sh(rgb):
    return (np.asarray(rgb, np.float64) - 0.5) / SH_C0


def sh2rgb(sh):
    return np.asarray(sh, np.float64) * SH_C0 + 0.5

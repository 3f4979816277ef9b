"""Shared test setup.  Markers: ``gpu`` = needs an MI355X (HIP kernels through the C ABI)."""
from __future__ import annotations

import glob
import importlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

PKG_NAME = "3d_gaussian_splatting_amd"
GOLDEN = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.npz")))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU (HIP kernels)")


def pkg(sub: str | None = None):
    return importlib.import_module(PKG_NAME if sub is None else f"{PKG_NAME}.{sub}")


def load_fixture(path):
    z = np.load(path, allow_pickle=False)
    meta = json.loads(bytes(z["meta_json"]).decode())
    gr = pkg("graphics")
    cam = gr.RasterCamera(meta["W"], meta["H"], meta["tanfovx"], meta["tanfovy"],
                          np.array(meta["viewmatrix"], np.float32), np.array(meta["projmatrix"], np.float32),
                          np.array(meta["campos"], np.float32))
    inp = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    out = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return meta, cam, inp, out


def rel_l2(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    nb = np.linalg.norm(b)
    if nb == 0.0:
        return float(np.linalg.norm(a))
    return float(np.linalg.norm(a - b) / nb)


def psnr(a, b) -> float:
    mse = float(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2))
    return float("inf") if mse == 0 else 10.0 * np.log10(1.0 / mse)


@pytest.fixture(scope="session")
def oracle():
    import gsr_oracle
    gsr_oracle.build()
    return gsr_oracle

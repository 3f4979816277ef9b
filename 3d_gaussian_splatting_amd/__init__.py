"""gsr -- MI355X-native differentiable 3D Gaussian splat rasterizer.

Drop-in for the render()/backward() hot path of seiya-kumada/3d_gaussian_splatting
(insertion point src/utils/train_utils.cpp:137-144).  Layers:

  include/gsr/gsr.h              C ABI (plain pointers, sizes, hipStream_t)
  csrc/*.hip -> lib/libgsr_hip.so  hand-written CDNA4 kernels behind that ABI
  csrc/torch/gsr_torch.cpp -> lib/_gsr_torch*.so  libtorch render() + autograd Function
  rasterizer.py                   Python mirror of the same surface (tests / bench)

Importing the package does not touch the GPU.  ``native`` loads the shared libraries
and raises if they are missing: there is no CPU fallback in the product path.
"""
from . import graphics, scene  # noqa: F401

__all__ = ["graphics", "scene"]

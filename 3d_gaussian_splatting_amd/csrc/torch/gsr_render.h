// gsr_render.h -- libtorch render() surface for the reference's C++ training loop.
//
// The reference (seiya-kumada/3d_gaussian_splatting) has no renderer; its loop body is a stub
// at src/utils/train_utils.cpp:128-145.  This header gives that loop the call it is missing:
//
//     auto out = gsr::render(cam, *gaussians, pipeline_params, bg, 1.f, std::nullopt, &binning);
//     auto loss = gsr::photometric_loss(out.render, gt, lambda_dssim);  loss.backward();
//
// (bg: gsr::background(background_tensor), read once before the loop; binning: a
// gsr::BinningCapacity, so no forward waits on the host for the instance count K.)
//
// `Model` is the reference's GaussianModel (src/scene/gaussian_model.h): render() only uses
// its public getters (get_xyz / get_opacity / get_scaling / get_rotation / get_covariance,
// gaussian_model.h:85-90), get_core_params() for active_sh_degree_ and the raw SH leaves
// (features_dc_ / features_rest_, gaussian_model.h:12-14 -- passed separately so the
// get_features() cat copy, gaussian_model.cpp:289-292, is never made) and get_max_sh_degree().
// `Pipe` is PipelineParams (src/arguments/params.h:93-106): convert_SHs_python_,
// compute_cov3D_python_, debug_.
#pragma once
#include <torch/torch.h>

#include <array>
#include <cmath>
#include <cstdint>
#include <optional>
#include <vector>

#include "gsr/gsr.h"

namespace gsr {

// POD view the rasterizer consumes (f32, column-major matrices: the reference Camera's
// row-vector-convention tensors flattened row-major, src/scene/camera.cpp:66-71).
struct RasterCamera {
    int width = 0, height = 0;
    float tanfovx = 0.f, tanfovy = 0.f;
    std::array<float, 16> viewmatrix{};
    std::array<float, 16> projmatrix{};
    std::array<float, 3> campos{};
    float znear = 0.01f, zfar = 100.f;

    // From the reference Camera's device tensors (world_view_transform_, full_proj_transform_,
    // camera_center_: camera.cpp:66-71) -- one host copy per camera, not per iteration.
    static RasterCamera from_tensors(int width, int height, double FoVx, double FoVy,
                                     const torch::Tensor& world_view_transform,
                                     const torch::Tensor& full_proj_transform,
                                     const torch::Tensor& camera_center);
    gsr_camera to_c() const;
};

struct RasterSettings {
    std::array<float, 3> bg{0.f, 0.f, 0.f};
    float scale_modifier = 1.f;
    int sh_degree = 0;
    int tile_y0 = 0, tile_y1 = INT32_MAX;  // tile-row band
    bool debug = false;
    int max_rendered = 0;  // > 0: binning sized for this many instances, no host read (gsr.h)
};

struct RenderOutput {
    torch::Tensor render;             // (3,H,W)
    torch::Tensor viewspace_points;   // (P,3) zeros requiring grad: receives dL/dmeans2D
    torch::Tensor visibility_filter;  // (P,) bool, radii > 0
    torch::Tensor radii;              // (P,) int32
    torch::Tensor num_rendered_device;  // (1,) int32 on the device: K (no host wait to get it)
    int num_rendered = -1;              // K when the forward read it back (max_rendered == 0), else -1
    int capacity = 0;                   // instances the forward's binning held
};

// K of a render, read back now (waits for the render's stream): gsr_read_num_rendered's
// contract -- throws std::overflow_error when K exceeded the capacity (the render dropped
// instances past it; re-run with a larger bound).
int read_num_rendered(const RenderOutput& out);

// A binning bound for a training loop's renders (the C++ twin of trainer.BinningCapacity):
// bound() is 0 right after the point set changes (that render sizes its binning exactly: one
// host read of K), afterwards headroom x the largest K seen; observe() copies each bounded
// render's K to pinned memory without waiting and checks it once the copy has landed, one or
// more iterations later.  A render found above its bound was truncated and the iteration that
// used it already applied: overflows() counts it, the next render is sized exactly, and with
// strict = true the check throws std::overflow_error instead.
class BinningCapacity {
   public:
    explicit BinningCapacity(double headroom = 1.5, int ring = 8, bool strict = false);
    ~BinningCapacity();
    BinningCapacity(const BinningCapacity&) = delete;
    BinningCapacity& operator=(const BinningCapacity&) = delete;
    int bound();                        // max_rendered for the next render (0 = exact)
    void observe(const RenderOutput& out);
    void observe(const torch::Tensor& k_device, int host_k);
    void reset();                       // the point set changed
    void sync();                        // wait for every pending check
    int64_t overflows() const { return overflows_; }
    int64_t exact_reads() const { return exact_reads_; }
    int64_t k_max() const { return k_max_; }
    int cap() const { return cap_; }

   private:
    struct Pending {
        int slot;
        void* event;
        int cap;
    };
    void poll(bool wait);
    void grow();
    double headroom_;
    bool strict_;
    int cap_ = 0;
    int64_t k_max_ = 0, overflows_ = 0, exact_reads_ = 0;
    std::vector<torch::Tensor> slots_;
    std::vector<void*> events_;
    std::vector<Pending> pending_;
    int next_ = 0;
};

// Background colour as host floats (one device read; do it once, outside the loop -- the
// reference keeps its background as a device tensor, train_utils.cpp:115-117).
std::array<float, 3> background(const torch::Tensor& bg);

// Differentiable rasterization (RasterizeGaussians autograd Function).  Absent optional
// inputs are undefined tensors.  Returns {color (3,H,W), radii (P,) int32, K (1,) int32 on the
// device, {host K or -1, capacity} (2,) int32 on the host}.
std::vector<torch::Tensor> rasterize_gaussians(
    const RasterCamera& cam, const RasterSettings& rs, const torch::Tensor& means3D,
    const torch::Tensor& means2D, const torch::Tensor& sh_dc, const torch::Tensor& sh_rest,
    const torch::Tensor& colors_precomp, const torch::Tensor& opacities, const torch::Tensor& scales,
    const torch::Tensor& rotations, const torch::Tensor& cov3D_precomp);

// torch-op SH evaluation (PipelineParams::convert_SHs_python_ path): colours for
// directions (P,3) and coefficients (P,M,3) at degree D; +0.5 and clamp at 0 as in-kernel.
torch::Tensor eval_sh_colors(int D, const torch::Tensor& sh, const torch::Tensor& dirs);

template <class Model, class Pipe>
RenderOutput render(const RasterCamera& cam, Model& pc, const Pipe& pipe, const std::array<float, 3>& bg,
                    float scaling_modifier = 1.f, std::optional<torch::Tensor> override_color = std::nullopt,
                    BinningCapacity* binning = nullptr) {
    const auto& xyz = pc.get_xyz();
    auto screenspace = torch::zeros_like(xyz).requires_grad_(true);
    RasterSettings rs;
    rs.bg = bg;
    rs.scale_modifier = scaling_modifier;
    auto& core = pc.get_core_params();
    rs.sh_degree = core.active_sh_degree_;
    rs.debug = pipe.debug_;
    rs.max_rendered = binning ? binning->bound() : 0;
    torch::Tensor scales, rotations, cov3D, sh_dc, sh_rest, colors;
    // The reference's GaussianModel::get_covariance takes an int modifier
    // (gaussian_model.h:89), so it is called only with an integral one; any other modifier is
    // applied in-kernel to get_scaling() (F1 builds the same R S S^T R^T covariance,
    // general_utils.cpp:88-99) instead of being truncated to an int.
    if (pipe.compute_cov3D_python_ && scaling_modifier == std::nearbyint(scaling_modifier)) {
        cov3D = pc.get_covariance(static_cast<int>(scaling_modifier));
    } else {
        scales = pc.get_scaling();
        rotations = pc.get_rotation();
    }
    if (override_color) {
        colors = *override_color;
    } else if (pipe.convert_SHs_python_) {
        auto feats = pc.get_features();  // (P, M, 3)
        auto cpos = torch::from_blob(const_cast<float*>(cam.campos.data()), {1, 3}, torch::kFloat32)
                        .to(xyz.device());
        auto dirs = xyz - cpos;
        dirs = dirs / dirs.norm(2, 1, true);
        colors = eval_sh_colors(core.active_sh_degree_, feats, dirs);
    } else {
        sh_dc = core.features_dc_;
        sh_rest = core.features_rest_;
    }
    std::vector<torch::Tensor> outs = rasterize_gaussians(cam, rs, xyz, screenspace, sh_dc, sh_rest, colors, pc.get_opacity(),
                                    scales, rotations, cov3D);
    RenderOutput o{outs[0], screenspace, outs[1] > 0, outs[1], outs[2]};
    o.num_rendered = outs[3][0].item<int32_t>();  // host tensor: no device wait
    o.capacity = outs[3][1].item<int32_t>();
    if (binning) binning->observe(o);
    return o;
}

// The reference keeps the background as a device tensor (train_utils.cpp:115-117): this
// overload reads it back on every call (one host wait); a loop should convert it once with
// gsr::background() and call the overload above.
template <class Model, class Pipe>
RenderOutput render(const RasterCamera& cam, Model& pc, const Pipe& pipe, const torch::Tensor& bg,
                    float scaling_modifier = 1.f, std::optional<torch::Tensor> override_color = std::nullopt,
                    BinningCapacity* binning = nullptr) {
    return render(cam, pc, pipe, background(bg), scaling_modifier, std::move(override_color), binning);
}

namespace detail {
// The forward / backward of RasterizeGaussians without autograd (the native trainer's path,
// gsr_trainer.h): torch owns every scratch byte; `Frame` keeps them from forward to backward.
struct Frame {
    torch::Tensor color, radii, geom, binning, image;
    gsr_buffers bufs{};
    gsr_camera cam{};
    gsr_raster_settings settings{};
    torch::Tensor k_device() const;  // (1,) int32 device copy of the scan's K
};
Frame forward(const RasterCamera& cam, const RasterSettings& rs, const torch::Tensor& means3D,
              const torch::Tensor& sh_dc, const torch::Tensor& sh_rest, const torch::Tensor& colors,
              const torch::Tensor& opac, const torch::Tensor& scales, const torch::Tensor& rots,
              const torch::Tensor& cov3D);
// gsr_backward into the given gradient tensors (undefined = not requested where nullable)
void backward(const Frame& f, const RasterSettings& rs, const torch::Tensor& means3D, const torch::Tensor& sh_dc,
              const torch::Tensor& sh_rest, const torch::Tensor& colors, const torch::Tensor& opac,
              const torch::Tensor& scales, const torch::Tensor& rots, const torch::Tensor& cov3D,
              const torch::Tensor& dL_dcolor, const gsr_grads& grads);
void check(int rc, const char* what);
void* current_stream();
}  // namespace detail

}  // namespace gsr

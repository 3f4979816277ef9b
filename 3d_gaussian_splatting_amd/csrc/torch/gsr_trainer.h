// gsr_trainer.h -- the training step around the rasterizer, in C++ on libtorch (SURVEY §8f rows
// 1-2): what the reference's loop body at src/utils/train_utils.cpp:128-145 is missing after
// render().  Two layers, both over the C ABI of include/gsr/gsr_train.h:
//
// 1. Drop-in pieces for the reference's own autograd loop (GaussianModel leaves, six
//    torch::optim::Adam instances, gaussian_model.cpp:316-345):
//      auto out  = gsr::render(cam, *gaussians, pipe, bg, 1.f, std::nullopt, &binning);
//      auto loss = gsr::photometric_loss(out.render, gt, opt.lambda_dssim_);
//      loss.backward();
//      gsr::densify_stats(out.radii, out.viewspace_points.grad(), core.max_radii2D_,
//                         core.xyz_gradient_accum_, core.denom_);
//      gsr::fused_adam_step(core.optimizers_);   // = opt->step() for the six, one launch
//
// 2. gsr::Trainer: the same iteration without autograd (activations and their backward fused
//    into the kernels, no per-op launches), densification and opacity reset included -- the
//    native twin of 3d_gaussian_splatting_amd/trainer.py (GaussianTrainer), op for op, so a loop
//    over it reproduces the Python loop bit for bit (tests/test_gpu_train_loop.py).
//
// OptimizationParams is the reference's struct (src/arguments/params.h:50-91: same fields,
// float types and defaults).
#pragma once
#include <torch/torch.h>

#include <array>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "gsr/gsr_train.h"
#include "gsr_render.h"

namespace gsr {

struct OptimizationParams {  // src/arguments/params.h:50-91
    int iterations_{30'000};
    float position_lr_init_{0.00016};
    float position_lr_final_{0.0000016};
    float position_lr_delay_mult_{0.01};
    int position_lr_max_steps_{30'000};
    float feature_lr_{0.0025};
    float opacity_lr_{0.05};
    float scaling_lr_{0.005};
    float rotation_lr_{0.001};
    float percent_dense_{0.01};
    float lambda_dssim_{0.2};
    int densification_interval_{100};
    int opacity_reset_interval_{3000};
    int densify_from_iter_{500};
    int densify_until_iter_{15'000};
    float densify_grad_threshold_{0.0002};
    bool random_background_{false};
};

// Exponential learning-rate schedule (src/utils/general_utils.cpp:112-142), called with the
// arguments its parameter names say (the reference's setup misbinds them,
// gaussian_model.cpp:347-351).
std::function<double(int)> get_expon_lr_func(double lr_init, double lr_final, int lr_delay_steps = 0,
                                             double lr_delay_mult = 1.0, int max_steps = 1000000);

// ---- drop-in pieces ---------------------------------------------------------------------
// (1 - lambda_dssim) L1 + lambda_dssim (1 - SSIM) of image vs gt (C,H,W), as an autograd
// Function over gsr_loss_forward / gsr_loss_backward (11x11 Gaussian window, sigma 1.5: the
// upstream definition -- the reference has no loss).  Returns the scalar loss on the device;
// `stats`, when given, receives [loss, l1, ssim] (device, 3).  No host wait.
torch::Tensor photometric_loss(const torch::Tensor& image, const torch::Tensor& gt, double lambda_dssim,
                               torch::Tensor* stats = nullptr);

// One step of every given torch::optim::Adam, fused into ONE gsr_adam_step launch over all
// their parameters, on libtorch's own state (AdamParamState exp_avg / exp_avg_sq / step, created
// as libtorch creates it): the same update as calling opt->step() on each.  Parameters without
// a gradient are skipped as libtorch skips them.  Options the kernel does not implement
// (amsgrad, weight_decay != 0) are refused with an exception.
// `guard`: the render whose gradients these are.  When it ran under a binning bound
// (RenderOutput::num_rendered < 0), the step is skipped ON THE DEVICE if its K exceeded that
// bound (gsr_adam_step_guarded): a truncated render never updates the model, with no host wait.
void fused_adam_step(const std::vector<torch::optim::Adam*>& optimizers, const RenderOutput* guard = nullptr);
template <class Map>
void fused_adam_step(Map& optimizers, const RenderOutput* guard = nullptr) {  // e.g. CoreParams::optimizers_
    std::vector<torch::optim::Adam*> v;
    for (auto& kv : optimizers) v.push_back(kv.second.get());
    fused_adam_step(static_cast<const std::vector<torch::optim::Adam*>&>(v), guard);
}

// Densification statistics of one render (gaussian_model.h:18-20, upstream
// add_densification_stats): for radii > 0, max_radii2D = max(max_radii2D, radii),
// grad_accum += |viewspace_grad[:, :2]|, denom += 1.  All (P) f32 device tensors.  `guard`: as
// fused_adam_step's (skipped on the device for a render truncated by its bound).
void densify_stats(const torch::Tensor& radii, const torch::Tensor& viewspace_grad, torch::Tensor& max_radii2D,
                   torch::Tensor& grad_accum, torch::Tensor& denom, const RenderOutput* guard = nullptr);
// Ascending int32 indices of the nonzero entries of a bool / uint8 mask (one host read of the count).
torch::Tensor compact_index(const torch::Tensor& mask);
// [t[idx] for t in tensors] (rows of contiguous f32 tensors) in one launch per 24 tensors.
std::vector<torch::Tensor> gather_rows(const std::vector<torch::Tensor>& tensors, const torch::Tensor& idx);
// Mean squared distance of each point (N,3) to its 3 nearest others (exact; create_from_pcd's scales).
torch::Tensor knn_mean_dist2(const torch::Tensor& points);
// Rotation matrices of (unnormalised) quaternions (N,4), w first (general_utils.cpp:12-40).
torch::Tensor build_rotation(const torch::Tensor& r);

// ---- native trainer -------------------------------------------------------------------------
class Trainer {
   public:
    static constexpr int kGroups = 6;
    static const std::array<const char*, kGroups> kGroupNames;  // xyz f_dc f_rest opacity scaling rotation

    Trainer(torch::Tensor xyz, torch::Tensor f_dc, torch::Tensor f_rest, torch::Tensor opacity,
            torch::Tensor scaling, torch::Tensor rotation, int max_sh_degree, const OptimizationParams& opt,
            double spatial_lr_scale, double cameras_extent, uint64_t seed);
    // upstream create_from_pcd: means = points, f_dc = RGB2SH(colours), f_rest = 0, scales from
    // the 3-NN mean squared distance, rotation (1,0,0,0), opacity inverse_sigmoid(0.1);
    // spatial_lr_scale = cameras_extent = the training cameras' extent.
    static std::unique_ptr<Trainer> from_point_cloud(const torch::Tensor& points, const torch::Tensor& colors,
                                                     int max_sh_degree, double extent,
                                                     const OptimizationParams& opt, uint64_t seed);

    struct StepResult {
        torch::Tensor stats;  // [loss, l1, ssim] (device)
        torch::Tensor radii;  // (P) int32 (device)
        torch::Tensor image;  // (3,H,W) (device)
        int num_points;
    };
    // One iteration in the upstream order (train_utils.cpp:128-145 plus the body its stub
    // omits): LR update, SH degree, render, loss, backward, densification statistics, densify /
    // prune and opacity reset, optimizer step (a group replaced by densification or the reset
    // takes no update that iteration).  No host wait unless a densification is due.
    StepResult step(int iteration, const RasterCamera& cam, const torch::Tensor& gt,
                    const std::array<float, 3>& bg = {0.f, 0.f, 0.f}, bool densify = true);

    double update_learning_rate(int iteration);
    void oneup_SH_degree();
    void densify_and_prune(double max_grad, double min_opacity, double extent, std::optional<double> max_screen_size,
                           const std::optional<torch::Tensor>& split_samples = std::nullopt);
    void prune_points(const torch::Tensor& mask);
    void reset_opacity();

    int num_points() const { return (int)params_.at("xyz").size(0); }
    int active_sh_degree() const { return active_sh_degree_; }
    const std::map<std::string, torch::Tensor>& params() const { return params_; }
    BinningCapacity& binning() { return binning_; }

   private:
    detail::Frame render(const RasterCamera& cam, const std::array<float, 3>& bg, torch::Tensor& s,
                         torch::Tensor& q, torch::Tensor& o);
    void setup();
    void optimizer_step(const std::map<std::string, torch::Tensor>& grads);
    const uint32_t* guard_ptr() const {
        return guard_k_.defined() ? reinterpret_cast<const uint32_t*>(guard_k_.data_ptr<int32_t>()) : nullptr;
    }
    void append(const std::map<std::string, torch::Tensor>& rows);
    std::map<std::string, torch::Tensor> rows(const torch::Tensor& mask);
    void densify_and_clone(const torch::Tensor& grads, double threshold, double extent);
    void densify_and_split(const torch::Tensor& grads, double threshold, double extent, int N,
                           const std::optional<torch::Tensor>& samples);

    OptimizationParams opt_;
    int max_sh_degree_, active_sh_degree_ = 0;
    double spatial_lr_scale_, cameras_extent_, percent_dense_;
    torch::Device device_;
    std::map<std::string, torch::Tensor> params_, exp_avg_, exp_avg_sq_;
    std::map<std::string, int> steps_;
    std::map<std::string, double> lr_;
    std::function<double(int)> xyz_scheduler_;
    torch::Tensor max_radii2D_, xyz_gradient_accum_, denom_;
    at::Generator gen_;
    BinningCapacity binning_;
    // the last render's K (device counter) and the bound it ran under (0: exact, no guard):
    // the device-side guard of that iteration's statistics and Adam step
    torch::Tensor guard_k_;
    int guard_cap_ = 0;
};

}  // namespace gsr

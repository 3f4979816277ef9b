// gsr_trainer.cpp -- see gsr_trainer.h.  Host C++ on libtorch; every device byte of the loss,
// optimizer, statistics and compaction goes through include/gsr/gsr_train.h into libgsr_hip.so,
// the rasterizer through include/gsr/gsr.h (gsr_render.h's detail::forward / backward).
//
// gsr::Trainer mirrors 3d_gaussian_splatting_amd/trainer.py (GaussianTrainer) op for op: the
// same kernels and the same torch ops in the same order, so the two produce the same bits.
#include "gsr_trainer.h"

#include <ATen/hip/HIPGeneratorImpl.h>
#include <c10/hip/HIPStream.h>

#include <cmath>
#include <stdexcept>

namespace gsr {
namespace {

using detail::check;

void* stream() { return detail::current_stream(); }

float* fp(const torch::Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }

void require_f32(const torch::Tensor& t, const char* what) {
    TORCH_CHECK(t.defined() && t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous(), what,
                " must be a contiguous float32 GPU tensor");
}

// ---- photometric loss autograd Function ----
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

class PhotometricLoss : public torch::autograd::Function<PhotometricLoss> {
   public:
    static variable_list forward(AutogradContext* ctx, torch::Tensor image, torch::Tensor gt, double lambda) {
        TORCH_CHECK(image.dim() == 3 && image.sizes() == gt.sizes(), "loss: image / gt must be matching (C,H,W)");
        auto img = image.contiguous(), g = gt.contiguous();
        require_f32(img, "image");
        require_f32(g, "gt");
        const int C = (int)img.size(0), H = (int)img.size(1), W = (int)img.size(2);
        auto maps = torch::empty({(int64_t)gsr_loss_scratch_bytes(C, H, W)},
                                 img.options().dtype(torch::kUInt8));
        auto stats = torch::empty({3}, img.options());
        check(gsr_loss_forward(img.data_ptr<float>(), g.data_ptr<float>(), C, H, W, (float)lambda, maps.data_ptr(),
                               stats.data_ptr<float>(), stream()),
              "gsr_loss_forward");
        ctx->save_for_backward({img, g, maps});
        ctx->saved_data["lambda"] = lambda;
        ctx->mark_non_differentiable({stats});
        return {stats.select(0, 0).clone(), stats};
    }

    static variable_list backward(AutogradContext* ctx, variable_list grad_out) {
        auto sv = ctx->get_saved_variables();
        auto img = sv[0], g = sv[1], maps = sv[2];
        const int C = (int)img.size(0), H = (int)img.size(1), W = (int)img.size(2);
        auto dimg = torch::empty_like(img);
        check(gsr_loss_backward(img.data_ptr<float>(), g.data_ptr<float>(), C, H, W,
                                (float)ctx->saved_data["lambda"].toDouble(), maps.data_ptr(), dimg.data_ptr<float>(),
                                stream()),
              "gsr_loss_backward");
        if (grad_out[0].defined()) dimg.mul_(grad_out[0]);  // dL/dloss (a device scalar, no host read)
        return {dimg, torch::Tensor(), torch::Tensor()};
    }
};

}  // namespace

std::function<double(int)> get_expon_lr_func(double lr_init, double lr_final, int lr_delay_steps,
                                             double lr_delay_mult, int max_steps) {
    return [=](int step) -> double {
        if (step < 0 || (lr_init == 0.0 && lr_final == 0.0)) return 0.0;
        double delay_rate = 1.0;
        if (lr_delay_steps > 0)
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) *
                                             std::sin(0.5 * M_PI * std::min(std::max((double)step / lr_delay_steps, 0.0), 1.0));
        const double t = std::min(std::max((double)step / max_steps, 0.0), 1.0);
        return delay_rate * std::exp(std::log(lr_init) * (1 - t) + std::log(lr_final) * t);
    };
}

torch::Tensor photometric_loss(const torch::Tensor& image, const torch::Tensor& gt, double lambda_dssim,
                               torch::Tensor* stats) {
    auto outs = PhotometricLoss::apply(image, gt, lambda_dssim);
    if (stats) *stats = outs[1];
    return outs[0];
}

namespace {
// (K device pointer, bound) of a bounded render, or (nullptr, 0)
std::pair<const uint32_t*, uint32_t> guard_of(const RenderOutput* r) {
    if (!r || r->num_rendered >= 0 || !r->num_rendered_device.defined()) return {nullptr, 0u};
    return {reinterpret_cast<const uint32_t*>(r->num_rendered_device.data_ptr<int32_t>()), (uint32_t)r->capacity};
}
}  // namespace

void fused_adam_step(const std::vector<torch::optim::Adam*>& optimizers, const RenderOutput* guard) {
    std::vector<gsr_adam_group> groups;
    std::vector<torch::Tensor> keep;
    double beta1 = -1, beta2 = -1, eps = -1;
    const auto gk = guard_of(guard);
    auto launch = [&]() {
        if (groups.empty()) return;
        check(gsr_adam_step_guarded(groups.data(), (int32_t)groups.size(), (float)beta1, (float)beta2, (float)eps,
                                    gk.first, gk.second, stream()),
              "gsr_adam_step");
        groups.clear();
        keep.clear();
    };
    for (torch::optim::Adam* opt : optimizers) {
        for (auto& group : opt->param_groups()) {
            auto& o = static_cast<torch::optim::AdamOptions&>(group.options());
            TORCH_CHECK(!o.amsgrad() && o.weight_decay() == 0.0,
                        "fused_adam_step: amsgrad / weight_decay are not fused (use opt->step())");
            const double b1 = std::get<0>(o.betas()), b2 = std::get<1>(o.betas());
            if (!groups.empty() && (b1 != beta1 || b2 != beta2 || o.eps() != eps)) launch();
            beta1 = b1, beta2 = b2, eps = o.eps();
            for (auto& p : group.params()) {
                if (!p.grad().defined()) continue;
                auto& states = opt->state();
                auto it = states.find(p.unsafeGetTensorImpl());
                if (it == states.end()) {  // created as libtorch's Adam::step creates it
                    auto st = std::make_unique<torch::optim::AdamParamState>();
                    st->step(0);
                    st->exp_avg(torch::zeros_like(p, torch::MemoryFormat::Preserve));
                    st->exp_avg_sq(torch::zeros_like(p, torch::MemoryFormat::Preserve));
                    it = states.emplace(p.unsafeGetTensorImpl(), std::move(st)).first;
                }
                auto& st = static_cast<torch::optim::AdamParamState&>(*it->second);
                TORCH_CHECK(p.is_contiguous() && st.exp_avg().is_contiguous() && st.exp_avg_sq().is_contiguous(),
                            "fused_adam_step: contiguous parameters and state only");
                st.step(st.step() + 1);
                auto g = p.grad().contiguous();
                keep.push_back(g);
                gsr_adam_group ag{};
                ag.param = p.data_ptr<float>();
                ag.grad = g.data_ptr<float>();
                ag.exp_avg = st.exp_avg().data_ptr<float>();
                ag.exp_avg_sq = st.exp_avg_sq().data_ptr<float>();
                ag.n = p.numel();
                ag.act = GSR_ACT_NONE;  // autograd already took the getters' activations
                ag.step = (int32_t)st.step();
                ag.lr = (float)o.lr();
                groups.push_back(ag);
                if ((int)groups.size() == GSR_ADAM_MAX_GROUPS) launch();
            }
        }
    }
    launch();
}

void densify_stats(const torch::Tensor& radii, const torch::Tensor& viewspace_grad, torch::Tensor& max_radii2D,
                   torch::Tensor& grad_accum, torch::Tensor& denom, const RenderOutput* guard) {
    const int64_t P = radii.size(0);
    TORCH_CHECK(radii.scalar_type() == torch::kInt32 && radii.is_contiguous(), "radii must be contiguous int32");
    auto g = viewspace_grad.contiguous();
    require_f32(g, "viewspace grad");
    TORCH_CHECK(g.numel() == 3 * P, "viewspace grad must be (P,3)");
    for (auto* t : {&max_radii2D, &grad_accum, &denom}) {
        require_f32(*t, "statistics");
        TORCH_CHECK(t->numel() == P, "statistics must have P entries");
    }
    const auto gk = guard_of(guard);
    check(gsr_densify_stats_guarded(radii.data_ptr<int32_t>(), g.data_ptr<float>(), (int32_t)P,
                                    max_radii2D.data_ptr<float>(), grad_accum.data_ptr<float>(),
                                    denom.data_ptr<float>(), gk.first, gk.second, stream()),
          "gsr_densify_stats");
}

torch::Tensor compact_index(const torch::Tensor& mask) {
    auto m = mask.to(torch::kUInt8).contiguous();
    const int32_t n = (int32_t)m.numel();
    auto opt = m.options();
    auto idx = torch::empty({std::max<int64_t>(n, 1)}, opt.dtype(torch::kInt32));
    auto cnt = torch::empty({1}, opt.dtype(torch::kInt32));
    auto scratch = torch::empty({(int64_t)gsr_compact_scratch_bytes(n)}, opt.dtype(torch::kUInt8));
    check(gsr_compact_index(m.data_ptr<uint8_t>(), n, idx.data_ptr<int32_t>(), cnt.data_ptr<int32_t>(),
                            scratch.data_ptr(), stream()),
          "gsr_compact_index");
    return idx.narrow(0, 0, cnt.item<int32_t>());
}

std::vector<torch::Tensor> gather_rows(const std::vector<torch::Tensor>& tensors, const torch::Tensor& idx) {
    const int64_t n_out = idx.numel();
    std::vector<torch::Tensor> outs;
    std::vector<int> live;
    for (size_t i = 0; i < tensors.size(); ++i) {
        auto shape = tensors[i].sizes().vec();
        shape[0] = n_out;
        outs.push_back(torch::empty(shape, tensors[i].options()));
        if (tensors[i].numel() > 0 && tensors[i].numel() / std::max<int64_t>(tensors[i].size(0), 1) > 0)
            live.push_back((int)i);
    }
    if (n_out == 0 || tensors.empty()) return outs;
    auto idx32 = idx.to(torch::kInt32).contiguous();
    for (size_t i0 = 0; i0 < live.size(); i0 += GSR_GATHER_MAX) {
        std::vector<gsr_row_copy> copies;
        for (size_t j = i0; j < std::min(live.size(), i0 + (size_t)GSR_GATHER_MAX); ++j) {
            const auto& t = tensors[live[j]];
            require_f32(t, "gather_rows input");
            gsr_row_copy c{};
            c.src = t.data_ptr<float>();
            c.dst = outs[live[j]].data_ptr<float>();
            c.width = (int32_t)(t.numel() / t.size(0));
            copies.push_back(c);
        }
        check(gsr_gather_rows(copies.data(), (int32_t)copies.size(), idx32.data_ptr<int32_t>(), (int32_t)n_out,
                              stream()),
              "gsr_gather_rows");
    }
    return outs;
}

torch::Tensor knn_mean_dist2(const torch::Tensor& points) {
    require_f32(points, "points");
    const int32_t n = (int32_t)points.size(0);
    auto out = torch::empty({n}, points.options());
    if (n == 0) return out;
    auto scratch = torch::empty({(int64_t)gsr_knn_scratch_bytes(n)}, points.options().dtype(torch::kUInt8));
    check(gsr_knn_mean_dist2(points.data_ptr<float>(), n, out.data_ptr<float>(), scratch.data_ptr(), stream()),
          "gsr_knn_mean_dist2");
    return out;
}

torch::Tensor build_rotation(const torch::Tensor& r) {  // general.py build_rotation, op for op
    auto c = [&](int k) { return r.select(1, k); };
    auto norm = torch::sqrt(c(0) * c(0) + c(1) * c(1) + c(2) * c(2) + c(3) * c(3));
    auto q = r / norm.unsqueeze(1);
    auto rr = q.select(1, 0), x = q.select(1, 1), y = q.select(1, 2), z = q.select(1, 3);
    auto R = torch::stack({1 - 2 * (y * y + z * z), 2 * (x * y - rr * z), 2 * (x * z + rr * y),
                           2 * (x * y + rr * z), 1 - 2 * (x * x + z * z), 2 * (y * z - rr * x),
                           2 * (x * z - rr * y), 2 * (y * z + rr * x), 1 - 2 * (x * x + y * y)},
                          1);
    return R.reshape({-1, 3, 3});
}

// ---------------------------------------------------------------------------------------------
const std::array<const char*, Trainer::kGroups> Trainer::kGroupNames = {"xyz",     "f_dc",    "f_rest",
                                                                        "opacity", "scaling", "rotation"};

namespace {
int act_of(const std::string& k) {
    if (k == "opacity") return GSR_ACT_SIGMOID;
    if (k == "scaling") return GSR_ACT_EXP;
    if (k == "rotation") return GSR_ACT_NORMALIZE4;
    return GSR_ACT_NONE;
}
}  // namespace

Trainer::Trainer(torch::Tensor xyz, torch::Tensor f_dc, torch::Tensor f_rest, torch::Tensor opacity,
                 torch::Tensor scaling, torch::Tensor rotation, int max_sh_degree, const OptimizationParams& opt,
                 double spatial_lr_scale, double cameras_extent, uint64_t seed)
    : opt_(opt),
      max_sh_degree_(max_sh_degree),
      spatial_lr_scale_((float)spatial_lr_scale),  // CoreParams::spatial_lr_scale_ is a float
      cameras_extent_(cameras_extent),
      percent_dense_(opt.percent_dense_),
      device_(xyz.device()),
      gen_(at::cuda::detail::createCUDAGenerator(xyz.device().index())) {
    TORCH_CHECK(xyz.is_cuda(), "Trainer: GPU tensors only (no CPU fallback)");
    const int64_t P = xyz.size(0);
    auto f = [&](const torch::Tensor& t, std::vector<int64_t> shape) {
        return t.to(device_, torch::kFloat32).reshape(shape).contiguous();
    };
    params_["xyz"] = f(xyz, {P, 3});
    params_["f_dc"] = f(f_dc, {P, 1, 3});
    params_["f_rest"] = f(f_rest, {P, -1, 3});
    params_["opacity"] = f(opacity, {P, 1});
    params_["scaling"] = f(scaling, {P, 3});
    params_["rotation"] = f(rotation, {P, 4});
    {
        std::lock_guard<std::mutex> lock(gen_.mutex());
        gen_.set_current_seed(seed);
    }
    setup();
}

std::unique_ptr<Trainer> Trainer::from_point_cloud(const torch::Tensor& points, const torch::Tensor& colors,
                                                   int max_sh_degree, double extent, const OptimizationParams& opt,
                                                   uint64_t seed) {
    auto pts = points.to(torch::kFloat32).reshape({-1, 3}).contiguous();
    const int64_t n = pts.size(0);
    auto d2 = knn_mean_dist2(pts);
    auto scales = torch::log(torch::sqrt(torch::clamp_min(d2, 1e-7))).unsqueeze(1).repeat({1, 3});
    auto fo = pts.options();
    auto rots = torch::zeros({n, 4}, fo);
    rots.select(1, 0).fill_(1.0);
    auto o = torch::full({n, 1}, 0.1, fo);
    auto opac = torch::log(o / (1 - o));
    auto rgb = colors.to(pts.device(), torch::kFloat32).reshape({-1, 3});
    auto f_dc = ((rgb - 0.5) / 0.28209479177387814).unsqueeze(1);  // RGB2SH
    auto f_rest = torch::zeros({n, (max_sh_degree + 1) * (max_sh_degree + 1) - 1, 3}, fo);
    return std::make_unique<Trainer>(pts, f_dc, f_rest, opac, scales, rots, max_sh_degree, opt, extent, extent, seed);
}

void Trainer::setup() {  // GaussianModel::setup (gaussian_model.cpp:316-352)
    const int64_t P = num_points();
    auto z = [&]() { return torch::zeros({P}, params_["xyz"].options()); };
    xyz_gradient_accum_ = z();
    denom_ = z();
    max_radii2D_ = z();
    for (auto& kv : params_) {
        exp_avg_[kv.first] = torch::zeros_like(kv.second);
        exp_avg_sq_[kv.first] = torch::zeros_like(kv.second);
    }
    for (const char* k : kGroupNames) steps_[k] = 0;
    lr_["xyz"] = (double)opt_.position_lr_init_ * spatial_lr_scale_;
    lr_["f_dc"] = opt_.feature_lr_;
    lr_["f_rest"] = (double)opt_.feature_lr_ / 20.0;
    lr_["opacity"] = opt_.opacity_lr_;
    lr_["scaling"] = opt_.scaling_lr_;
    lr_["rotation"] = opt_.rotation_lr_;
    xyz_scheduler_ = get_expon_lr_func((double)opt_.position_lr_init_ * spatial_lr_scale_,
                                       (double)opt_.position_lr_final_ * spatial_lr_scale_, 0,
                                       opt_.position_lr_delay_mult_, opt_.position_lr_max_steps_);
}

double Trainer::update_learning_rate(int iteration) {
    const double lr = xyz_scheduler_(iteration);
    lr_["xyz"] = lr;
    return lr;
}

void Trainer::oneup_SH_degree() {
    if (active_sh_degree_ < max_sh_degree_) ++active_sh_degree_;
}

detail::Frame Trainer::render(const RasterCamera& cam, const std::array<float, 3>& bg, torch::Tensor& s,
                              torch::Tensor& q, torch::Tensor& o) {
    const int64_t P = num_points();
    s = torch::empty_like(params_["scaling"]);
    q = torch::empty_like(params_["rotation"]);
    o = torch::empty_like(params_["opacity"]);
    check(gsr_activate(fp(params_["scaling"]), fp(params_["rotation"]), fp(params_["opacity"]), (int32_t)P, fp(s),
                       fp(q), fp(o), stream()),
          "gsr_activate");
    RasterSettings rs;
    rs.bg = bg;
    rs.sh_degree = active_sh_degree_;
    const int bound = binning_.bound();
    rs.max_rendered = bound;
    o = o.reshape({-1});
    const auto& rest = params_["f_rest"];
    auto f = detail::forward(cam, rs, params_["xyz"], params_["f_dc"], rest.size(1) ? rest : torch::Tensor(),
                             torch::Tensor(), o, s, q, torch::Tensor());
    guard_k_ = bound > 0 ? f.k_device() : torch::Tensor();
    guard_cap_ = bound;
    binning_.observe(f.k_device(), f.bufs.num_rendered);
    return f;
}

Trainer::StepResult Trainer::step(int iteration, const RasterCamera& cam, const torch::Tensor& gt,
                                  const std::array<float, 3>& bg, bool densify) {
    update_learning_rate(iteration);
    if (iteration % 1000 == 0) oneup_SH_degree();
    torch::Tensor s, q, o;
    detail::Frame fr = render(cam, bg, s, q, o);
    const int64_t P = num_points();
    // loss forward / backward (gsr_train.h)
    const int C = 3, H = cam.height, W = cam.width;
    TORCH_CHECK(gt.is_contiguous() && gt.numel() == (int64_t)C * H * W, "gt must be a contiguous (3,H,W) tensor");
    auto maps = torch::empty({(int64_t)gsr_loss_scratch_bytes(C, H, W)}, fr.color.options().dtype(torch::kUInt8));
    auto stats = torch::empty({3}, fr.color.options());
    check(gsr_loss_forward(fp(fr.color), fp(gt), C, H, W, opt_.lambda_dssim_, maps.data_ptr(), fp(stats), stream()),
          "gsr_loss_forward");
    auto dimg = torch::empty_like(fr.color);
    check(gsr_loss_backward(fp(fr.color), fp(gt), C, H, W, opt_.lambda_dssim_, maps.data_ptr(), fp(dimg), stream()),
          "gsr_loss_backward");
    // rasterizer backward (the gradients w.r.t. the ACTIVATED values; Adam applies the
    // activations' backward in-kernel)
    auto fo = params_["xyz"].options();
    auto g_means2D = torch::empty({P, 3}, fo), g_conic = torch::empty({P, 3}, fo), g_opac = torch::empty({P, 1}, fo),
         g_means3D = torch::empty({P, 3}, fo), g_dc = torch::empty({P, 1, 3}, fo), g_scales = torch::empty({P, 3}, fo),
         g_rots = torch::empty({P, 4}, fo);
    const auto& rest = params_["f_rest"];
    torch::Tensor g_rest = rest.size(1) ? torch::empty_like(rest) : torch::Tensor();
    gsr_grads gg{};
    gg.dL_dmeans2D = fp(g_means2D);
    gg.dL_dconic = fp(g_conic);
    gg.dL_dopacity = fp(g_opac);
    gg.dL_dmeans3D = fp(g_means3D);
    gg.dL_dsh_dc = fp(g_dc);
    gg.dL_dsh_rest = fp(g_rest);
    gg.dL_dscales = fp(g_scales);
    gg.dL_drotations = fp(g_rots);
    RasterSettings rs;
    rs.bg = bg;
    rs.sh_degree = active_sh_degree_;
    detail::backward(fr, rs, params_["xyz"], params_["f_dc"], rest.size(1) ? rest : torch::Tensor(), torch::Tensor(),
                     o, s, q, torch::Tensor(), dimg, gg);
    std::map<std::string, torch::Tensor> grads{
        {"xyz", g_means3D}, {"f_dc", g_dc}, {"opacity", g_opac}, {"scaling", g_scales}, {"rotation", g_rots}};
    if (rest.size(1)) grads["f_rest"] = g_rest;
    std::vector<std::string> replaced;
    if (iteration < opt_.densify_until_iter_) {
        check(gsr_densify_stats_guarded(fr.radii.data_ptr<int32_t>(), fp(g_means2D), (int32_t)P, fp(max_radii2D_),
                                        fp(xyz_gradient_accum_), fp(denom_), guard_ptr(), (uint32_t)guard_cap_,
                                        stream()),
              "gsr_densify_stats");
        if (densify) {
            if (iteration > opt_.densify_from_iter_ && iteration % opt_.densification_interval_ == 0) {
                std::optional<double> size_threshold;
                if (iteration > opt_.opacity_reset_interval_) size_threshold = 20.0;
                densify_and_prune(opt_.densify_grad_threshold_, 0.005, cameras_extent_, size_threshold);
                binning_.reset();
                for (const char* k : kGroupNames) replaced.push_back(k);
            }
            if (iteration % opt_.opacity_reset_interval_ == 0) {
                reset_opacity();
                binning_.reset();
                replaced.push_back("opacity");
            }
        }
    }
    if (iteration < opt_.iterations_) {
        for (const auto& k : replaced) grads.erase(k);
        optimizer_step(grads);
    }
    return {stats, fr.radii, fr.color, num_points()};
}

void Trainer::optimizer_step(const std::map<std::string, torch::Tensor>& grads) {
    std::vector<gsr_adam_group> groups;
    std::vector<torch::Tensor> keep;
    for (const char* name : kGroupNames) {
        auto it = grads.find(name);
        if (it == grads.end()) continue;
        const std::string k = name;
        steps_[k] += 1;
        auto g = it->second.reshape(params_[k].sizes()).contiguous();
        keep.push_back(g);
        gsr_adam_group ag{};
        ag.param = fp(params_[k]);
        ag.grad = fp(g);
        ag.exp_avg = fp(exp_avg_[k]);
        ag.exp_avg_sq = fp(exp_avg_sq_[k]);
        ag.n = params_[k].numel();
        ag.act = act_of(k);
        ag.step = steps_[k];
        ag.lr = (float)lr_[k];
        groups.push_back(ag);
    }
    if (!groups.empty())
        check(gsr_adam_step_guarded(groups.data(), (int32_t)groups.size(), 0.9f, 0.999f, 1e-8f, guard_ptr(),
                                    (uint32_t)guard_cap_, stream()),
              "gsr_adam_step");
}

// ---- densification (upstream semantics; trainer.py) ----
void Trainer::append(const std::map<std::string, torch::Tensor>& rows) {
    for (const char* name : kGroupNames) {
        const std::string k = name;
        params_[k] = torch::cat({params_[k], rows.at(k).contiguous()}, 0).contiguous();
        auto zeros = torch::zeros_like(rows.at(k));
        exp_avg_[k] = torch::cat({exp_avg_[k], zeros}, 0).contiguous();
        exp_avg_sq_[k] = torch::cat({exp_avg_sq_[k], zeros}, 0).contiguous();
    }
    const int64_t P = num_points();
    auto z = [&]() { return torch::zeros({P}, params_["xyz"].options()); };
    xyz_gradient_accum_ = z();
    denom_ = z();
    max_radii2D_ = z();
}

void Trainer::prune_points(const torch::Tensor& mask) {
    auto idx = compact_index(mask.logical_not());
    std::vector<torch::Tensor> src;
    for (auto* m : {&params_, &exp_avg_, &exp_avg_sq_})
        for (const char* k : kGroupNames) src.push_back((*m)[k]);
    src.push_back(xyz_gradient_accum_);
    src.push_back(denom_);
    src.push_back(max_radii2D_);
    auto out = gather_rows(src, idx);
    size_t i = 0;
    for (auto* m : {&params_, &exp_avg_, &exp_avg_sq_})
        for (const char* k : kGroupNames) (*m)[k] = out[i++];
    xyz_gradient_accum_ = out[i++];
    denom_ = out[i++];
    max_radii2D_ = out[i++];
}

std::map<std::string, torch::Tensor> Trainer::rows(const torch::Tensor& mask) {
    auto idx = compact_index(mask);
    std::vector<torch::Tensor> src;
    for (const char* k : kGroupNames) src.push_back(params_[k]);
    auto out = gather_rows(src, idx);
    std::map<std::string, torch::Tensor> r;
    for (int i = 0; i < kGroups; ++i) r[kGroupNames[i]] = out[i];
    return r;
}

void Trainer::densify_and_clone(const torch::Tensor& grads, double threshold, double extent) {
    auto scaling = torch::exp(params_["scaling"]);
    auto mask = (grads >= threshold) & (std::get<0>(scaling.max(1)) <= percent_dense_ * extent);
    append(rows(mask));
}

void Trainer::densify_and_split(const torch::Tensor& grads, double threshold, double extent, int N,
                                const std::optional<torch::Tensor>& samples_in) {
    const int64_t n_init = num_points();
    auto padded = torch::zeros({n_init}, params_["xyz"].options());
    padded.narrow(0, 0, grads.size(0)).copy_(grads);
    auto scaling = torch::exp(params_["scaling"]);
    auto mask = (padded >= threshold) & (std::get<0>(scaling.max(1)) > percent_dense_ * extent);
    auto sel = rows(mask);
    auto stds = torch::exp(sel["scaling"]).repeat({N, 1});
    torch::Tensor samples = samples_in ? *samples_in : at::normal(torch::zeros_like(stds), stds, gen_);
    auto rots = build_rotation(sel["rotation"]).repeat({N, 1, 1});
    std::map<std::string, torch::Tensor> nw;
    nw["xyz"] = torch::bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + sel["xyz"].repeat({N, 1});
    nw["scaling"] = torch::log(torch::exp(sel["scaling"]).repeat({N, 1}) / (0.8 * N));
    nw["rotation"] = sel["rotation"].repeat({N, 1});
    nw["f_dc"] = sel["f_dc"].repeat({N, 1, 1});
    nw["f_rest"] = sel["f_rest"].repeat({N, 1, 1});
    nw["opacity"] = sel["opacity"].repeat({N, 1});
    append(nw);
    auto prune = torch::cat(
        {mask, torch::zeros({N * sel["xyz"].size(0)}, mask.options().dtype(torch::kBool))});
    prune_points(prune);
}

void Trainer::densify_and_prune(double max_grad, double min_opacity, double extent,
                                std::optional<double> max_screen_size,
                                const std::optional<torch::Tensor>& split_samples) {
    auto grads = xyz_gradient_accum_ / denom_;
    grads.index_put_({grads.isnan()}, 0.0);
    densify_and_clone(grads, max_grad, extent);
    densify_and_split(grads, max_grad, extent, 2, split_samples);
    auto prune = (torch::sigmoid(params_["opacity"]) < min_opacity).squeeze(1);
    if (max_screen_size && *max_screen_size != 0.0) {
        auto big_vs = max_radii2D_ > *max_screen_size;
        auto big_ws = std::get<0>(torch::exp(params_["scaling"]).max(1)) > 0.1 * extent;
        prune = prune | big_vs | big_ws;
    }
    prune_points(prune);
}

void Trainer::reset_opacity() {
    auto o = torch::sigmoid(params_["opacity"]);
    o = torch::minimum(o, torch::full_like(o, 0.01));
    params_["opacity"] = torch::log(o / (1 - o)).contiguous();  // inverse_sigmoid
    exp_avg_["opacity"].zero_();
    exp_avg_sq_["opacity"].zero_();
}

}  // namespace gsr

// gsr_torch.cpp -- libtorch layer over the C ABI: RasterizeGaussians autograd Function,
// render() helpers and the Python binding (_gsr_torch).  Host C++ only: every byte of device
// work goes through include/gsr/gsr.h into libgsr_hip.so (no torch types cross that ABI).
//
// Scratch buffers (geometry / binning / image) are uint8 tensors from torch's caching
// allocator, created inside the C ABI's allocation callbacks and kept in the autograd context
// until backward -- the library itself allocates nothing persistent.
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/Event.h>
#include <c10/hip/HIPStream.h>
#ifdef GSR_NO_PYBIND
#include <torch/torch.h>
#else
#include <torch/extension.h>
#endif

#include <cmath>
#include <cstdio>
#include <stdexcept>

#include "gsr_render.h"

namespace gsr {
namespace detail {
void check(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) + "): " +
                                          gsr_last_error());
}
void* current_stream() { return (void*)c10::hip::getCurrentHIPStream().stream(); }
}  // namespace detail

namespace {
using detail::check;

struct AllocCtx {
    torch::Device device;
    std::vector<torch::Tensor> keep;
};

void* alloc_cb(void* ctx, size_t bytes) {
    auto* c = static_cast<AllocCtx*>(ctx);
    auto t = torch::empty({(int64_t)std::max<size_t>(bytes, 16)},
                          torch::TensorOptions().dtype(torch::kUInt8).device(c->device));
    c->keep.push_back(t);
    return t.data_ptr();
}

// absent optional inputs travel through autograd as defined 0-element tensors (undefined
// tensors are rejected by Function::apply's input bookkeeping)
bool present(const torch::Tensor& t) { return t.defined() && t.numel() > 0; }

const float* fptr(const torch::Tensor& t, const char* name, int64_t P, int64_t per) {
    if (!present(t)) return nullptr;
    TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
    TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    TORCH_CHECK(t.numel() == P * per, name, " has ", t.numel(), " elements, expected ", P * per);
    return t.data_ptr<float>();
}

gsr_gaussians make_gaussians(const RasterSettings& rs, const torch::Tensor& means3D,
                             const torch::Tensor& sh_dc, const torch::Tensor& sh_rest,
                             const torch::Tensor& colors, const torch::Tensor& opac,
                             const torch::Tensor& scales, const torch::Tensor& rots,
                             const torch::Tensor& cov3D) {
    gsr_gaussians g{};
    const int64_t P = means3D.size(0);
    g.P = (int32_t)P;
    g.sh_degree = rs.sh_degree;
    g.scale_modifier = rs.scale_modifier;
    g.means3D = fptr(means3D, "means3D", P, 3);
    g.opacities = fptr(opac, "opacities", P, 1);
    if (present(colors)) {
        g.colors_precomp = fptr(colors, "colors_precomp", P, 3);
        g.sh_degree = 0;
    } else {
        g.sh_dc = fptr(sh_dc, "sh_dc", P, 3);
        if (present(sh_rest)) {
            const int64_t M = sh_rest.numel() / std::max<int64_t>(P, 1) / 3;
            g.sh_rest = fptr(sh_rest, "sh_rest", P, 3 * M);
            g.sh_rest_coeffs = (int32_t)M;
        }
    }
    if (present(cov3D)) {
        g.cov3D_precomp = fptr(cov3D, "cov3D_precomp", P, 6);
    } else {
        g.scales = fptr(scales, "scales", P, 3);
        g.rotations = fptr(rots, "rotations", P, 4);
    }
    return g;
}

gsr_raster_settings make_settings(const RasterSettings& rs) {
    gsr_raster_settings s{};
    for (int c = 0; c < 3; ++c) s.bg[c] = rs.bg[c];
    s.tile_y0 = rs.tile_y0;
    s.tile_y1 = rs.tile_y1;
    s.flags = rs.debug ? GSR_FLAG_DEBUG : 0u;
    s.max_rendered = rs.max_rendered;
    return s;
}

void* cur_stream() { return detail::current_stream(); }

using FwdResult = detail::Frame;

FwdResult forward_impl(const RasterCamera& cam, const RasterSettings& rs, const torch::Tensor& means3D,
                       const torch::Tensor& sh_dc, const torch::Tensor& sh_rest,
                       const torch::Tensor& colors, const torch::Tensor& opac,
                       const torch::Tensor& scales, const torch::Tensor& rots,
                       const torch::Tensor& cov3D) {
    TORCH_CHECK(means3D.dim() == 2 && means3D.size(1) == 3, "means3D must be (P,3)");
    const int64_t P = means3D.size(0);
    auto dev = means3D.device();
    auto fopt = torch::TensorOptions().dtype(torch::kFloat32).device(dev);
    FwdResult r;
    r.color = torch::empty({3, cam.height, cam.width}, fopt);
    r.radii = torch::empty({P}, fopt.dtype(torch::kInt32));
    const gsr_camera c = cam.to_c();
    const gsr_gaussians g = make_gaussians(rs, means3D, sh_dc, sh_rest, colors, opac, scales, rots, cov3D);
    const gsr_raster_settings s = make_settings(rs);
    AllocCtx geom{dev, {}}, bin{dev, {}}, img{dev, {}};
    gsr_buffers b{};
    AllocCtx* ctxs[3] = {&geom, &bin, &img};  // one context per role
    check(gsr_forward(&c, &g, &s, r.color.data_ptr<float>(), P ? r.radii.data_ptr<int32_t>() : nullptr,
                      [](void* ctx, size_t n) { return alloc_cb(static_cast<AllocCtx**>(ctx)[0], n); },
                      [](void* ctx, size_t n) { return alloc_cb(static_cast<AllocCtx**>(ctx)[1], n); },
                      [](void* ctx, size_t n) { return alloc_cb(static_cast<AllocCtx**>(ctx)[2], n); },
                      (void*)ctxs, &b, cur_stream()),
          "gsr_forward");
    r.geom = geom.keep.at(0);
    r.binning = bin.keep.empty() ? torch::Tensor() : bin.keep.at(0);
    r.image = img.keep.at(0);
    r.bufs = b;
    r.cam = c;
    r.settings = s;
    return r;
}

gsr_buffers buffers_of(const torch::Tensor& geom, const torch::Tensor& binning, const torch::Tensor& image,
                       int32_t K, int32_t cap, int32_t n_local, uint32_t layout) {
    gsr_buffers b{};
    b.layout = layout;  // the forward's layout word (gsr.h): the backward checks it
    b.geom = geom.data_ptr();
    b.binning = binning.defined() ? binning.data_ptr() : nullptr;
    b.image = image.data_ptr();
    b.num_rendered = K;
    b.capacity = cap;
    b.n_local = n_local;
    return b;
}

using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

class RasterizeGaussians : public torch::autograd::Function<RasterizeGaussians> {
   public:
    static variable_list forward(AutogradContext* ctx, const RasterCamera& cam, const RasterSettings& rs,
                                 torch::Tensor means3D, torch::Tensor means2D, torch::Tensor sh_dc,
                                 torch::Tensor sh_rest, torch::Tensor colors, torch::Tensor opac,
                                 torch::Tensor scales, torch::Tensor rots, torch::Tensor cov3D) {
        ctx->saved_data["has_m2d"] = present(means2D);
        auto r = forward_impl(cam, rs, means3D, sh_dc, sh_rest, colors, opac, scales, rots, cov3D);
        ctx->save_for_backward({means3D, sh_dc, sh_rest, colors, opac, scales, rots, cov3D, r.geom, r.binning,
                                r.image});
        ctx->saved_data["K"] = (int64_t)r.bufs.num_rendered;
        ctx->saved_data["cap"] = (int64_t)r.bufs.capacity;
        ctx->saved_data["n_local"] = (int64_t)r.bufs.n_local;
        ctx->saved_data["layout"] = (int64_t)r.bufs.layout;
        ctx->saved_data["cam_w"] = (int64_t)cam.width;
        ctx->saved_data["cam_h"] = (int64_t)cam.height;
        ctx->saved_data["cam_tx"] = (double)cam.tanfovx;
        ctx->saved_data["cam_ty"] = (double)cam.tanfovy;
        ctx->saved_data["cam_v"] = std::vector<double>(cam.viewmatrix.begin(), cam.viewmatrix.end());
        ctx->saved_data["cam_p"] = std::vector<double>(cam.projmatrix.begin(), cam.projmatrix.end());
        ctx->saved_data["cam_c"] = std::vector<double>(cam.campos.begin(), cam.campos.end());
        ctx->saved_data["bg"] = std::vector<double>(rs.bg.begin(), rs.bg.end());
        ctx->saved_data["smod"] = (double)rs.scale_modifier;
        ctx->saved_data["D"] = (int64_t)rs.sh_degree;
        ctx->saved_data["ty0"] = (int64_t)rs.tile_y0;
        ctx->saved_data["ty1"] = (int64_t)rs.tile_y1;
        ctx->saved_data["debug"] = rs.debug;
        ctx->saved_data["max_rendered"] = (int64_t)rs.max_rendered;
        auto kdev = r.k_device();
        auto kinfo = torch::tensor({r.bufs.num_rendered, r.bufs.capacity}, torch::kInt32);
        ctx->mark_non_differentiable({r.radii, kdev, kinfo});
        return {r.color, r.radii, kdev, kinfo};
    }

    static variable_list backward(AutogradContext* ctx, variable_list grad_out) {
        auto sv = ctx->get_saved_variables();
        auto means3D = sv[0], sh_dc = sv[1], sh_rest = sv[2], colors = sv[3], opac = sv[4], scales = sv[5],
             rots = sv[6], cov3D = sv[7], geom = sv[8], binning = sv[9], image = sv[10];
        RasterCamera cam;
        cam.width = (int)ctx->saved_data["cam_w"].toInt();
        cam.height = (int)ctx->saved_data["cam_h"].toInt();
        cam.tanfovx = (float)ctx->saved_data["cam_tx"].toDouble();
        cam.tanfovy = (float)ctx->saved_data["cam_ty"].toDouble();
        auto V = ctx->saved_data["cam_v"].toDoubleVector();
        auto Pm = ctx->saved_data["cam_p"].toDoubleVector();
        auto C = ctx->saved_data["cam_c"].toDoubleVector();
        for (int i = 0; i < 16; ++i) cam.viewmatrix[i] = (float)V[i], cam.projmatrix[i] = (float)Pm[i];
        for (int i = 0; i < 3; ++i) cam.campos[i] = (float)C[i];
        RasterSettings rs;
        auto bg = ctx->saved_data["bg"].toDoubleVector();
        for (int i = 0; i < 3; ++i) rs.bg[i] = (float)bg[i];
        rs.scale_modifier = (float)ctx->saved_data["smod"].toDouble();
        rs.sh_degree = (int)ctx->saved_data["D"].toInt();
        rs.tile_y0 = (int)ctx->saved_data["ty0"].toInt();
        rs.tile_y1 = (int)ctx->saved_data["ty1"].toInt();
        rs.debug = ctx->saved_data["debug"].toBool();
        rs.max_rendered = (int)ctx->saved_data["max_rendered"].toInt();
        const int32_t K = (int32_t)ctx->saved_data["K"].toInt();
        const int32_t cap = (int32_t)ctx->saved_data["cap"].toInt();
        const int32_t n_local = (int32_t)ctx->saved_data["n_local"].toInt();
        const uint32_t layout = (uint32_t)ctx->saved_data["layout"].toInt();
        auto dL_dcolor = grad_out[0].contiguous();
        const int64_t P = means3D.size(0);
        auto fo = means3D.options();
        auto g_means2D = torch::empty({P, 3}, fo);
        auto g_opac = torch::empty_like(opac);
        auto g_means3D = torch::empty({P, 3}, fo);
        torch::Tensor g_dc, g_rest, g_colors, g_scales, g_rots, g_cov;
        gsr_grads gg{};
        gg.dL_dmeans2D = g_means2D.data_ptr<float>();
        gg.dL_dopacity = g_opac.data_ptr<float>();
        gg.dL_dmeans3D = g_means3D.data_ptr<float>();
        if (present(colors)) {
            g_colors = torch::empty_like(colors);
            gg.dL_dcolors = g_colors.data_ptr<float>();
        } else {
            g_dc = torch::empty_like(sh_dc);
            gg.dL_dsh_dc = g_dc.data_ptr<float>();
            if (present(sh_rest)) {
                g_rest = torch::empty_like(sh_rest);
                gg.dL_dsh_rest = g_rest.data_ptr<float>();
            }
        }
        if (present(cov3D)) {
            g_cov = torch::empty_like(cov3D);
            gg.dL_dcov3D = g_cov.data_ptr<float>();
        } else {
            g_scales = torch::empty_like(scales);
            g_rots = torch::empty_like(rots);
            gg.dL_dscales = g_scales.data_ptr<float>();
            gg.dL_drotations = g_rots.data_ptr<float>();
        }
        const gsr_camera c = cam.to_c();
        const gsr_gaussians g = make_gaussians(rs, means3D, sh_dc, sh_rest, colors, opac, scales, rots, cov3D);
        const gsr_raster_settings s = make_settings(rs);
        const gsr_buffers b = buffers_of(geom, binning, image, K, cap, n_local, layout);
        AllocCtx scratch{means3D.device(), {}};
        check(gsr_backward(&c, &g, &s, &b, dL_dcolor.data_ptr<float>(), alloc_cb, &scratch, &gg, cur_stream()),
              "gsr_backward");
        // inputs of forward(): cam, rs, means3D, means2D, sh_dc, sh_rest, colors, opac, scales, rots, cov3D
        if (!ctx->saved_data["has_m2d"].toBool()) g_means2D = torch::Tensor();
        return {torch::Tensor(), torch::Tensor(), g_means3D, g_means2D, g_dc, g_rest, g_colors, g_opac,
                g_scales, g_rots, g_cov};
    }
};

}  // namespace

namespace detail {
torch::Tensor Frame::k_device() const {
    const void* p = gsr_view(&cam, bufs.n_local, &bufs, GSR_VIEW_COUNTS);
    TORCH_CHECK(p != nullptr, "gsr_view(COUNTS) returned NULL");
    const int64_t off = static_cast<const uint8_t*>(p) - static_cast<const uint8_t*>(image.data_ptr());
    TORCH_CHECK(off >= 0 && off + 4 <= image.numel(), "K counter outside the image buffer");
    return image.narrow(0, off, 4).view(torch::kInt32).clone();  // async device copy
}

Frame forward(const RasterCamera& cam, const RasterSettings& rs, const torch::Tensor& means3D,
              const torch::Tensor& sh_dc, const torch::Tensor& sh_rest, const torch::Tensor& colors,
              const torch::Tensor& opac, const torch::Tensor& scales, const torch::Tensor& rots,
              const torch::Tensor& cov3D) {
    return forward_impl(cam, rs, means3D, sh_dc, sh_rest, colors, opac, scales, rots, cov3D);
}

void backward(const Frame& f, const RasterSettings& rs, const torch::Tensor& means3D, const torch::Tensor& sh_dc,
              const torch::Tensor& sh_rest, const torch::Tensor& colors, const torch::Tensor& opac,
              const torch::Tensor& scales, const torch::Tensor& rots, const torch::Tensor& cov3D,
              const torch::Tensor& dL_dcolor, const gsr_grads& grads) {
    const gsr_gaussians g = make_gaussians(rs, means3D, sh_dc, sh_rest, colors, opac, scales, rots, cov3D);
    TORCH_CHECK(dL_dcolor.is_contiguous() && dL_dcolor.numel() == 3LL * f.cam.width * f.cam.height,
                "dL_dcolor must be a contiguous (3,H,W) tensor");
    AllocCtx scratch{means3D.device(), {}};
    check(gsr_backward(&f.cam, &g, &f.settings, &f.bufs, dL_dcolor.data_ptr<float>(), alloc_cb, &scratch, &grads,
                       cur_stream()),
          "gsr_backward");
}
}  // namespace detail

int read_num_rendered(const RenderOutput& out) {
    const int k = out.num_rendered_device.item<int32_t>();  // waits for the render's stream
    if (k > out.capacity)
        throw std::overflow_error("num_rendered " + std::to_string(k) + " exceeded the binning capacity " +
                                  std::to_string(out.capacity) + " (GSR_ERR_OVERFLOW): re-render with a larger bound");
    return k;
}

std::array<float, 3> background(const torch::Tensor& bg) {
    TORCH_CHECK(bg.numel() == 3, "background must have 3 values");
    auto h = bg.to(torch::kCPU, torch::kFloat32).contiguous();
    return {h.data_ptr<float>()[0], h.data_ptr<float>()[1], h.data_ptr<float>()[2]};
}

BinningCapacity::BinningCapacity(double headroom, int ring, bool strict) : headroom_(headroom), strict_(strict) {
    const bool pin = torch::cuda::is_available();
    for (int i = 0; i < ring; ++i) {
        slots_.push_back(torch::zeros({1}, torch::TensorOptions().dtype(torch::kInt32).pinned_memory(pin)));
        events_.push_back(new c10::Event(c10::DeviceType::CUDA));  // torch's event: one HIP runtime
    }
}

BinningCapacity::~BinningCapacity() {
    for (void* e : events_) delete static_cast<c10::Event*>(e);
}

void BinningCapacity::grow() { cap_ = (int)(((int64_t)(k_max_ * headroom_) + 65536 + 4095) / 4096 * 4096); }

int BinningCapacity::bound() {
    poll(false);
    return cap_;
}

void BinningCapacity::reset() {
    pending_.clear();
    cap_ = 0;
    k_max_ = 0;
}

void BinningCapacity::observe(const RenderOutput& out) { observe(out.num_rendered_device, out.num_rendered); }

void BinningCapacity::observe(const torch::Tensor& k_device, int host_k) {
    if (cap_ == 0) {  // an exactly sized render: its K was read back by the forward
        ++exact_reads_;
        k_max_ = std::max<int64_t>(k_max_, host_k);
        grow();
        return;
    }
    if (pending_.size() == slots_.size()) poll(true);  // ring full: wait for the oldest
    const int slot = next_;
    next_ = (next_ + 1) % (int)slots_.size();
    slots_[slot].copy_(k_device, /*non_blocking=*/true);
    static_cast<c10::Event*>(events_[slot])->record(at::hip::getCurrentHIPStreamMasqueradingAsCUDA().unwrap());
    pending_.push_back({slot, events_[slot], cap_});
}

void BinningCapacity::sync() {
    while (!pending_.empty()) poll(true);
}

void BinningCapacity::poll(bool wait_one) {
    bool waited = false;
    while (!pending_.empty()) {
        auto* e = static_cast<c10::Event*>(pending_.front().event);
        if (wait_one && !waited) {
            e->synchronize();
            waited = true;
        } else if (!e->query()) {
            break;
        }
        const Pending p = pending_.front();
        pending_.erase(pending_.begin());
        const int64_t k = slots_[p.slot].data_ptr<int32_t>()[0];
        if (k > p.cap) {  // that render was truncated (its statistics / Adam step skipped on the device)
            if (overflows_ == 0)
                std::fprintf(stderr, "[gsr] BinningCapacity: a render's K = %lld exceeded its bound %d; that "
                             "iteration's update was skipped on the device, renders are sized exactly again\n",
                             (long long)k, p.cap);
            ++overflows_;
            k_max_ = std::max(k_max_, k);
            pending_.clear();
            cap_ = 0;  // the next render is sized exactly
            if (strict_)
                throw std::overflow_error("a render's K = " + std::to_string(k) + " exceeded its bound " +
                                          std::to_string(p.cap));
            return;
        }
        if (k > k_max_) {
            k_max_ = k;
            if (k * 1.2 > cap_) grow();
        }
    }
}

RasterCamera RasterCamera::from_tensors(int width, int height, double FoVx, double FoVy,
                                        const torch::Tensor& wv, const torch::Tensor& fp,
                                        const torch::Tensor& cc) {
    RasterCamera c;
    c.width = width;
    c.height = height;
    c.tanfovx = (float)std::tan(FoVx * 0.5);
    c.tanfovy = (float)std::tan(FoVy * 0.5);
    auto v = wv.to(torch::kCPU, torch::kFloat32).contiguous();
    auto p = fp.to(torch::kCPU, torch::kFloat32).contiguous();
    auto o = cc.to(torch::kCPU, torch::kFloat32).contiguous();
    for (int i = 0; i < 16; ++i) c.viewmatrix[i] = v.data_ptr<float>()[i], c.projmatrix[i] = p.data_ptr<float>()[i];
    for (int i = 0; i < 3; ++i) c.campos[i] = o.data_ptr<float>()[i];
    return c;
}

gsr_camera RasterCamera::to_c() const {
    gsr_camera c{};
    c.width = width;
    c.height = height;
    c.tanfovx = tanfovx;
    c.tanfovy = tanfovy;
    for (int i = 0; i < 16; ++i) c.viewmatrix[i] = viewmatrix[i], c.projmatrix[i] = projmatrix[i];
    for (int i = 0; i < 3; ++i) c.campos[i] = campos[i];
    return c;
}

std::vector<torch::Tensor> rasterize_gaussians(const RasterCamera& cam, const RasterSettings& rs,
                                               const torch::Tensor& means3D, const torch::Tensor& means2D,
                                               const torch::Tensor& sh_dc, const torch::Tensor& sh_rest,
                                               const torch::Tensor& colors, const torch::Tensor& opac,
                                               const torch::Tensor& scales, const torch::Tensor& rots,
                                               const torch::Tensor& cov3D) {
    auto none = torch::empty({0}, means3D.options());
    auto opt_in = [&](const torch::Tensor& t) { return t.defined() ? t : none; };
    return RasterizeGaussians::apply(cam, rs, means3D, opt_in(means2D), opt_in(sh_dc), opt_in(sh_rest),
                                     opt_in(colors), opac, opt_in(scales), opt_in(rots), opt_in(cov3D));
}

torch::Tensor eval_sh_colors(int D, const torch::Tensor& sh, const torch::Tensor& dirs) {
    // same basis and constants as the kernels
    const double C0 = 0.28209479177387814, C1 = 0.4886025119029199;
    const double C2[5] = {1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
                          0.5462742152960396};
    const double C3[7] = {-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
                          -0.4570457994644658, 1.445305721320277, -0.5900435899266435};
    using torch::indexing::Slice;
    auto c = [&](int k) { return sh.index({Slice(), k}); };
    auto res = C0 * c(0);
    if (D > 0) {
        auto x = dirs.index({Slice(), Slice(0, 1)}), y = dirs.index({Slice(), Slice(1, 2)}),
             z = dirs.index({Slice(), Slice(2, 3)});
        res = res - C1 * y * c(1) + C1 * z * c(2) - C1 * x * c(3);
        if (D > 1) {
            auto xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            res = res + C2[0] * xy * c(4) + C2[1] * yz * c(5) + C2[2] * (2.0 * zz - xx - yy) * c(6) +
                  C2[3] * xz * c(7) + C2[4] * (xx - yy) * c(8);
            if (D > 2) {
                res = res + C3[0] * y * (3 * xx - yy) * c(9) + C3[1] * xy * z * c(10) +
                      C3[2] * y * (4 * zz - xx - yy) * c(11) + C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * c(12) +
                      C3[4] * x * (4 * zz - xx - yy) * c(13) + C3[5] * z * (xx - yy) * c(14) +
                      C3[6] * x * (xx - 3 * yy) * c(15);
            }
        }
    }
    return torch::clamp_min(res + 0.5, 0.0);
}

}  // namespace gsr

// ------------------------------------------------------------------------------------------
// Python binding (compile with -DGSR_NO_PYBIND when linking into a C++ executable)
// ------------------------------------------------------------------------------------------
#ifndef GSR_NO_PYBIND
namespace py = pybind11;

static gsr::RasterCamera cam_from_py(int w, int h, float tx, float ty, const std::vector<float>& v,
                                     const std::vector<float>& p, const std::vector<float>& c) {
    TORCH_CHECK(v.size() == 16 && p.size() == 16 && c.size() == 3, "bad camera arrays");
    gsr::RasterCamera cam;
    cam.width = w;
    cam.height = h;
    cam.tanfovx = tx;
    cam.tanfovy = ty;
    for (int i = 0; i < 16; ++i) cam.viewmatrix[i] = v[i], cam.projmatrix[i] = p[i];
    for (int i = 0; i < 3; ++i) cam.campos[i] = c[i];
    return cam;
}

static gsr::RasterSettings settings_from_py(const std::vector<float>& bg, float smod, int D, int ty0, int ty1,
                                            bool debug, int max_rendered) {
    gsr::RasterSettings rs;
    rs.max_rendered = max_rendered;
    for (int i = 0; i < 3; ++i) rs.bg[i] = bg.at(i);
    rs.scale_modifier = smod;
    rs.sh_degree = D;
    rs.tile_y0 = ty0;
    rs.tile_y1 = ty1;
    rs.debug = debug;
    return rs;
}

static torch::Tensor opt(const c10::optional<torch::Tensor>& t) { return t.has_value() ? *t : torch::Tensor(); }

namespace gsr {
void bind_shard(pybind11::module& m);  // gsr_shard.cpp
}

PYBIND11_MODULE(_gsr_torch, m) {
    m.doc() = "libtorch RasterizeGaussians over the gsr C ABI (libgsr_hip.so)";
    py::class_<gsr::RasterCamera>(m, "RasterCamera")
        .def(py::init(&cam_from_py), py::arg("width"), py::arg("height"), py::arg("tanfovx"),
             py::arg("tanfovy"), py::arg("viewmatrix"), py::arg("projmatrix"), py::arg("campos"))
        .def_readonly("width", &gsr::RasterCamera::width)
        .def_readonly("height", &gsr::RasterCamera::height)
        .def_readonly("tanfovx", &gsr::RasterCamera::tanfovx)
        .def_readonly("tanfovy", &gsr::RasterCamera::tanfovy)
        .def_readonly("viewmatrix", &gsr::RasterCamera::viewmatrix)
        .def_readonly("projmatrix", &gsr::RasterCamera::projmatrix)
        .def_readonly("campos", &gsr::RasterCamera::campos);
    py::class_<gsr::RasterSettings>(m, "RasterSettings")
        .def(py::init(&settings_from_py), py::arg("bg"), py::arg("scale_modifier") = 1.0f,
             py::arg("sh_degree") = 0, py::arg("tile_y0") = 0, py::arg("tile_y1") = INT32_MAX,
             py::arg("debug") = false, py::arg("max_rendered") = 0);
    m.def(
        "rasterize_gaussians",
        [](const gsr::RasterCamera& cam, const gsr::RasterSettings& rs, torch::Tensor means3D,
           torch::Tensor means2D, c10::optional<torch::Tensor> sh_dc, c10::optional<torch::Tensor> sh_rest,
           c10::optional<torch::Tensor> colors, torch::Tensor opac, c10::optional<torch::Tensor> scales,
           c10::optional<torch::Tensor> rots, c10::optional<torch::Tensor> cov3D) {
            auto r = gsr::rasterize_gaussians(cam, rs, means3D, means2D, opt(sh_dc), opt(sh_rest), opt(colors),
                                              opac, opt(scales), opt(rots), opt(cov3D));
            return py::make_tuple(r[0], r[1]);
        },
        py::arg("cam"), py::arg("settings"), py::arg("means3D"), py::arg("means2D"), py::arg("sh_dc"),
        py::arg("sh_rest"), py::arg("colors_precomp"), py::arg("opacities"), py::arg("scales"),
        py::arg("rotations"), py::arg("cov3D_precomp"));
    m.def("eval_sh_colors", &gsr::eval_sh_colors);
    m.def(
        "camera_from_tensors",
        [](int w, int h, double fovx, double fovy, torch::Tensor wv, torch::Tensor fp, torch::Tensor cc) {
            return gsr::RasterCamera::from_tensors(w, h, fovx, fovy, wv, fp, cc);
        },
        py::arg("width"), py::arg("height"), py::arg("FoVx"), py::arg("FoVy"), py::arg("world_view_transform"),
        py::arg("full_proj_transform"), py::arg("camera_center"));
    m.def("abi_version", []() { return gsr_abi_version(); });
    gsr::bind_shard(m);
}
#endif  // GSR_NO_PYBIND

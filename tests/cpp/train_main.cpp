// train_main.cpp -- the reference's training loop, src/utils/train_utils.cpp:97-146, with the
// body its stub leaves out, in C++ on gsr::Trainer (csrc/torch/gsr_trainer.h): per iteration
// update_learning_rate, oneup_SH_degree every 1000 iterations, a camera from the shuffled
// viewpoint stack, render -> L1 + D-SSIM -> backward, densification statistics, densify / prune
// and opacity reset on the OptimizationParams schedule (params.h:50-91), the optimizer step.
//
// Built by __graft_entry__.build() into 3d_gaussian_splatting_amd/lib/gsr_train_loop; run by
// tests/test_gpu_train_loop.py (against the Python train_loop.train on the same scene) and by
// `bench.py --mode loop` (the 30k-iteration configs[4] line).
//
// usage: gsr_train_loop SCENE.bin RESULT.json [FINAL_PARAMS.bin]
// SCENE.bin (little-endian, written by train_loop.write_scene):
//   char[8] "GSRLOOP1"
//   int32 n_views, W, H, n_init, iterations, max_sh_degree, seed, log_every, densify, progress_every
//   int32 OptimizationParams ints: iterations, position_lr_max_steps, densification_interval,
//         opacity_reset_interval, densify_from_iter, densify_until_iter, random_background
//   f32   OptimizationParams floats: position_lr_init, position_lr_final, position_lr_delay_mult,
//         feature_lr, opacity_lr, scaling_lr, rotation_lr, percent_dense, lambda_dssim,
//         densify_grad_threshold
//   f64   extent;  f32 bg[3]
//   f32   cameras[n_views][37]: tanfovx, tanfovy, viewmatrix[16], projmatrix[16], campos[3]
//   f32   gt[n_views][3][H][W];  f32 points[n_init][3];  f32 colors[n_init][3]
//   int32 views[iterations]: the camera of each iteration (the viewpoint-stack order)
#include <torch/torch.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <vector>

#include "gsr_trainer.h"

namespace {
template <class T>
std::vector<T> read_n(std::ifstream& f, size_t n) {
    std::vector<T> v(n);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(sizeof(T) * n));
    if (!f) throw std::runtime_error("short scene file");
    return v;
}
double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void write_t(std::ofstream& f, const torch::Tensor& t) {
    auto c = t.detach().to(torch::kCPU).contiguous();
    f.write(reinterpret_cast<const char*>(c.data_ptr()), (std::streamsize)(c.numel() * c.element_size()));
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s SCENE.bin RESULT.json [FINAL_PARAMS.bin]\n", argv[0]);
        return 2;
    }
    try {
        std::ifstream in(argv[1], std::ios::binary);
        if (!in) throw std::runtime_error("cannot open scene file");
        char magic[8];
        in.read(magic, 8);
        if (!in || std::memcmp(magic, "GSRLOOP1", 8) != 0) throw std::runtime_error("not a GSRLOOP1 scene file");
        auto h = read_n<int32_t>(in, 10);
        const int n_views = h[0], W = h[1], H = h[2], n_init = h[3], iterations = h[4], max_sh = h[5];
        const uint64_t seed = (uint64_t)h[6];
        const int log_every = h[7], progress_every = h[9];
        const bool densify = h[8] != 0;
        auto oi = read_n<int32_t>(in, 7);
        auto of = read_n<float>(in, 10);
        gsr::OptimizationParams opt;
        opt.iterations_ = oi[0];
        opt.position_lr_max_steps_ = oi[1];
        opt.densification_interval_ = oi[2];
        opt.opacity_reset_interval_ = oi[3];
        opt.densify_from_iter_ = oi[4];
        opt.densify_until_iter_ = oi[5];
        opt.random_background_ = oi[6] != 0;
        opt.position_lr_init_ = of[0];
        opt.position_lr_final_ = of[1];
        opt.position_lr_delay_mult_ = of[2];
        opt.feature_lr_ = of[3];
        opt.opacity_lr_ = of[4];
        opt.scaling_lr_ = of[5];
        opt.rotation_lr_ = of[6];
        opt.percent_dense_ = of[7];
        opt.lambda_dssim_ = of[8];
        opt.densify_grad_threshold_ = of[9];
        const double extent = read_n<double>(in, 1)[0];
        auto bgv = read_n<float>(in, 3);
        const std::array<float, 3> bg{bgv[0], bgv[1], bgv[2]};
        std::vector<gsr::RasterCamera> cams(n_views);
        for (auto& c : cams) {
            auto v = read_n<float>(in, 37);
            c.width = W;
            c.height = H;
            c.tanfovx = v[0];
            c.tanfovy = v[1];
            for (int i = 0; i < 16; ++i) c.viewmatrix[i] = v[2 + i], c.projmatrix[i] = v[18 + i];
            for (int i = 0; i < 3; ++i) c.campos[i] = v[34 + i];
        }
        const torch::Device dev(torch::kCUDA, 0);
        std::vector<torch::Tensor> gts;
        {
            std::vector<float> buf((size_t)3 * H * W);
            for (int v = 0; v < n_views; ++v) {
                in.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)(buf.size() * sizeof(float)));
                if (!in) throw std::runtime_error("short scene file (gt)");
                gts.push_back(torch::from_blob(buf.data(), {3, H, W}, torch::kFloat32).to(dev).contiguous());
            }
        }
        auto pts = read_n<float>(in, (size_t)n_init * 3), cols = read_n<float>(in, (size_t)n_init * 3);
        auto seq = read_n<int32_t>(in, (size_t)iterations);
        auto points = torch::from_blob(pts.data(), {n_init, 3}, torch::kFloat32).to(dev);
        auto colors = torch::from_blob(cols.data(), {n_init, 3}, torch::kFloat32).to(dev);

        // train_utils.cpp:104-108: the model and GaussianModel::setup (here create_from_pcd + setup)
        auto trainer = gsr::Trainer::from_point_cloud(points, colors, max_sh, extent, opt, seed);
        std::vector<std::pair<int, torch::Tensor>> logged;
        std::vector<std::pair<int, int>> counts;
        int peak = trainer->num_points();
        torch::cuda::synchronize();
        const double t0 = now();
        // train_utils.cpp:128-145
        for (int iteration = 1; iteration <= iterations; ++iteration) {
            const int v = seq[iteration - 1];  // viewpoint stack pick
            if (v < 0 || v >= n_views) throw std::runtime_error("view index out of range");
            auto out = trainer->step(iteration, cams[v], gts[v], bg, densify);
            if (iteration % log_every == 0 || iteration == 1 || iteration == iterations)
                logged.emplace_back(iteration, out.stats);
            if (iteration < opt.densify_until_iter_ && iteration > opt.densify_from_iter_ &&
                iteration % opt.densification_interval_ == 0)
                counts.emplace_back(iteration, out.num_points);
            peak = std::max(peak, out.num_points);
            if (progress_every > 0 && iteration % progress_every == 0) {
                std::fprintf(stderr, "[gsr_train_loop] iteration %d points %d %.1f s\n", iteration, out.num_points,
                             now() - t0);
                std::fflush(stderr);
            }
        }
        torch::cuda::synchronize();
        const double secs = now() - t0;
        trainer->binning().sync();
        std::FILE* f = std::fopen(argv[2], "w");
        if (!f) throw std::runtime_error("cannot write the result file");
        std::fprintf(f, "{\"iterations\": %d, \"seconds\": %.6f, \"iters_per_s\": %.4f, \"final_points\": %d, "
                        "\"peak_points\": %d, \"binning_overflows\": %lld, \"exact_k_reads\": %lld, "
                        "\"active_sh_degree\": %d,\n \"num_points\": [",
                     iterations, secs, iterations / secs, trainer->num_points(), peak,
                     (long long)trainer->binning().overflows(), (long long)trainer->binning().exact_reads(),
                     trainer->active_sh_degree());
        for (size_t i = 0; i < counts.size(); ++i)
            std::fprintf(f, "%s[%d, %d]", i ? ", " : "", counts[i].first, counts[i].second);
        std::fprintf(f, "],\n \"loss\": [");
        for (size_t i = 0; i < logged.size(); ++i) {
            auto s = logged[i].second.to(torch::kCPU);
            const float* p = s.data_ptr<float>();
            std::fprintf(f, "%s[%d, %.9g, %.9g, %.9g]", i ? ", " : "", logged[i].first, p[0], p[1], p[2]);
        }
        std::fprintf(f, "]}\n");
        std::fclose(f);
        if (argc > 3) {  // the final raw leaves, in group order
            std::ofstream o(argv[3], std::ios::binary);
            for (const char* k : gsr::Trainer::kGroupNames) write_t(o, trainer->params().at(k));
        }
        std::printf("gsr_train_loop ok: %d iterations in %.2f s (%.1f it/s), %d final points\n", iterations, secs,
                    iterations / secs, trainer->num_points());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "gsr_train_loop failed: %s\n", e.what());
        return 1;
    }
    return 0;
}

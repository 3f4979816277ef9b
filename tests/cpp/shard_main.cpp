// shard_main.cpp -- one rank of the C++ multi-GPU step (gsr::ShardStep, csrc/torch/gsr_shard.h),
// run as its own process: the drop-in shape of a sharded src/train.cpp (train_utils.cpp:97-146
// would construct the Exchange and the ShardStep once and call step() in its loop).
//
// usage: gsr_shard_step SCENE.bin OUT.bin
//   env RANK, WORLD_SIZE, MASTER_ADDR (default 127.0.0.1), MASTER_PORT: the c10d::TCPStore
//   rendezvous (rank 0 hosts it); GSR_TRANSPORT = store (host-staged, ranks may share a GPU) |
//   rccl (one GPU per rank); GSR_GRAPH = 1: capture the step into a hipGraph (rccl only);
//   GSR_STEPS (default 2); GSR_FORCE_PAIR_CAP > 0: shrink pair_cap after plan() (overflow test);
//   GSR_CAM_PATH = file of cameras (f32 tanfovx, tanfovy, view[16], proj[16], campos[3] each): step i
//   renders camera i mod n (set_camera before the step); GSR_LIVE = 1: live re-planning;
//   GSR_ALL_IMAGES = 1: OUT.bin ends with every step's image (steps x 3 x H x W f32);
//   GSR_TIMING = 1: synchronise after every step and print its wall time (re-plan cost).
//
// SCENE.bin ("GSRSHRD1"): int32 P, W, H, sh_degree, M (sh_rest coefficients per Gaussian);
//   f32 tanfovx, tanfovy, view[16], proj[16], campos[3]; f32 arrays means3D (P,3), opacities (P),
//   scales (P,3), rotations (P,4), sh_dc (P,1,3), sh_rest (P,M,3), dL_dpix (3,H,W).
// OUT.bin ("GSRSHOUT"): int64 g0, g1, pair_cap, capacity, steps_done, overflow_step (-1: none),
//   overflow_rank, graph_active; int32 rows[world + 1]; f32 image (3,H,W); int32 radii (g1-g0);
//   f32 grads means2D (n,3), opacities (n), means3D (n,3), sh_dc (n,3), sh_rest (n,M,3),
//   scales (n,3), rotations (n,4).
#include <torch/csrc/distributed/c10d/TCPStore.hpp>
#include <torch/torch.h>

#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "gsr_shard.h"

namespace {
int env_int(const char* k, int d) {
    const char* v = std::getenv(k);
    return v && *v ? std::atoi(v) : d;
}
std::string env_str(const char* k, const char* d) {
    const char* v = std::getenv(k);
    return v && *v ? v : d;
}
template <class T>
void put(std::ofstream& o, const T& v) {
    o.write(reinterpret_cast<const char*>(&v), sizeof v);
}
void put_t(std::ofstream& o, const torch::Tensor& t) {
    auto c = t.contiguous().cpu();
    o.write(reinterpret_cast<const char*>(c.data_ptr()), c.numel() * c.element_size());
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s SCENE.bin OUT.bin\n", argv[0]);
        return 2;
    }
    try {
        const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1);
        const std::string transport = env_str("GSR_TRANSPORT", "store");
        const bool graph = env_int("GSR_GRAPH", 0) != 0;
        const int steps = env_int("GSR_STEPS", 2), force_cap = env_int("GSR_FORCE_PAIR_CAP", 0);
        std::ifstream in(argv[1], std::ios::binary);
        char magic[8];
        in.read(magic, 8);
        if (!in || std::string(magic, 8) != "GSRSHRD1") throw std::runtime_error("bad scene file");
        int32_t h[5];
        in.read(reinterpret_cast<char*>(h), sizeof h);
        const int P = h[0], W = h[1], H = h[2], D = h[3], M = h[4];
        gsr::RasterCamera cam;
        cam.width = W;
        cam.height = H;
        in.read(reinterpret_cast<char*>(&cam.tanfovx), 4);
        in.read(reinterpret_cast<char*>(&cam.tanfovy), 4);
        in.read(reinterpret_cast<char*>(cam.viewmatrix.data()), 64);
        in.read(reinterpret_cast<char*>(cam.projmatrix.data()), 64);
        in.read(reinterpret_cast<char*>(cam.campos.data()), 12);
        torch::Device dev(torch::kCUDA, 0);
        auto rd = [&](std::vector<int64_t> shape) {
            auto t = torch::empty(shape, torch::kFloat32);
            in.read(reinterpret_cast<char*>(t.data_ptr<float>()), t.numel() * 4);
            if (!in) throw std::runtime_error("truncated scene file");
            return t.to(dev);
        };
        gsr::ShardInputs si;
        si.means3D = rd({P, 3});
        si.opacities = rd({P});
        si.scales = rd({P, 3});
        si.rotations = rd({P, 4});
        si.sh_dc = rd({P, 1, 3});
        si.sh_rest = rd({P, M, 3});
        si.sh_degree = D;
        auto dpix = rd({3, H, W});
        auto read_cam = [&](std::ifstream& f) {
            gsr::RasterCamera c = cam;
            f.read(reinterpret_cast<char*>(&c.tanfovx), 4);
            f.read(reinterpret_cast<char*>(&c.tanfovy), 4);
            f.read(reinterpret_cast<char*>(c.viewmatrix.data()), 64);
            f.read(reinterpret_cast<char*>(c.projmatrix.data()), 64);
            f.read(reinterpret_cast<char*>(c.campos.data()), 12);
            return c;
        };
        std::vector<gsr::RasterCamera> path;
        if (const std::string pf = env_str("GSR_CAM_PATH", ""); !pf.empty()) {
            std::ifstream cf(pf, std::ios::binary);
            while (true) {
                gsr::RasterCamera c = read_cam(cf);
                if (!cf) break;
                path.push_back(c);
            }
            if (path.empty()) throw std::runtime_error("empty camera path");
        }
        const bool live = env_int("GSR_LIVE", 0) != 0, all_images = env_int("GSR_ALL_IMAGES", 0) != 0,
                   timing = env_int("GSR_TIMING", 0) != 0;

        c10d::TCPStoreOptions opts;
        opts.port = (uint16_t)env_int("MASTER_PORT", 29500);
        opts.isServer = rank == 0;
        opts.numWorkers = world;
        auto store = c10::make_intrusive<c10d::TCPStore>(env_str("MASTER_ADDR", "127.0.0.1"), opts);
        std::shared_ptr<c10d::Store> sstore(store.get(), [keep = store](c10d::Store*) mutable { keep.reset(); });
        std::unique_ptr<gsr::Exchange> ex = transport == "rccl" ? gsr::rccl_exchange(*store, rank, world)
                                                                : gsr::store_exchange(sstore, rank, world);
        gsr::ShardStep step(*ex, path.empty() ? cam : path[0], si, {0.f, 0.f, 0.f}, 1.25, graph, 2);
        step.plan();
        if (force_cap > 0) step.set_pair_cap(force_cap);
        step.set_live_replan(live);
        gsr::ShardStep::Result res;
        int64_t done = 0, ovf_step = -1, ovf_rank = -1;
        std::vector<torch::Tensor> images;
        try {
            for (int i = 0; i < steps; ++i) {
                if (!path.empty()) step.set_camera(path[i % path.size()]);
                const int64_t lr0 = step.live_replans();
                const auto t0 = std::chrono::steady_clock::now();
                res = step.step(dpix);
                if (timing) {
                    torch::cuda::synchronize();
                    const double ms =
                        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                    std::fprintf(stderr, "{\"rank\": %d, \"step\": %d, \"ms\": %.4f, \"replanned\": %d, \"graph\": %d}\n",
                                 rank, i, ms, (int)(step.live_replans() > lr0), (int)step.graph_active());
                }
                if (all_images) images.push_back(res.image.clone());
                ++done;
            }
            step.check();
        } catch (const gsr::ShardOverflowError& e) {
            ovf_step = e.step;
            ovf_rank = e.rank;
            std::fprintf(stderr, "[gsr_shard_step rank %d] %s\n", rank, e.what());
        }
        torch::cuda::synchronize();
        std::ofstream o(argv[2], std::ios::binary);
        o.write("GSRSHOUT", 8);
        for (int64_t v : {step.g0(), step.g1(), (int64_t)step.pair_cap(), (int64_t)step.capacity(), done, ovf_step,
                          ovf_rank, (int64_t)step.graph_active()})
            put(o, v);
        for (int r : step.rows()) put(o, (int32_t)r);
        if (done > 0) {
            put_t(o, res.image);
            put_t(o, res.radii);
            for (const char* k : {"means2D", "opacities", "means3D", "sh_dc", "sh_rest", "scales", "rotations"})
                put_t(o, res.grads.at(k));
        }
        for (const auto& im : images) put_t(o, im);
        const long long store_keys = (long long)store->getNumKeys();
        // rank 0 hosts the store: it leaves only after every rank is past its last store call
        store->add("gsr_main/exit", 1);
        for (int spin = 0; rank == 0 && spin < 30000 && store->add("gsr_main/exit", 0) < world; ++spin)
            std::this_thread::sleep_for(std::chrono::milliseconds(1));  // (bounded: a failed rank never arrives)
        std::fprintf(stderr,
                     "[gsr_shard_step rank %d/%d] %s exchange, graph %d, %lld steps, pair_cap %d, capacity %d, "
                     "store_keys %lld, live_replans %lld\n",
                     rank, world, ex->name(), (int)step.graph_active(), (long long)done, step.pair_cap(),
                     step.capacity(), store_keys, (long long)step.live_replans());
        return 0;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "gsr_shard_step failed: %s\n", e.what());
        return 1;
    }
}

// gsr_shard.cpp -- the multi-GPU step in C++ over RCCL (see gsr_shard.h).
#include "gsr_shard.h"

#include <ATen/hip/HIPGraph.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/Event.h>
#include <c10/core/StreamGuard.h>
#include <torch/csrc/distributed/c10d/Store.hpp>

#include "gsr/gsr_comm.h"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <thread>

namespace gsr {
namespace {

int64_t round_up(int64_t x, int64_t m = 256) { return (x + m - 1) / m * m; }
constexpr int kMaxLocalRanks = 16;

using Stream = c10::hip::HIPStreamMasqueradingAsCUDA;
// c10's device-generic guard and events (they dispatch through the registered HIP guard
// implementation): this file then references no HIP runtime symbol itself, so an executable
// linking it keeps libtorch's one HIP runtime (tests/test_native_abi.py).
using StreamGuard = c10::StreamGuard;

Stream current_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(); }
// a device tensor over raw device memory (no ownership)
torch::Tensor dev_view(void* p, int64_t n, torch::ScalarType t) {
    return torch::from_blob(p, {n}, torch::TensorOptions().dtype(t).device(torch::kCUDA, c10::hip::current_device()));
}

// ---- RCCL exchange: the C ABI of libgsr_hip.so (include/gsr/gsr_comm.h) ----
class RcclExchange final : public Exchange {
   public:
    RcclExchange(const std::vector<uint8_t>& id, int rank, int world) : rank_(rank), world_(world) {
        if (id.size() != GSR_COMM_ID_BYTES) throw std::invalid_argument("rccl: bad unique id size");
        detail::check(gsr_comm_init(&comm_, id.data(), world, rank), "gsr_comm_init");
    }
    ~RcclExchange() override { (void)gsr_comm_destroy(comm_); }
    int rank() const override { return rank_; }
    int world() const override { return world_; }
    bool capturable() const override { return true; }
    const char* name() const override { return "rccl"; }
    int comm_world() const override {
        int32_t n = 0, r = 0;
        detail::check(gsr_comm_size(comm_, &n, &r), "gsr_comm_size");
        return n;
    }
    void all_to_all(const void* send, void* recv, size_t bb, hipStream_t s) override {
        detail::check(gsr_comm_all_to_all(comm_, send, recv, bb, s), "gsr_comm_all_to_all");
    }
    void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        detail::check(gsr_comm_all_gather(comm_, send, recv, bytes, s), "gsr_comm_all_gather");
    }
    void all_reduce_i64(int64_t* buf, size_t n, bool max, hipStream_t s) override {
        detail::check(gsr_comm_all_reduce_i64(comm_, buf, n, max ? 1 : 0, s), "gsr_comm_all_reduce_i64");
    }

   private:
    int rank_, world_;
    gsr_comm* comm_ = nullptr;
};

// ---- host-staged exchange through a c10d::Store (ranks sharing one GPU) ----
class StoreExchange final : public Exchange {
   public:
    // Every rank announces itself under this exchange's join key (exchanges are created in the
    // same order on every rank, so the per-process counter names the same key everywhere) and
    // waits until `world` ranks have: comm_world() is then the store's own count of the ranks
    // that joined, not the number the caller claimed.
    StoreExchange(std::shared_ptr<c10d::Store> store, int rank, int world)
        : store_(std::move(store)), rank_(rank), world_(world) {
        static int instances = 0;
        join_key_ = "gsr/join/" + std::to_string(instances++);
        store_->add(join_key_, 1);
        for (int spin = 0; store_->add(join_key_, 0) < world_; ++spin) {
            if (spin > 600000) throw std::runtime_error("store exchange: ranks did not join within 120 s");
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }
    int rank() const override { return rank_; }
    int world() const override { return world_; }
    bool capturable() const override { return false; }
    const char* name() const override { return "store"; }
    int comm_world() const override { return (int)store_->add(join_key_, 0); }
    void all_to_all(const void* send, void* recv, size_t bb, hipStream_t s) override {
        const std::string tag = "gsr/a2a/" + std::to_string(seq_++) + "/";
        std::vector<uint8_t> h((size_t)world_ * bb);
        d2h(h.data(), send, h.size(), s);
        for (int p = 0; p < world_; ++p)
            put(tag + std::to_string(rank_) + ">" + std::to_string(p), h.data() + (size_t)p * bb, bb);
        for (int p = 0; p < world_; ++p) {
            const std::string key = tag + std::to_string(p) + ">" + std::to_string(rank_);
            take(key, h.data() + (size_t)p * bb, bb, /*erase=*/true);
        }
        h2d(recv, h.data(), h.size(), s);
    }
    void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        const std::string tag = "gsr/ag/" + std::to_string(seq_++) + "/";
        std::vector<uint8_t> h(bytes);
        d2h(h.data(), send, bytes, s);
        put(tag + std::to_string(rank_), h.data(), bytes);
        std::vector<uint8_t> all((size_t)world_ * bytes);
        for (int p = 0; p < world_; ++p) take(tag + std::to_string(p), all.data() + (size_t)p * bytes, bytes, false);
        barrier(tag);
        release(tag, bytes);
        h2d(recv, all.data(), all.size(), s);
    }
    void all_reduce_i64(int64_t* buf, size_t n, bool max, hipStream_t s) override {
        std::vector<int64_t> mine(n), acc(n);
        all_gather_host(mine, buf, n, s, acc, max);
        h2d(buf, acc.data(), n * sizeof(int64_t), s);
    }

   private:
    void all_gather_host(std::vector<int64_t>& mine, const int64_t* dev, size_t n, hipStream_t s,
                         std::vector<int64_t>& acc, bool max) {
        d2h(mine.data(), dev, n * sizeof(int64_t), s);
        const std::string tag = "gsr/ar/" + std::to_string(seq_++) + "/";
        std::vector<uint8_t> b(n * sizeof(int64_t));
        std::memcpy(b.data(), mine.data(), b.size());
        store_->set(tag + std::to_string(rank_), b);
        for (int p = 0; p < world_; ++p) {
            auto v = store_->get(tag + std::to_string(p));
            const int64_t* x = reinterpret_cast<const int64_t*>(v.data());
            for (size_t i = 0; i < n; ++i) acc[i] = p == 0 ? x[i] : (max ? std::max(acc[i], x[i]) : acc[i] + x[i]);
        }
        barrier(tag);
        release(tag);
    }
    void barrier(const std::string& tag) {
        store_->add(tag + "done", 1);
        while (store_->add(tag + "done", 0) < world_) std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    // After barrier(tag): every rank has read every payload, so the last rank to leave deletes the
    // payloads and both counters -- a long run leaves no keys behind in the store.
    void release(const std::string& tag, size_t bytes = 0) {
        if (store_->add(tag + "left", 1) < world_) return;
        for (int p = 0; p < world_; ++p) {
            if (bytes == 0) {
                store_->deleteKey(tag + std::to_string(p));
            } else {
                for (size_t c = 0; c < chunks(bytes); ++c) store_->deleteKey(tag + std::to_string(p) + "#" + std::to_string(c));
            }
        }
        store_->deleteKey(tag + "done");
        store_->deleteKey(tag + "left");
    }
    // Values go through the store in pieces of at most kChunk bytes (the libuv TCPStore refuses
    // payloads above 8 MiB; a 1M / 1080p splat block for 2 ranks is 17.8 MB).  The reader knows the
    // size, hence the number of pieces.
    static constexpr size_t kChunk = 4u << 20;
    static size_t chunks(size_t n) { return n == 0 ? 1 : (n + kChunk - 1) / kChunk; }
    void put(const std::string& key, const uint8_t* data, size_t n) {
        for (size_t c = 0; c < chunks(n); ++c) {
            const size_t a = c * kChunk, b = std::min(n, a + kChunk);
            store_->set(key + "#" + std::to_string(c), std::vector<uint8_t>(data + a, data + b));
        }
    }
    void take(const std::string& key, uint8_t* out, size_t n, bool erase) {
        for (size_t c = 0; c < chunks(n); ++c) {
            const std::string k = key + "#" + std::to_string(c);
            auto v = store_->get(k);
            const size_t a = c * kChunk, want = std::min(n, a + kChunk) - a;
            if (v.size() != want) throw std::runtime_error("store exchange: block size mismatch");
            std::memcpy(out + a, v.data(), want);
            if (erase) store_->deleteKey(k);
        }
    }
    // synchronous copies on the caller's current stream (the step runs with it set to its own)
    static void d2h(void* h, const void* d, size_t n, hipStream_t) {
        auto src = dev_view(const_cast<void*>(d), (int64_t)n, torch::kUInt8);
        torch::from_blob(h, {(int64_t)n}, torch::kUInt8).copy_(src);
    }
    static void h2d(void* d, const void* h, size_t n, hipStream_t) {
        dev_view(d, (int64_t)n, torch::kUInt8).copy_(torch::from_blob(const_cast<void*>(h), {(int64_t)n}, torch::kUInt8));
        current_stream().unwrap().synchronize();  // h is a host buffer of this call
    }
    std::shared_ptr<c10d::Store> store_;
    int rank_, world_;
    int64_t seq_ = 0;
    std::string join_key_;
};

}  // namespace

// ---- in-process rank group (one-GPU rehearsal; gsr_shard.h) ----
class LocalGroup {
   public:
    explicit LocalGroup(int world) : world_(world), pub_(world), fin_(world), host_(world) {}
    int world() const { return world_; }
    void barrier() {
        std::unique_lock<std::mutex> lk(mu_);
        const int64_t gen = gen_;
        if (++count_ == world_) {
            count_ = 0;
            ++gen_;
            cv_.notify_all();
        } else {
            cv_.wait(lk, [&] { return gen_ != gen; });
        }
    }
    struct Pub {
        const void* ptr = nullptr;
        c10::Event* ev = nullptr;
    };
    std::vector<Pub> pub_;             // per rank: its send buffer and the event after it was written
    std::vector<c10::Event*> fin_;     // per rank: the event after its copies from the peers
    std::vector<std::vector<int64_t>> host_;  // all-reduce contributions

   private:
    int world_;
    std::mutex mu_;
    std::condition_variable cv_;
    int count_ = 0;
    int64_t gen_ = 0;
};

namespace {
class LocalExchange final : public Exchange {
   public:
    LocalExchange(std::shared_ptr<LocalGroup> g, int rank) : g_(std::move(g)), rank_(rank) {
        if (rank < 0 || rank >= g_->world()) throw std::invalid_argument("local exchange: rank out of range");
    }
    int rank() const override { return rank_; }
    int world() const override { return g_->world(); }
    bool capturable() const override { return replay_; }
    const char* name() const override { return replay_ ? "local-replay" : "local"; }
    // copies = false: replay without moving any bytes -- the step's receive buffers still hold
    // the last delivery, so the results are the same and the time is the rank's compute + glue
    void set_replay(bool on, bool copies) {
        if (on && snap_.size() < 3) throw std::runtime_error("local exchange: replay needs one live step first");
        replay_ = on;
        replay_copies_ = copies;
    }
    void all_to_all(const void* send, void* recv, size_t bb, hipStream_t s) override {
        const int w = g_->world();
        deliver(s, send, recv, (size_t)w * bb, /*always=*/false, [&](int p, const char* src) {
            copy(static_cast<char*>(recv) + (size_t)p * bb, src + (size_t)rank_ * bb, bb);
        });
    }
    // (the image all-gather runs on the step's side stream, overlapping B1: replayed with its
    // copy in both replay modes, as RCCL's would overlap -- and so that the side stream's branch
    // of a captured graph is never empty)
    void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        deliver(s, send, recv, (size_t)g_->world() * bytes, /*always=*/true, [&](int p, const char* src) {
            copy(static_cast<char*>(recv) + (size_t)p * bytes, src, bytes);
        });
    }
    void all_reduce_i64(int64_t* buf, size_t n, bool max, hipStream_t) override {
        auto d = dev_view(buf, (int64_t)(n * sizeof(int64_t)), torch::kUInt8);
        std::vector<int64_t> mine(n);
        torch::from_blob(mine.data(), {(int64_t)(n * sizeof(int64_t))}, torch::kUInt8).copy_(d);
        g_->host_[rank_] = mine;
        g_->barrier();
        std::vector<int64_t> acc = g_->host_[0];
        for (int p = 1; p < g_->world(); ++p)
            for (size_t i = 0; i < n; ++i) acc[i] = max ? std::max(acc[i], g_->host_[p][i]) : acc[i] + g_->host_[p][i];
        g_->barrier();  // everyone has read every contribution
        d.copy_(torch::from_blob(acc.data(), {(int64_t)(n * sizeof(int64_t))}, torch::kUInt8));
        current_stream().unwrap().synchronize();  // acc is a host buffer of this call
    }

   private:
    static void copy(void* dst, const void* src, size_t n) {
        dev_view(dst, (int64_t)n, torch::kUInt8).copy_(dev_view(const_cast<void*>(src), (int64_t)n, torch::kUInt8));
    }
    // A step makes three calls in a fixed order (splats all-to-all, image all-gather, gradient
    // all-to-all): call k % 3 keeps its delivery for replay.  Every copy and event is on the
    // stream the step passed (its main stream, or the side stream of the overlapped all-gather).
    template <class F>
    void deliver(hipStream_t s, const void* send, void* recv, size_t total, bool always, F&& from_peer) {
        const int k = (int)(calls_++ % 3);
        const Stream cs = s ? c10::hip::getStreamFromExternalMasqueradingAsCUDA(s, c10::hip::current_device())
                            : current_stream();
        StreamGuard on(cs.unwrap());
        if (replay_) {
            if (replay_copies_ || always) copy(recv, snap_[k].data_ptr(), total);
            return;
        }
        ready_.record(cs.unwrap());
        g_->pub_[rank_] = {send, &ready_};
        g_->barrier();  // every rank's send buffer is published
        for (int p = 0; p < g_->world(); ++p) {
            g_->pub_[p].ev->block(cs.unwrap());
            from_peer(p, static_cast<const char*>(g_->pub_[p].ptr));
        }
        done_.record(cs.unwrap());
        g_->fin_[rank_] = &done_;
        g_->barrier();  // every rank has issued its copies (pub_ may be reused after the next barrier)
        for (int p = 0; p < g_->world(); ++p) g_->fin_[p]->block(cs.unwrap());  // peers done reading my send
        g_->barrier();  // fin_ read by everyone
        if ((int)snap_.size() <= k) snap_.resize(k + 1);
        if (!snap_[k].defined() || (size_t)snap_[k].numel() != total)
            snap_[k] = torch::empty({(int64_t)total}, torch::TensorOptions().dtype(torch::kUInt8).device(
                                                           torch::kCUDA, c10::hip::current_device()));
        copy(snap_[k].data_ptr(), recv, total);
    }
    std::shared_ptr<LocalGroup> g_;
    int rank_;
    bool replay_ = false, replay_copies_ = true;
    int64_t calls_ = 0;
    c10::Event ready_{c10::DeviceType::CUDA}, done_{c10::DeviceType::CUDA};
    std::vector<torch::Tensor> snap_;
};

template <class F>
void run_threads(const std::vector<ShardStep*>& steps, F&& body) {
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(steps.size());
    const c10::Device dev(c10::DeviceType::CUDA, c10::hip::current_device());
    for (size_t r = 0; r < steps.size(); ++r)
        th.emplace_back([&, r] {
            try {
                c10::DeviceGuard g(dev);
                body(*steps[r]);
            } catch (...) {
                err[r] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}

// Fixed-address arena behind one gsr_alloc_fn role: the i-th request of a step gets slot i,
// grown only when a request is larger (never during a captured step: capacities are fixed).
struct Arena {
    torch::Device dev;
    std::vector<torch::Tensor> slots;
    size_t next = 0;
    bool frozen = false;
    static void* cb(void* ctx, size_t bytes) {
        auto* a = static_cast<Arena*>(ctx);
        const size_t i = a->next++;
        if (i == a->slots.size()) {
            if (a->frozen) return nullptr;
            a->slots.push_back(torch::empty({(int64_t)std::max<size_t>(bytes, 16)},
                                            torch::TensorOptions().dtype(torch::kUInt8).device(a->dev)));
        } else if ((size_t)a->slots[i].numel() < bytes) {
            if (a->frozen) return nullptr;
            a->slots[i] = torch::empty({(int64_t)bytes}, torch::TensorOptions().dtype(torch::kUInt8).device(a->dev));
        }
        return a->slots[i].data_ptr();
    }
};

}  // namespace

std::vector<uint8_t> rccl_unique_id() {
    std::vector<uint8_t> out(GSR_COMM_ID_BYTES);
    detail::check(gsr_comm_unique_id(out.data()), "gsr_comm_unique_id");
    return out;
}

std::unique_ptr<Exchange> rccl_exchange(const std::vector<uint8_t>& unique_id, int rank, int world) {
    return std::make_unique<RcclExchange>(unique_id, rank, world);
}

std::unique_ptr<Exchange> rccl_exchange(c10d::Store& store, int rank, int world) {
    std::vector<uint8_t> id;
    if (rank == 0) {
        id = rccl_unique_id();
        store.set("gsr/rccl_id", id);
    } else {
        id = store.get("gsr/rccl_id");
    }
    return rccl_exchange(id, rank, world);
}

std::unique_ptr<Exchange> store_exchange(std::shared_ptr<c10d::Store> store, int rank, int world) {
    return std::make_unique<StoreExchange>(std::move(store), rank, world);
}

std::shared_ptr<LocalGroup> local_group(int world) {
    if (world < 1 || world > kMaxLocalRanks) throw std::invalid_argument("local group: 1..16 ranks");
    return std::make_shared<LocalGroup>(world);
}
std::unique_ptr<Exchange> local_exchange(std::shared_ptr<LocalGroup> group, int rank) {
    return std::make_unique<LocalExchange>(std::move(group), rank);
}
void local_exchange_set_replay(Exchange& ex, bool on, bool copies) {
    auto* l = dynamic_cast<LocalExchange*>(&ex);
    if (!l) throw std::invalid_argument("not a local exchange");
    l->set_replay(on, copies);
}
void run_ranks_plan(const std::vector<ShardStep*>& steps) {
    run_threads(steps, [](ShardStep& s) { s.plan(); });
}
void run_ranks_steps(const std::vector<ShardStep*>& steps, const torch::Tensor& dpix, int n) {
    run_threads(steps, [&](ShardStep& s) {
        for (int i = 0; i < n; ++i) s.step(dpix);
        s.check();
    });
}

// ---- partition: the same arithmetic as bands.py ----
std::pair<int64_t, int64_t> gaussian_shard(int64_t P, int world, int rank) {
    const int64_t S = (P + world - 1) / world;
    return {std::min<int64_t>(rank * S, P), std::min<int64_t>((int64_t)(rank + 1) * S, P)};
}

std::vector<int> equal_bands(int grid_y, int world) {
    std::vector<int> r(world + 1);
    for (int i = 0; i <= world; ++i) r[i] = (int)((int64_t)i * grid_y / world);
    return r;
}

std::vector<int> balance_bands(const std::vector<int64_t>& c, int world) {
    const int gy = (int)c.size();
    if (world > gy) throw std::invalid_argument("balance_bands: more bands than tile rows");
    std::vector<double> pre(gy + 1, 0.0);
    for (int i = 0; i < gy; ++i) pre[i + 1] = pre[i] + (double)c[i];
    const double total = pre[gy];
    if (total <= 0) return equal_bands(gy, world);
    std::vector<int> rows{0};
    for (int k = 1; k < world; ++k) {
        const double t = k * total / world;
        int y = 0;
        double best = std::fabs(pre[0] - t);
        for (int i = 1; i <= gy; ++i)  // first index of the minimum, as numpy.argmin
            if (std::fabs(pre[i] - t) < best) best = std::fabs(pre[i] - t), y = i;
        y = std::max(y, rows.back() + 1);
        y = std::min(y, gy - (world - k));
        rows.push_back(y);
    }
    rows.push_back(gy);
    return rows;
}

StatsPlan plan_from_stats(const std::vector<int64_t>& inst, const std::vector<std::vector<int64_t>>& starts,
                          const std::vector<std::vector<int64_t>>& ends, int world) {
    const int gy = (int)inst.size();
    StatsPlan sp;
    sp.rows = balance_bands(inst, world);
    sp.band_k.assign(world, 0);
    for (int b = 0; b < world; ++b)
        for (int y = sp.rows[b]; y < sp.rows[b + 1]; ++y) sp.band_k[b] += inst[y];
    for (size_t s = 0; s < starts.size(); ++s) {
        std::vector<int64_t> ps(gy + 1, 0), pe(gy + 1, 0);  // prefix sums of starts / ends
        for (int y = 0; y < gy; ++y) ps[y + 1] = ps[y] + starts[s][y], pe[y + 1] = pe[y] + ends[s][y];
        for (int b = 0; b < world; ++b)
            sp.max_splats = std::max(sp.max_splats, ps[sp.rows[b + 1]] - pe[sp.rows[b]]);
    }
    return sp;
}

ShardOverflowError::ShardOverflowError(int64_t step_, int rank_, std::vector<int64_t> counts_, int pair_cap_,
                                       int64_t band_k_, int capacity_)
    : std::overflow_error([&] {
          std::string s = "multi-GPU step " + std::to_string(step_) + " overflowed on rank " + std::to_string(rank_) +
                          ": splats per band [";
          for (size_t i = 0; i < counts_.size(); ++i) s += (i ? ", " : "") + std::to_string(counts_[i]);
          return s + "] vs pair_cap " + std::to_string(pair_cap_) + ", band instances " + std::to_string(band_k_) +
                 " vs capacity " + std::to_string(capacity_);
      }()),
      step(step_), rank(rank_), counts(std::move(counts_)), pair_cap(pair_cap_), band_k(band_k_),
      capacity(capacity_) {}

// ---- the step ----
// gsr_band_forward takes one ctx for its three allocation roles: ctx = the Pool, one callback
// per role.  Streams, events and the captured graph are libtorch's (no HIP runtime call here).
struct ShardStep::Pool {
    torch::Device dev;
    torch::Tensor send, recv, state, radii, color, g2, back, mine, gathered, image;
    std::map<std::string, torch::Tensor> grads;
    gsr_grads gg{};
    Arena geom{dev}, bin{dev}, img{dev}, scratch{dev};
    gsr_buffers bufs{};
    size_t block_bytes = 0, grad_block = 0, mine_floats = 0, status_off = 0;
    int tall = 0;
    Stream main, side;  // the step's stream (capturable) and the all-gather's
    c10::Event enter{c10::DeviceType::CUDA}, leave{c10::DeviceType::CUDA}, fork{c10::DeviceType::CUDA},
        join{c10::DeviceType::CUDA};
    std::vector<torch::Tensor> ring;  // pinned (world x foot_words) int32 per slot
    std::vector<std::unique_ptr<c10::Event>> ring_ev;
    std::unique_ptr<at::cuda::CUDAGraph> graph;
    const void* graph_dpix = nullptr;
    // capture only once the camera and dL_dpix have been the same for one eager step: a loop that
    // changes the camera every iteration then runs eagerly instead of capturing graphs it never
    // replays
    const void* last_dpix = nullptr;
    int eager_since_change = 0;
    torch::Tensor guard;  // (1,) int32: ranks that overflowed in the last step (device, agreed)
    explicit Pool(torch::Device d)
        : dev(d),
          main(c10::hip::getStreamFromPoolMasqueradingAsCUDA(false, d.index())),
          side(c10::hip::getStreamFromPoolMasqueradingAsCUDA(false, d.index())) {}
    static void* geom_cb(void* c, size_t n) { return Arena::cb(&static_cast<Pool*>(c)->geom, n); }
    static void* bin_cb(void* c, size_t n) { return Arena::cb(&static_cast<Pool*>(c)->bin, n); }
    static void* img_cb(void* c, size_t n) { return Arena::cb(&static_cast<Pool*>(c)->img, n); }
};

static constexpr int kStatusWords = 16;  // per rank: nb header counts, band K (nb <= 15)
// then 3 x grid_y words of row statistics (GSR_FLAG_ROW_SPANS): the footer is foot_words_ long

ShardStep::ShardStep(Exchange& ex, const RasterCamera& cam, const ShardInputs& in, std::array<float, 3> bg,
                     double headroom, bool graph, int lag)
    : ex_(ex), cam_(cam), ccam_(cam.to_c()), in_(in), bg_(bg), headroom_(headroom),
      graph_(graph && ex.capturable()), lag_(std::max(lag, 1)), world_(ex.world()), rank_(ex.rank()) {
    TORCH_CHECK(in.means3D.defined() && in.means3D.is_cuda(), "ShardStep: means3D must be a device tensor");
    TORCH_CHECK(world_ >= 1 && world_ < kStatusWords, "ShardStep: 1..15 ranks");
    P_ = in.means3D.size(0);
    std::tie(g0_, g1_) = gaussian_shard(P_, world_, rank_);
    grid_y_ = (cam.height + GSR_TILE - 1) / GSR_TILE;
    TORCH_CHECK(world_ <= grid_y_, "ShardStep: more ranks than tile rows");
    rows_ = equal_bands(grid_y_, world_);
    foot_words_ = kStatusWords + 3 * grid_y_;
    pool_ = std::make_unique<Pool>(in.means3D.device());
    for (int i = 0; i < lag_ + 2; ++i) {
        pool_->ring.push_back(torch::empty({(int64_t)world_, (int64_t)foot_words_},
                                           torch::TensorOptions().dtype(torch::kInt32).pinned_memory(true)));
        pool_->ring_ev.push_back(std::make_unique<c10::Event>(c10::DeviceType::CUDA));
    }
}

ShardStep::~ShardStep() = default;

bool ShardStep::graph_active() const { return pool_ && pool_->graph != nullptr; }

void ShardStep::drop_graph() {
    pool_->graph.reset();
    pool_->graph_dpix = nullptr;
    pool_->eager_since_change = 0;
}

torch::Tensor ShardStep::overflow_guard() const { return pool_->guard; }

gsr_gaussians ShardStep::shard_struct() const {
    gsr_gaussians g{};
    g.P = (int32_t)(g1_ - g0_);
    g.sh_degree = in_.sh_degree;
    g.scale_modifier = in_.scale_modifier;
    auto row = [&](const torch::Tensor& t) -> const float* {
        if (!t.defined()) return nullptr;
        TORCH_CHECK(t.is_contiguous() && t.scalar_type() == torch::kFloat32 && t.size(0) == P_,
                    "ShardStep: inputs must be contiguous f32 with P rows");
        return t.data_ptr<float>() + g0_ * (t.numel() / std::max<int64_t>(P_, 1));
    };
    g.means3D = row(in_.means3D);
    g.sh_dc = row(in_.sh_dc);
    g.sh_rest = in_.sh_rest.defined() && in_.sh_rest.numel() ? row(in_.sh_rest) : nullptr;
    g.sh_rest_coeffs = g.sh_rest ? (int32_t)(in_.sh_rest.numel() / std::max<int64_t>(P_, 1) / 3) : 0;
    g.colors_precomp = row(in_.colors_precomp);
    g.opacities = row(in_.opacities);
    g.scales = row(in_.scales);
    g.rotations = row(in_.rotations);
    g.cov3D_precomp = row(in_.cov3D_precomp);
    return g;
}

gsr_raster_settings ShardStep::shard_settings() const {
    gsr_raster_settings s{};
    for (int i = 0; i < 3; ++i) s.bg[i] = bg_[i];
    s.tile_y0 = 0;
    s.tile_y1 = INT32_MAX;
    return s;
}

gsr_raster_settings ShardStep::band_settings() const {
    gsr_raster_settings s = shard_settings();
    s.flags = 0;
    s.tile_y0 = rows_[rank_];
    s.tile_y1 = rows_[rank_ + 1];
    s.max_rendered = capacity_;
    return s;
}

void ShardStep::size_buffers() {
    Pool& p = *pool_;
    drop_graph();
    const int nb = world_;
    const auto u8 = torch::TensorOptions().dtype(torch::kUInt8).device(p.dev);
    const auto f32 = torch::TensorOptions().dtype(torch::kFloat32).device(p.dev);
    const int64_t Ps = g1_ - g0_;
    p.block_bytes = gsr_exchange_block_bytes(pair_cap_);
    p.grad_block = (size_t)pair_cap_ * GSR_SPLAT_GRAD_BYTES;
    p.send = torch::empty({(int64_t)(nb * p.block_bytes)}, u8);
    p.recv = torch::empty({(int64_t)(nb * p.block_bytes)}, u8);
    p.state = torch::empty({(int64_t)gsr_shard_state_bytes((int32_t)Ps, nb, pair_cap_)}, u8);
    p.radii = torch::empty({Ps}, f32.dtype(torch::kInt32));
    p.color = torch::zeros({3, cam_.height, cam_.width}, f32);
    p.g2 = torch::empty({(int64_t)nb * pair_cap_, GSR_GRAD2D_STRIDE}, f32);
    p.back = torch::empty({(int64_t)(nb * p.grad_block)}, u8);
    int tall = 1;
    for (int r = 0; r < world_; ++r) {
        const int a = std::min(rows_[r] * GSR_TILE, cam_.height), b = std::min(rows_[r + 1] * GSR_TILE, cam_.height);
        tall = std::max(tall, b - a);
    }
    p.tall = tall;
    p.status_off = (size_t)3 * tall * cam_.width;
    p.mine_floats = p.status_off + foot_words_;
    p.mine = torch::zeros({(int64_t)p.mine_floats}, f32);
    p.gathered = torch::empty({(int64_t)world_, (int64_t)p.mine_floats}, f32);
    p.image = torch::empty({3, cam_.height, cam_.width}, f32);
    p.guard = torch::zeros({1}, f32.dtype(torch::kInt32));
    auto e = [&](std::initializer_list<int64_t> sh) { return torch::empty(sh, f32); };
    p.grads.clear();
    p.grads["means2D"] = e({Ps, 3});
    p.grads["conic"] = e({Ps, 3});
    p.grads["opacities"] = e({Ps, 1});
    p.grads["means3D"] = e({Ps, 3});
    if (in_.colors_precomp.defined()) {
        p.grads["colors"] = e({Ps, 3});
    } else {
        p.grads["sh_dc"] = e({Ps, 1, 3});
        const gsr_gaussians g = shard_struct();
        if (g.sh_rest) p.grads["sh_rest"] = e({Ps, g.sh_rest_coeffs, 3});
    }
    if (in_.cov3D_precomp.defined()) {
        p.grads["cov3D"] = e({Ps, 6});
    } else {
        p.grads["scales"] = e({Ps, 3});
        p.grads["rotations"] = e({Ps, 4});
    }
    auto ptr = [&](const char* k) -> float* {
        auto it = p.grads.find(k);
        return it == p.grads.end() ? nullptr : it->second.data_ptr<float>();
    };
    p.gg = gsr_grads{};
    p.gg.dL_dmeans2D = ptr("means2D");
    p.gg.dL_dconic = ptr("conic");
    p.gg.dL_dopacity = ptr("opacities");
    p.gg.dL_dcolors = ptr("colors");
    p.gg.dL_dmeans3D = ptr("means3D");
    p.gg.dL_dsh_dc = ptr("sh_dc");
    p.gg.dL_dsh_rest = ptr("sh_rest");
    p.gg.dL_dscales = ptr("scales");
    p.gg.dL_drotations = ptr("rotations");
    p.gg.dL_dcov3D = ptr("cov3D");
    for (Arena* a : {&p.geom, &p.bin, &p.img, &p.scratch}) {
        a->slots.clear();
        a->frozen = false;
    }
}

void ShardStep::plan() {
    const Stream cs = current_stream();
    const hipStream_t s = cs.stream();
    const gsr_gaussians g = shard_struct();
    const gsr_raster_settings rs = shard_settings();
    auto i32 = torch::TensorOptions().dtype(torch::kInt32).device(pool_->dev);
    const int nb = world_;
    rows_ = equal_bands(grid_y_, world_);
    std::vector<int32_t> rows32(rows_.begin(), rows_.end());
    // probe 1: the shard's per-tile-row instance histogram (pair_cap 0: headers only)
    auto hist = torch::zeros({grid_y_}, i32);
    auto send0 = torch::empty({(int64_t)(nb * gsr_exchange_block_bytes(0))}, i32.dtype(torch::kUInt8));
    auto state0 = torch::empty({(int64_t)gsr_shard_state_bytes(g.P, nb, 0)}, i32.dtype(torch::kUInt8));
    auto radii0 = torch::empty({(int64_t)std::max(g.P, 1)}, i32);
    detail::check(gsr_shard_forward(&ccam_, &g, &rs, nb, rows32.data(), 0, send0.data_ptr(), radii0.data_ptr<int32_t>(),
                                    state0.data_ptr(), reinterpret_cast<uint32_t*>(hist.data_ptr<int32_t>()), s),
                  "gsr_shard_forward (probe)");
    auto hist64 = hist.to(torch::kInt64).bitwise_and(0xFFFFFFFFLL).contiguous();  // u32 counts, widened
    ex_.all_reduce_i64(hist64.data_ptr<int64_t>(), (size_t)grid_y_, false, s);
    auto hc = hist64.cpu();
    std::vector<int64_t> counts(hc.data_ptr<int64_t>(), hc.data_ptr<int64_t>() + grid_y_);
    rows_ = balance_bands(counts, world_);
    rows32.assign(rows_.begin(), rows_.end());
    // probe 2: splats per (shard, band) with the balanced cuts
    detail::check(gsr_shard_forward(&ccam_, &g, &rs, nb, rows32.data(), 0, send0.data_ptr(), radii0.data_ptr<int32_t>(),
                                    state0.data_ptr(), nullptr, s),
                  "gsr_shard_forward (probe)");
    const int64_t bb0 = (int64_t)gsr_exchange_block_bytes(0);
    auto heads = send0.view(torch::kInt32).view({nb, bb0 / 4}).select(1, 0).to(torch::kInt64);
    heads = heads.bitwise_and(0xFFFFFFFFLL).max().reshape({1}).contiguous();
    ex_.all_reduce_i64(heads.data_ptr<int64_t>(), 1, true, s);
    const int64_t pc = heads.cpu().item<int64_t>();
    pair_cap_ = (int)round_up((int64_t)std::ceil(std::max<int64_t>(pc, 1) * headroom_));
    band_k_.assign(world_, 0);
    for (int b = 0; b < world_; ++b)
        for (int y = rows_[b]; y < rows_[b + 1]; ++y) band_k_[b] += counts[y];
    const int64_t kmax = *std::max_element(band_k_.begin(), band_k_.end());
    const int64_t cap = round_up((int64_t)std::ceil(std::max<int64_t>(kmax, 1) * headroom_));
    if (cap >= INT32_MAX || (int64_t)pair_cap_ * world_ >= INT32_MAX)
        throw std::overflow_error("ShardStep: band capacity / pair_cap exceed int32: use more ranks");
    capacity_ = (int)cap;
    pending_.clear();
    size_buffers();
}

void ShardStep::set_pair_cap(int pair_cap) {
    pair_cap_ = pair_cap;
    size_buffers();
}

void ShardStep::set_camera(const RasterCamera& cam) {
    TORCH_CHECK(cam.width == cam_.width && cam.height == cam_.height,
                "ShardStep::set_camera: the image size must stay the plan's");
    cam_ = cam;
    ccam_ = cam.to_c();
    drop_graph();  // the captured launches hold the old camera's values
    for (Arena* a : {&pool_->geom, &pool_->bin, &pool_->img, &pool_->scratch}) a->frozen = false;
}

void ShardStep::set_rebalance_every(int m) {
    TORCH_CHECK(m >= 0, "ShardStep: rebalance_every must be >= 0");
    rebalance_every_ = m;
}

// One step's work on the current stream (= the Pool's main stream, set by step()).  Called
// eagerly, or once under stream capture to record the graph that later steps replay.
void ShardStep::run(const torch::Tensor& dpix) {
    Pool& p = *pool_;
    const hipStream_t s = p.main.stream();
    const int nb = world_;
    const gsr_gaussians g = shard_struct();
    const gsr_raster_settings rs = shard_settings(), bs = band_settings();
    std::vector<int32_t> rows32(rows_.begin(), rows_.end());
    for (Arena* a : {&p.geom, &p.bin, &p.img, &p.scratch}) a->next = 0;
    // 1. F1 on the shard + splat packing; with live re-planning the shard's row statistics
    //    (instances per tile row, rect start / end rows) go straight into this rank's status
    //    footer (zeroed by the previous step's gsr_gather_finish, or by size_buffers)
    float* const stats = p.mine.data_ptr<float>() + p.status_off + kStatusWords;
    gsr_raster_settings rss = rs;
    if (live_) rss.flags |= GSR_FLAG_ROW_SPANS;
    detail::check(gsr_shard_forward(&ccam_, &g, &rss, nb, rows32.data(), pair_cap_, p.send.data_ptr(),
                                    g.P ? p.radii.data_ptr<int32_t>() : nullptr, p.state.data_ptr(),
                                    live_ ? reinterpret_cast<uint32_t*>(stats) : nullptr, s),
                  "gsr_shard_forward");
    // 2. splats -> bands
    ex_.all_to_all(p.send.data_ptr(), p.recv.data_ptr(), p.block_bytes, s);
    // 3. F2..F6 on this band
    detail::check(gsr_band_forward(&ccam_, &bs, nb, pair_cap_, p.recv.data_ptr(), p.color.data_ptr<float>(),
                                   Pool::geom_cb, Pool::bin_cb, Pool::img_cb, &p, &p.bufs, s),
                  "gsr_band_forward");
    // 4. the band's pixels + status footer (send-header counts, band K) -> all-gather on the side
    //    stream, overlapping B1 (one launch: gsr_band_publish)
    detail::check(gsr_band_publish(&ccam_, &bs, p.tall, p.color.data_ptr<float>(), nb, p.send.data_ptr(), pair_cap_,
                                   &p.bufs, p.mine.data_ptr<float>(), (int64_t)p.status_off, s),
                  "gsr_band_publish");
    const bool overlap = ex_.capturable();
    if (overlap) {
        p.fork.record(p.main.unwrap());
        p.fork.block(p.side.unwrap());
    }
    ex_.all_gather(p.mine.data_ptr<float>(), p.gathered.data_ptr<float>(), p.mine_floats * sizeof(float),
                   overlap ? p.side.stream() : s);
    if (overlap) p.join.record(p.side.unwrap());
    // 5. B1 on the band, per-splat 2D gradients in the received slot layout
    detail::check(gsr_band_backward(&ccam_, &bs, nb, pair_cap_, &p.bufs, dpix.data_ptr<float>(), Arena::cb,
                                    &p.scratch, p.g2.data_ptr<float>(), s),
                  "gsr_band_backward");
    // 6. gradients -> owning shards
    ex_.all_to_all(p.g2.data_ptr<float>(), p.back.data_ptr(), p.grad_block, s);
    // 7. band-order sums + B2 on the shard
    detail::check(gsr_shard_backward(&ccam_, &g, &rs, nb, rows32.data(), pair_cap_, p.state.data_ptr(),
                                     p.back.data_ptr(), &p.gg, s),
                  "gsr_shard_backward");
    // 8. join the all-gather; one launch (gsr_gather_finish) unpacks the bands into the full image,
    //    writes the agreed overflow word (the number of ranks whose splat counts or band K exceeded
    //    the plan's capacities in THIS step, the same on every rank; the optimizer guard of a
    //    training loop, no host wait) and clears this rank's row statistics for the next step
    if (overlap) p.join.block(p.main.unwrap());
    detail::check(gsr_gather_finish(&ccam_, world_, rows32.data(), p.tall, p.gathered.data_ptr<float>(),
                                    (int64_t)p.mine_floats, (int64_t)p.status_off, pair_cap_, capacity_,
                                    p.image.data_ptr<float>(), p.guard.data_ptr<int32_t>(), stats,
                                    live_ ? 3 * (int64_t)grid_y_ : 0, s),
                  "gsr_gather_finish");
}

void ShardStep::set_graph(bool on) {
    const bool g = on && ex_.capturable();
    if (g == graph_) return;
    graph_ = g;
    drop_graph();
}

void ShardStep::set_live_replan(bool on) {
    if (on == live_) return;
    live_ = on;
    drop_graph();  // the captured pack collects the statistics or not
}

void ShardStep::push_status() {
    Pool& p = *pool_;
    // poll(false) at the start of every step leaves at most lag_ older entries pending
    TORCH_CHECK(pending_.size() < p.ring.size(), "ShardStep: overflow ring full");
    const int slot = ring_next_;
    ring_next_ = (ring_next_ + 1) % (int)p.ring.size();
    // (a hipMemcpy2DAsync straight into the pinned slot would skip the gather into a contiguous
    // temporary, but it makes this object reference the HIP runtime directly, which the C++
    // executables must not link a second copy of: _build._exe_flags)
    auto st = p.gathered.narrow(1, (int64_t)p.status_off, foot_words_).contiguous().view(torch::kInt32);
    p.ring[slot].copy_(st, /*non_blocking=*/true);
    p.ring_ev[slot]->record(p.main.unwrap());
    pending_.push_back({steps_, slot, pair_cap_, capacity_, live_});
}

void ShardStep::poll(bool wait_all) {
    // the step exactly lag_ back (and anything older) is checked on every rank at the same call
    while (!pending_.empty() && (wait_all || pending_.front().step <= steps_ - lag_)) {
        const Pending q = pending_.front();
        pool_->ring_ev[q.slot]->synchronize();
        pending_.erase(pending_.begin());
        const int32_t* st = pool_->ring[q.slot].data_ptr<int32_t>();
        for (int r = 0; r < world_; ++r) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(st + r * foot_words_);
            std::vector<int64_t> counts(w, w + world_);
            const int64_t k = w[world_];
            if (*std::max_element(counts.begin(), counts.end()) > q.pair_cap || k > q.capacity) {
                pending_.clear();
                throw ShardOverflowError(q.step, r, counts, q.pair_cap, k, q.capacity);
            }
        }
        if (q.stats) {  // a step without statistics (live re-planning off) leaves the last ones
            last_stats_.assign(st, st + (size_t)world_ * foot_words_);
            last_stats_step_ = q.step;
        }
    }
}

void ShardStep::replan_live() {
    if (last_stats_step_ < 0 || last_stats_step_ == stats_used_step_) return;
    stats_used_step_ = last_stats_step_;
    const int gy = grid_y_;
    std::vector<int64_t> inst(gy, 0);
    std::vector<std::vector<int64_t>> starts(world_, std::vector<int64_t>(gy)), ends = starts;
    for (int r = 0; r < world_; ++r) {
        const uint32_t* f = reinterpret_cast<const uint32_t*>(last_stats_.data() + (size_t)r * foot_words_) + kStatusWords;
        for (int y = 0; y < gy; ++y) {
            inst[y] += f[y];
            starts[r][y] = f[gy + y];
            ends[r][y] = f[2 * gy + y];
        }
    }
    const StatsPlan sp = plan_from_stats(inst, starts, ends, world_);
    const int64_t kmax = *std::max_element(sp.band_k.begin(), sp.band_k.end());
    const int64_t pc_need = std::max<int64_t>(sp.max_splats, 1), cap_need = std::max<int64_t>(kmax, 1);
    const bool short_caps = pc_need > pair_cap_ || cap_need > capacity_;
    const bool fat_caps = pair_cap_ > 2 * round_up((int64_t)std::ceil(pc_need * headroom_)) ||
                          capacity_ > 2 * round_up((int64_t)std::ceil(cap_need * headroom_));
    if (sp.rows == rows_ && !short_caps && !fat_caps) return;
    const int64_t pc = round_up((int64_t)std::ceil(pc_need * headroom_));
    const int64_t cap = round_up((int64_t)std::ceil(cap_need * headroom_));
    if (cap >= INT32_MAX || pc * world_ >= INT32_MAX)
        throw std::overflow_error("ShardStep: band capacity / pair_cap exceed int32: use more ranks");
    rows_ = sp.rows;
    band_k_ = sp.band_k;
    pair_cap_ = (int)pc;
    capacity_ = (int)cap;
    size_buffers();  // new cuts / capacities: buffers re-sized, the captured graph dropped
    ++live_replans_;
}

void ShardStep::check() { poll(true); }

int64_t ShardStep::band_num_rendered() const {
    void* k = const_cast<void*>(gsr_view(&ccam_, world_ * pair_cap_, &pool_->bufs, GSR_VIEW_COUNTS));
    TORCH_CHECK(k != nullptr && steps_ > 0, "ShardStep: no step yet");
    return (int64_t)(uint32_t)dev_view(k, 1, torch::kInt32).item<int32_t>();
}

ShardStep::Result ShardStep::step(const torch::Tensor& dL_dpix) {
    TORCH_CHECK(pair_cap_ > 0 && capacity_ > 0, "ShardStep: call plan() first");
    TORCH_CHECK(dL_dpix.is_cuda() && dL_dpix.scalar_type() == torch::kFloat32 && dL_dpix.is_contiguous() &&
                    dL_dpix.numel() == (int64_t)3 * cam_.height * cam_.width,
                "ShardStep: dL_dpix must be a contiguous (3,H,W) f32 device tensor");
    if (rebalance_every_ > 0 && steps_ > 0 && steps_ % rebalance_every_ == 0) {
        poll(true);  // the old plan's pending checks first
        plan();      // drops the graph; this step runs eagerly and captures again
        ++replans_;
    }
    poll(false);
    if (live_) replan_live();
    Pool& p = *pool_;
    // the step runs on its own stream (capturable), ordered after / before the caller's
    const Stream caller = current_stream();
    p.enter.record(caller.unwrap());
    p.enter.block(p.main.unwrap());
    {
        StreamGuard guard(p.main.unwrap());
        if (graph_ && p.graph && p.graph_dpix == dL_dpix.data_ptr()) {
            p.graph->replay();
        } else {
            run(dL_dpix);  // this step's result, eagerly
            const bool stable = p.eager_since_change > 0 && p.last_dpix == dL_dpix.data_ptr();
            p.last_dpix = dL_dpix.data_ptr();
            ++p.eager_since_change;
            if (graph_ && stable) {
                // every arena slot now exists: capture the same calls on the same buffers
                drop_graph();
                for (Arena* a : {&p.geom, &p.bin, &p.img, &p.scratch}) a->frozen = true;
                p.main.unwrap().synchronize();
                p.graph = std::make_unique<at::cuda::CUDAGraph>();
                p.graph->capture_begin({0, 0}, hipStreamCaptureModeRelaxed);
                try {
                    run(dL_dpix);
                } catch (...) {
                    try {
                        p.graph->capture_end();
                    } catch (...) {
                    }
                    drop_graph();
                    throw;
                }
                p.graph->capture_end();
                p.graph_dpix = dL_dpix.data_ptr();
            }
        }
        push_status();
    }
    p.leave.record(p.main.unwrap());
    p.leave.block(caller.unwrap());
    ++steps_;
    return {p.image, p.grads, p.radii};
}

}  // namespace gsr

// ---- Python binding (the benchmark's multi-GPU path; off in the C++ executables) ----
#ifndef GSR_NO_PYBIND
#include <pybind11/stl.h>
#include <torch/extension.h>

namespace gsr {
namespace py = pybind11;
void bind_shard(py::module& m) {
    static py::exception<ShardOverflowError> ovf(m, "ShardOverflowError", PyExc_OverflowError);
    py::register_exception_translator([](std::exception_ptr p) {
        try {
            if (p) std::rethrow_exception(p);
        } catch (const ShardOverflowError& e) {
            py::object cls = py::reinterpret_borrow<py::object>(ovf.ptr());
            py::object err = cls(e.what());
            err.attr("step") = e.step;
            err.attr("rank") = e.rank;
            err.attr("counts") = e.counts;
            err.attr("pair_cap") = e.pair_cap;
            err.attr("band_k") = e.band_k;
            err.attr("capacity") = e.capacity;
            PyErr_SetObject(ovf.ptr(), err.ptr());
        }
    });
    py::class_<Exchange>(m, "Exchange")
        .def_property_readonly("rank", &Exchange::rank)
        .def_property_readonly("world", &Exchange::world)
        .def_property_readonly("name", &Exchange::name)
        .def_property_readonly("comm_world", &Exchange::comm_world)
        .def_property_readonly("capturable", &Exchange::capturable);
    m.def(
        "plan_from_stats",
        [](const std::vector<int64_t>& inst, const std::vector<std::vector<int64_t>>& starts,
           const std::vector<std::vector<int64_t>>& ends, int world) {
            const StatsPlan sp = plan_from_stats(inst, starts, ends, world);
            return py::make_tuple(sp.rows, sp.max_splats, sp.band_k);
        },
        py::arg("inst"), py::arg("starts"), py::arg("ends"), py::arg("world"));
    m.def("rccl_unique_id", []() {
        auto v = rccl_unique_id();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
    });
    m.def(
        "rccl_exchange",
        [](py::bytes id, int rank, int world) {
            const std::string b = id;
            return rccl_exchange(std::vector<uint8_t>(b.begin(), b.end()), rank, world);
        },
        py::arg("unique_id"), py::arg("rank"), py::arg("world"));
    // host-staged exchange through a torch.distributed Store (e.g. the default group's,
    // torch.distributed.distributed_c10d._get_default_store()): ranks may share a GPU (rehearsal)
    m.def(
        "store_exchange",
        [](const c10::intrusive_ptr<c10d::Store>& store, int rank, int world) {
            std::shared_ptr<c10d::Store> s(store.get(), [keep = store](c10d::Store*) mutable { keep.reset(); });
            py::gil_scoped_release nogil;  // the join waits for the other ranks
            return store_exchange(std::move(s), rank, world);
        },
        py::arg("store"), py::arg("rank"), py::arg("world"));
    py::class_<LocalGroup, std::shared_ptr<LocalGroup>>(m, "LocalGroup")
        .def(py::init([](int world) { return local_group(world); }), py::arg("world"))
        .def_property_readonly("world", &LocalGroup::world);
    m.def("local_exchange", &local_exchange, py::arg("group"), py::arg("rank"), py::keep_alive<0, 1>());
    m.def("local_exchange_set_replay", &local_exchange_set_replay, py::arg("exchange"), py::arg("on"),
          py::arg("copies") = true);
    m.def(
        "run_ranks_plan", [](const std::vector<ShardStep*>& steps) { run_ranks_plan(steps); }, py::arg("steps"),
        py::call_guard<py::gil_scoped_release>());
    m.def(
        "run_ranks_steps",
        [](const std::vector<ShardStep*>& steps, const torch::Tensor& dpix, int n) { run_ranks_steps(steps, dpix, n); },
        py::arg("steps"), py::arg("dL_dpix"), py::arg("n"), py::call_guard<py::gil_scoped_release>());
    py::class_<ShardStep>(m, "ShardStep")
        .def(py::init([](Exchange& ex, const RasterCamera& cam, py::dict inputs, int sh_degree,
                         std::array<float, 3> bg, double headroom, bool graph, int lag) {
                 ShardInputs in;
                 auto get = [&](const char* k) {
                     return inputs.contains(k) && !inputs[k].is_none() ? inputs[k].cast<torch::Tensor>()
                                                                        : torch::Tensor();
                 };
                 in.means3D = get("means3D");
                 in.opacities = get("opacities");
                 in.scales = get("scales");
                 in.rotations = get("rotations");
                 in.sh_dc = get("sh_dc");
                 in.sh_rest = get("sh_rest");
                 in.colors_precomp = get("colors_precomp");
                 in.cov3D_precomp = get("cov3D_precomp");
                 in.sh_degree = sh_degree;
                 return std::make_unique<ShardStep>(ex, cam, in, bg, headroom, graph, lag);
             }),
             py::arg("exchange"), py::arg("cam"), py::arg("inputs"), py::arg("sh_degree"),
             py::arg("bg") = std::array<float, 3>{0.f, 0.f, 0.f}, py::arg("headroom") = 1.25,
             py::arg("graph") = true, py::arg("lag") = 2, py::keep_alive<1, 2>())
        .def("plan", &ShardStep::plan, py::call_guard<py::gil_scoped_release>())
        .def(
            "step",
            [](ShardStep& s, const torch::Tensor& dpix) {
                ShardStep::Result r;
                {
                    py::gil_scoped_release nogil;
                    r = s.step(dpix);
                }
                return py::make_tuple(r.image, r.grads, r.radii);
            },
            py::arg("dL_dpix"))
        .def("check", &ShardStep::check, py::call_guard<py::gil_scoped_release>())
        .def("set_pair_cap", &ShardStep::set_pair_cap)
        .def("set_camera", &ShardStep::set_camera, py::arg("cam"))
        .def("set_rebalance_every", &ShardStep::set_rebalance_every, py::arg("m"))
        .def_property_readonly("replans", &ShardStep::replans)
        .def("set_live_replan", &ShardStep::set_live_replan, py::arg("on"))
        .def("set_graph", &ShardStep::set_graph, py::arg("on"))
        .def_property_readonly("live_replans", &ShardStep::live_replans)
        .def("band_num_rendered", &ShardStep::band_num_rendered)
        .def_property_readonly("rows", &ShardStep::rows)
        .def_property_readonly("pair_cap", &ShardStep::pair_cap)
        .def_property_readonly("capacity", &ShardStep::capacity)
        .def_property_readonly("band_instances", &ShardStep::band_instances)
        .def_property_readonly("g0", &ShardStep::g0)
        .def_property_readonly("g1", &ShardStep::g1)
        .def_property_readonly("exchange_world", &ShardStep::exchange_world)
        .def_property_readonly("overflow_guard", &ShardStep::overflow_guard)
        .def_property_readonly("exchange_name", &ShardStep::exchange_name)
        .def_property_readonly("graph_active", &ShardStep::graph_active)
        .def_property_readonly("steps", &ShardStep::steps);
}
}  // namespace gsr
#endif  // GSR_NO_PYBIND

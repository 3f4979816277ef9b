// gsr_shard.h -- the multi-GPU step in C++ (SURVEY §8e "scaling version"): the
// native twin of bands.ShardStep, so that a C++ training loop (src/utils/train_utils.cpp:97-146,
// src/train.cpp:12-47 -- host code stays C++) runs the sharded path without Python.
//
// Rank r of N owns the Gaussian shard [g0, g1) and the band of tile rows [rows[r], rows[r+1]).
// One step on the rank's stream:
//   gsr_shard_forward -> all-to-all of the splat blocks -> gsr_band_forward
//   -> all-gather of the band images (on a second stream, overlapping B1)
//   -> gsr_band_backward -> all-to-all of the 2D-gradient rows back -> gsr_shard_backward.
// The collectives go through an `Exchange`: RCCL over xGMI (grouped ncclSend / ncclRecv for the
// all-to-alls, ncclAllGather for the bands) on the GPU box, or a host-staged exchange through a
// c10d::Store for ranks that share one GPU (the two-process test; RCCL refuses two ranks on one
// device).  The step is sync-free (fixed capacities from plan(); K stays on the device), so with
// an RCCL exchange it is captured once into a hipGraph and replayed: one graph launch per step.
//
// Overflow agreement: each rank's send-header counts and band K ride in a status footer of its
// band image, so the all-gather hands every rank the status of ALL ranks; the gathered footers
// are copied to pinned memory after the step and checked exactly `lag` steps later (waiting on
// that step's event if needed).  Every rank therefore sees the same counts at the same step and
// raises ShardOverflowError together -- no rank is left blocked in a collective its peers no
// longer join.
#pragma once
#include <hip/hip_runtime.h>  // hipStream_t only: the step itself uses libtorch streams / graphs
#include <torch/torch.h>

#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "gsr/gsr.h"
#include "gsr_render.h"

namespace c10d {
class Store;
}

namespace gsr {

// ---- transport -----------------------------------------------------------------------------
class Exchange {
   public:
    virtual ~Exchange() = default;
    virtual int rank() const = 0;
    virtual int world() const = 0;
    virtual bool capturable() const = 0;  // may be recorded into a hipGraph
    virtual const char* name() const = 0;
    // the transport's own count of ranks (RCCL: ncclCommCount), for reports
    virtual int comm_world() const { return world(); }
    // block b of `send` (block_bytes each) -> rank b; block s of `recv` <- rank s
    virtual void all_to_all(const void* send, void* recv, size_t block_bytes, hipStream_t s) = 0;
    // `bytes` from every rank into recv, rank-major
    virtual void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
    // in place over ranks (setup only)
    virtual void all_reduce_i64(int64_t* buf, size_t n, bool max, hipStream_t s) = 0;
};

// RCCL: rank 0 makes the unique id, the caller broadcasts it (torch.distributed, a store, ...).
std::vector<uint8_t> rccl_unique_id();
std::unique_ptr<Exchange> rccl_exchange(const std::vector<uint8_t>& unique_id, int rank, int world);
// RCCL with the id passed through a c10d::Store (key "gsr/rccl_id").
std::unique_ptr<Exchange> rccl_exchange(c10d::Store& store, int rank, int world);
// Host-staged through a c10d::Store (device -> host -> store -> host -> device); not capturable.
std::unique_ptr<Exchange> store_exchange(std::shared_ptr<c10d::Store> store, int rank, int world);

// In-process rank group (one-GPU rehearsal of the N-rank step, scripts/band_sim.py --cpp): every
// rank's ShardStep runs in its own host thread on the same device, and the collectives are
// device-to-device copies between the ranks' own buffers, ordered by events and host barriers.
// After a live step each exchange keeps what it delivered (recv blocks, gathered rows, gradient
// blocks); in replay mode it copies those instead of waiting for peers, so ONE rank's whole C++
// step (glue, graph replay and exchange-sized copies included) can be timed alone on the GPU.
class LocalGroup;
std::shared_ptr<LocalGroup> local_group(int world);
std::unique_ptr<Exchange> local_exchange(std::shared_ptr<LocalGroup> group, int rank);
// replay: copy the last live step's deliveries (copies) or move nothing (the receive buffers
// still hold them); throws unless ex is a local exchange
void local_exchange_set_replay(Exchange& ex, bool on, bool copies = true);
class ShardStep;
// steps[r].plan() / steps[r].step(dpix) x n in one host thread per rank (exceptions rethrown)
void run_ranks_plan(const std::vector<ShardStep*>& steps);
void run_ranks_steps(const std::vector<ShardStep*>& steps, const torch::Tensor& dpix, int n);

// ---- partition (bands.py) -------------------------------------------------------------------
std::pair<int64_t, int64_t> gaussian_shard(int64_t P, int world, int rank);
std::vector<int> equal_bands(int grid_y, int world);
std::vector<int> balance_bands(const std::vector<int64_t>& row_counts, int world);

// Band cuts and capacities from one step's statistics (GSR_FLAG_ROW_SPANS of every shard, summed
// or per shard): inst[y] = instances in tile row y over all shards; starts[s][y] / ends[s][y] =
// shard s's visible Gaussians whose rect's first / last tile row is y.  The splats shard s sends
// to band [r0, r1) are exactly sum_{y<r1} starts[s][y] - sum_{y<r0} ends[s][y], so the needed
// pair_cap and band capacity (before headroom) follow for any cuts.  Same arithmetic as
// bands.plan_from_stats.
struct StatsPlan {
    std::vector<int> rows;
    int64_t max_splats = 0;  // largest (shard, band) splat count under `rows`
    std::vector<int64_t> band_k;
};
StatsPlan plan_from_stats(const std::vector<int64_t>& inst, const std::vector<std::vector<int64_t>>& starts,
                          const std::vector<std::vector<int64_t>>& ends, int world);

class ShardOverflowError : public std::overflow_error {
   public:
    ShardOverflowError(int64_t step, int rank, std::vector<int64_t> counts, int pair_cap, int64_t band_k,
                       int capacity);
    int64_t step;
    int rank;                     // the (first) rank whose counts exceeded a capacity
    std::vector<int64_t> counts;  // that rank's splats per band
    int pair_cap;
    int64_t band_k;
    int capacity;
};

// The shard's input rows (activated values, as gsr_gaussians): device f32 tensors over ALL P
// Gaussians; the step reads rows [g0, g1) only.  Unused ones undefined.
struct ShardInputs {
    torch::Tensor means3D, opacities, scales, rotations, sh_dc, sh_rest, colors_precomp, cov3D_precomp;
    int sh_degree = 0;
    float scale_modifier = 1.f;
};

class ShardStep {
   public:
    // graph: capture the step into a hipGraph on the first step after plan() (RCCL exchange
    // only; the host-staged one always runs eagerly).  lag: steps between a step and its
    // overflow check (>= 1).  headroom: capacity factor over the probed counts.
    ShardStep(Exchange& ex, const RasterCamera& cam, const ShardInputs& in, std::array<float, 3> bg = {0, 0, 0},
              double headroom = 1.25, bool graph = true, int lag = 2);
    ~ShardStep();
    ShardStep(const ShardStep&) = delete;
    ShardStep& operator=(const ShardStep&) = delete;

    // Probe (synchronous, setup only): balanced band cuts from the summed row histogram, then
    // pair_cap and the band capacity with headroom.  Drops a captured graph.
    void plan();
    struct Result {
        torch::Tensor image;                         // (3,H,W): every band, gathered
        std::map<std::string, torch::Tensor> grads;  // the shard's leaf gradients (rows g0..g1)
        torch::Tensor radii;                         // (g1 - g0) int32
    };
    // One forward + backward; raises ShardOverflowError for the step `lag` earlier if any rank
    // overflowed there.  The returned tensors are the step's own buffers: consume them before
    // the next step().  dL_dpix: (3,H,W) f32 device (its band rows are read).
    Result step(const torch::Tensor& dL_dpix);
    // Check every completed step now (waits); raises like step().
    void check();
    // (1,) int32 device word, written by every step: the number of ranks whose splats or band
    // instances exceeded the plan's capacities in THAT step, from the gathered status footers --
    // the same value on every rank, with no host wait.  Pass it as the guard of the optimizer step
    // (gsr_adam_step_guarded / gsr_densify_stats_guarded with guard_cap 0) so that a truncated
    // step never updates the model, before the lagged check raises.
    torch::Tensor overflow_guard() const;

    const std::vector<int>& rows() const { return rows_; }
    int pair_cap() const { return pair_cap_; }
    int capacity() const { return capacity_; }
    const std::vector<int64_t>& band_instances() const { return band_k_; }
    int64_t g0() const { return g0_; }
    int64_t g1() const { return g1_; }
    // ranks as the exchange's communicator counts them (RCCL: ncclCommCount)
    int exchange_world() const { return ex_.comm_world(); }
    const char* exchange_name() const { return ex_.name(); }
    bool graph_active() const;
    int64_t steps() const { return steps_; }
    // the last step's band instance count K (reads the device counter back: waits)
    int64_t band_num_rendered() const;
    // test hook: force a (smaller) pair capacity after plan()
    void set_pair_cap(int pair_cap);
    // Moving cameras (training, train_utils.cpp:128-145 picks a view per iteration): render from
    // `cam` (same size) from the next step on -- a captured graph is dropped, and a new one is
    // captured only after one eager step with the same camera and dL_dpix (a camera that changes
    // every step runs eagerly, capturing nothing).
    // The cuts and capacities stay the last plan's until a re-plan: with rebalance_every = M > 0,
    // step() re-plans (checks the pending steps, then plan() for the camera in use) before every
    // M-th step; every rank does so at the same step count.
    void set_camera(const RasterCamera& cam);
    void set_rebalance_every(int m);
    int64_t replans() const { return replans_; }
    // Live re-planning (SURVEY §8e "reuse the previous iteration's counts"): every step carries
    // its shard's row statistics (GSR_FLAG_ROW_SPANS) in the status footer of the image
    // all-gather; when step s - lag is checked, every rank computes the cuts and capacities those
    // statistics call for (plan_from_stats, headroom) and, at that same call, adopts them if the
    // cuts moved, a capacity is short, or a capacity is over twice what is needed -- no probe
    // forward, no collective and no host wait beyond the lagged ring.  live_replans() counts them.
    // The statistics are collected only while live re-planning is on (the pack then takes its
    // row-spans form); switching it drops a captured graph.
    void set_live_replan(bool on);
    // Graph capture on / off after construction (on only with a capturable exchange; a local
    // exchange becomes capturable in replay mode).
    void set_graph(bool on);
    int64_t live_replans() const { return live_replans_; }

   private:
    struct Pool;  // buffers (stable addresses across steps: graph-replayable), streams, events, graph
    void run(const torch::Tensor& dpix);
    void push_status();
    void poll(bool wait_all);
    void replan_live();
    gsr_gaussians shard_struct() const;
    gsr_raster_settings shard_settings() const;
    gsr_raster_settings band_settings() const;
    void size_buffers();
    void drop_graph();

    Exchange& ex_;
    RasterCamera cam_;
    gsr_camera ccam_;
    ShardInputs in_;
    std::array<float, 3> bg_;
    double headroom_;
    bool graph_;
    int lag_;
    int world_, rank_;
    int64_t P_ = 0, g0_ = 0, g1_ = 0;
    int grid_y_ = 0;
    std::vector<int> rows_;
    int pair_cap_ = 0, capacity_ = 0;
    std::vector<int64_t> band_k_;
    int64_t steps_ = 0;
    int rebalance_every_ = 0;
    int64_t replans_ = 0;
    bool live_ = false;
    int64_t live_replans_ = 0;
    int foot_words_ = 0;                  // status words + 3 x grid_y row statistics, per rank
    std::vector<int32_t> last_stats_;     // the latest checked step's footers (world x foot_words_)
    int64_t last_stats_step_ = -1, stats_used_step_ = -1;
    std::unique_ptr<Pool> pool_;
    // overflow ring: gathered status footers (pinned), checked `lag_` steps later
    struct Pending {
        int64_t step;
        int slot;
        int pair_cap, capacity;  // the plan the step ran under
        bool stats;              // the step collected row statistics (live re-planning on)
    };
    std::vector<Pending> pending_;
    int ring_next_ = 0;
};

}  // namespace gsr

// gsr_api.cpp -- the C ABI (include/gsr/gsr.h) over the CDNA4 kernels.
//
// Stage order (forward, shipped binning): F1 preprocess -> scan of tiles_touched in gid order
// (a band: compaction of its candidates first) -> ONE device->host read of K -> F3 duplicate
// -> tile-key sort (K keys) -> F5 finalize (tile ranges) -> per-tile depth sort -> F6 blend.
// Backward: B1 blend backward -> gather -> B2 preprocess backward (or B1 -> per-Gaussian grad2d
// for the multi-GPU exchange).
// No persistent allocations; every scratch buffer comes from the caller's callbacks.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "gsr_kernels.h"

using namespace gsr;

namespace {

thread_local std::string g_err;

// A/B selector (bench/ablation only): 0 = three-kernel scan then duplicate, 1 = fused
// look-back scan + duplicate.  Shipped: fused for up to 2^19 ranked Gaussians (a band's
// candidates: 0.030 vs 0.037 ms at 133k), three kernels above (0.084 vs 0.102 ms at 1M: the
// look-back chain over n / 256 blocks dominates).
int scan_variant(int n) {
    const char* e = std::getenv("GSR_SCAN_VARIANT");
    return e ? std::atoi(e) : (n <= (1 << 19) ? 1 : 0);
}

// Binning scheme (A/B, bench/ablation only); all three give the same canonical order.
// Stage sums at 1M/1080p (scripts/ablate.py), whole forward + backward step:
//   1 (shipped, 1.406 ms) = no global depth sort: the instances are emitted in gid order (the
//       scan and F3 read tiles / rects coalesced), a stable LSD sort of the tile keys groups
//       them by tile in gid order, and each tile's slice is sorted by depth alone with a stable
//       LDS radix sort (launch_tile_depth_sort); the gather of B1's partials then also walks
//       the Gaussians in gid order (0.079 vs 0.108 ms);
//   0 (1.464 ms) = global LSD depth sort of the P (or band-candidate) keys before the scan,
//       then the tile-key LSD sort (round-1's first design);
//   2 (1.537 ms) = count binning: F3 counts instances per tile with atomics, one scan gives the
//       ranges, a scatter with returning atomics groups them by tile (unordered), then a
//       bitonic (depth, gid) sort per tile.  The 6.5 M atomics on 8160 hot words cost
//       0.088 ms in F3 and 0.16 ms in the scatter -- more than the two LSD passes they replace.
int bin_variant() {
    const char* e = std::getenv("GSR_BIN_VARIANT");
    return e ? std::atoi(e) : 1;
}

// A/B (bench/ablation only): 1 = binning variant 1 carries each instance's depth key through
// the tile sort so the per-tile sort reads its keys contiguously; 0 (shipped) = the per-tile
// sort gathers depth_key[gid].  Measured at 1M/1080p: carrying costs the tile sort +0.048 ms
// (a third array per pass) and saves the per-tile sort only 0.005 ms -- the random 4-B gathers
// hit L2 / MALL, and that sort is VALU-bound, not gather-bound.
bool carry_depth() {
    const char* e = std::getenv("GSR_CARRY_DEPTH");
    return e ? std::atoi(e) != 0 : false;
}

// A/B (bench/ablation only): 1 = gsr_backward runs the gather and B2 as one kernel when the
// ranking is the identity; 0 (shipped) = two kernels through the grad2d buffer.  Measured at
// 1M/1080p: fused 0.215 ms vs 0.078 + 0.118 ms -- the fused block holds B2's 46 KB of SH
// staging through the latency-bound gather phase (3 blocks per CU instead of 8), which costs
// more than the 96 MB grad2d round trip it saves.
bool fuse_gather() {
    const char* e = std::getenv("GSR_FUSE_GATHER");
    return e ? std::atoi(e) != 0 : false;
}

// Low-latency device->host read of one u32: DMA into a per-thread pinned word, then spin on
// it.  hipStreamSynchronize after a pageable copy measured ~100 us from the end of the scan
// to the next launch (profiles/r01_kernel_stats + trace); the spin wakes within ~µs.
struct PinnedWord {
    static constexpr int kWords = 256;
    volatile uint32_t* p = nullptr;
    PinnedWord() {
        void* q = nullptr;
        if (hipHostMalloc(&q, 4 * kWords, hipHostMallocDefault) == hipSuccess) p = static_cast<volatile uint32_t*>(q);
    }
    ~PinnedWord() {
        if (p) (void)hipHostFree(const_cast<uint32_t*>(p));
    }
};
thread_local PinnedWord g_pinned;

// Reads n <= PinnedWord::kWords consecutive u32 counts (each < 2^31) in two steps: begin_read enqueues one DMA
// into the pinned words (stream-ordered: it lands when the producing kernel is done);
// end_read spins until every word has changed from the sentinel.  Work enqueued between the
// two keeps the GPU busy while the host waits.
int begin_read(const uint32_t* dev, int n, hipStream_t stream) {
    if (!g_pinned.p) return 0;
    for (int i = 0; i < n; ++i) g_pinned.p[i] = 0xFFFFFFFFu;
    return (int)hipMemcpyAsync(const_cast<uint32_t*>(g_pinned.p), dev, sizeof(uint32_t) * n,
                               hipMemcpyDeviceToHost, stream);
}

int end_read(const uint32_t* dev, uint32_t* out, int n, hipStream_t stream) {
    if (!g_pinned.p) {  // no pinned memory: plain copy + stream sync
        if (hipError_t e = hipMemcpyAsync(out, dev, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, stream))
            return (int)e;
        return (int)hipStreamSynchronize(stream);
    }
    auto done = [&] {
        for (int i = 0; i < n; ++i)
            if (g_pinned.p[i] == 0xFFFFFFFFu) return false;
        return true;
    };
    for (long spins = 0; !done(); ++spins) {
        if (spins > (1l << 20) && hipStreamQuery(stream) == hipSuccess) {
            if (!done()) return (int)hipErrorUnknown;  // stream drained, words never written
            break;
        }
        __builtin_ia32_pause();
    }
    for (int i = 0; i < n; ++i) out[i] = g_pinned.p[i];
    return 0;
}

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define GSR_CHECK_HIP(expr, stage)                                                             \
    do {                                                                                       \
        int _e = (int)(expr);                                                                  \
        if (_e != 0) return fail(-10, "%s: %s", stage, hipGetErrorString((hipError_t)_e));    \
        if (debug) {                                                                           \
            hipError_t _s = hipStreamSynchronize(stream);                                      \
            if (_s != hipSuccess) return fail(-11, "%s (sync): %s", stage, hipGetErrorString(_s)); \
        }                                                                                      \
    } while (0)

// ---- optional stage profiler ----
struct Profiler {
    std::mutex mu;
    uint32_t mask = 0;
    std::vector<hipEvent_t> pool;
    struct Rec {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Rec> pending;
    double ms[GSR_NUM_STAGES] = {};
    uint32_t counts[GSR_NUM_STAGES] = {};
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        return e;
    }
};
Profiler& prof() {
    static Profiler p;
    return p;
}

// RAII bracket of one stage on `stream` (no-op unless the stage is enabled)
struct StageTimer {
    int stage;
    hipStream_t stream;
    hipEvent_t a = nullptr, b = nullptr;
    StageTimer(int s, hipStream_t st) : stage(s), stream(st) {
        Profiler& p = prof();
        if (!(__atomic_load_n(&p.mask, __ATOMIC_RELAXED) & (1u << s))) return;
        std::lock_guard<std::mutex> lk(p.mu);
        a = p.get();
        b = p.get();
        if (a && b) hipEventRecord(a, stream);
    }
    ~StageTimer() {
        if (!a || !b) return;
        hipEventRecord(b, stream);
        Profiler& p = prof();
        std::lock_guard<std::mutex> lk(p.mu);
        p.pending.push_back({stage, a, b});
    }
};

#define GSR_STAGE(id, expr, name)          \
    do {                                   \
        StageTimer _timer((id), stream);   \
        GSR_CHECK_HIP(expr, name);         \
    } while (0)

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int validate(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs) {
    if (!cam || !gs || !rs) return fail(-1, "null camera/gaussians/settings");
    if (cam->width <= 0 || cam->height <= 0) return fail(-1, "bad image size %dx%d", cam->width, cam->height);
    if ((long long)div_up(cam->width, kTile) >= 65535 || (long long)div_up(cam->height, kTile) >= 65535)
        return fail(-1, "image too large");
    if (gs->P < 0) return fail(-1, "negative P");
    if (gs->P == 0) return 0;
    if (!gs->means3D || !gs->opacities) return fail(-1, "means3D/opacities required");
    if (gs->sh_degree < 0 || gs->sh_degree > 3) return fail(-1, "sh_degree must be 0..3");
    if (!gs->colors_precomp) {
        if (!gs->sh_dc) return fail(-1, "sh_dc required without colors_precomp");
        const int need = (gs->sh_degree + 1) * (gs->sh_degree + 1) - 1;
        if (need > 0 && (!gs->sh_rest || gs->sh_rest_coeffs < need))
            return fail(-1, "sh_rest must hold >= %d coefficients for degree %d", need, gs->sh_degree);
        if (gs->sh_rest_coeffs > 15) return fail(-1, "sh_rest_coeffs > 15");
    }
    if (!gs->cov3D_precomp) {
        if (!gs->scales || !gs->rotations) return fail(-1, "scales/rotations required without cov3D_precomp");
        if (!aligned16(gs->rotations)) return fail(-1, "rotations must be 16-byte aligned");
    }
    return 0;
}

gsr::GaussIn gauss_in(const gsr_gaussians* gs) {
    GaussIn in;
    in.P = gs->P;
    in.D = gs->sh_degree;
    in.M_rest = gs->sh_rest ? gs->sh_rest_coeffs : 0;
    in.smod = gs->scale_modifier;
    in.means3D = gs->means3D;
    in.sh_dc = gs->sh_dc;
    in.sh_rest = gs->sh_rest;
    in.colors = gs->colors_precomp;
    in.opac = gs->opacities;
    in.scales = gs->scales;
    in.rots = gs->rotations;
    in.cov3D = gs->cov3D_precomp;
    return in;
}

void band(const gsr_camera* cam, const gsr_raster_settings* rs, int* y0, int* y1) {
    const int gy = div_up(cam->height, kTile);
    *y0 = rs->tile_y0 < 0 ? 0 : (rs->tile_y0 > gy ? gy : rs->tile_y0);
    *y1 = rs->tile_y1 > gy ? gy : rs->tile_y1;
    if (*y1 < *y0) *y1 = *y0;
}

struct Views {
    uint32_t *depth_key, *tiles, *offsets, *gid_by_rank;
    float4* rec;
    uint2* ranges;
    float* final_T;
    float* accum;
    uint32_t *sorted_tile, *sorted_gid, *inst_gid;
    uint4* rect;
    float4* ck;  // B1 chunk checkpoints (nullptr: not chunked)
};

Views views(const gsr_camera* cam, int P, const gsr_buffers* b, int ck_tiles = 0) {
    Views v{};
    GeomLayout gl(P);
    ImgLayout il(cam->width, cam->height, ck_tiles);
    v.depth_key = at<uint32_t>(b->geom, gl.depth_key);
    v.tiles = at<uint32_t>(b->geom, gl.tiles);
    v.rec = at<float4>(b->geom, gl.rec);
    v.offsets = at<uint32_t>(b->geom, gl.offsets);
    v.rect = at<uint4>(b->geom, gl.rect);
    // 32-bit depth key = 4 passes (even) -> result in the A buffers
    v.gid_by_rank = at<uint32_t>(b->geom, gl.sA_v);
    v.ranges = at<uint2>(b->image, il.ranges);
    v.final_T = at<float>(b->image, il.final_T);
    v.accum = at<float>(b->image, il.accum);
    v.ck = ck_tiles ? at<float4>(b->image, il.ck) : nullptr;
    if (b->binning) {
        BinLayout bl(b->num_rendered);
        const int tiles = div_up(cam->width, kTile) * div_up(cam->height, kTile);
        const bool odd = (tile_passes(tiles) & 1) != 0;
        v.sorted_tile = at<uint32_t>(b->binning, odd ? bl.kB : bl.kA);
        v.sorted_gid = at<uint32_t>(b->binning, odd ? bl.vB : bl.vA);
        v.inst_gid = at<uint32_t>(b->binning, bl.inst_gid);
    }
    return v;
}

__global__ void fill_background(float* out_color, float* final_T, float* accum,
                                int npix, float bg0, float bg1, float bg2) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= npix) return;
    accum[i] = 0.0f;
    accum[npix + i] = 0.0f;
    accum[2 * (size_t)npix + i] = 0.0f;
    out_color[i] = bg0;
    out_color[npix + i] = bg1;
    out_color[2 * (size_t)npix + i] = bg2;
    final_T[i] = 1.0f;
}

}  // namespace

namespace gsr {
// error hook for the other translation units of the library (gsr_train.hip)
int set_error(int code, const char* msg) {
    g_err = msg;
    return code;
}
}  // namespace gsr

extern "C" {

int gsr_abi_version(void) { return GSR_ABI_VERSION; }
const char* gsr_last_error(void) { return g_err.c_str(); }

size_t gsr_geom_bytes(int32_t P) { return GeomLayout(P).total; }
size_t gsr_binning_bytes(int32_t K) { return BinLayout(K).total; }
size_t gsr_image_bytes(int32_t w, int32_t h) {
    return ImgLayout(w, h, chunked_tiles(w, 0, div_up(h, kTile))).total;
}
size_t gsr_scratch_bytes(int32_t K) { return PartLayout(K).total; }

// GSR_BIN_VARIANT=0 (A/B only): global depth sort of the P (or band-candidate) keys first.
static int forward_global_depth(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                                float* out_color, int32_t* radii, gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_binning,
                                gsr_alloc_fn alloc_image, void* ctx, gsr_buffers* bufs, void* stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    const int P = gs->P;
    const int W = cam->width, H = cam->height;
    const int gx = div_up(W, kTile), gy = div_up(H, kTile);
    int ty0, ty1;
    band(cam, rs, &ty0, &ty1);
    std::memset(bufs, 0, sizeof *bufs);
    bufs->geom = alloc_geom(ctx, GeomLayout(P).total);
    const int ckt = chunked_tiles(W, ty0, ty1);
    bufs->image = alloc_image(ctx, ImgLayout(W, H, ckt).total);
    if (!bufs->geom || !bufs->image) return fail(-2, "allocation failed (geometry/image)");
    GeomLayout gl(P);
    ImgLayout il(W, H, ckt);
    uint32_t* depth_key = at<uint32_t>(bufs->geom, gl.depth_key);
    uint32_t* tiles = at<uint32_t>(bufs->geom, gl.tiles);
    float4* rec = at<float4>(bufs->geom, gl.rec);
    uint32_t* offsets = at<uint32_t>(bufs->geom, gl.offsets);
    uint32_t* cand_tmp = at<uint32_t>(bufs->geom, gl.cand_tmp);
    uint2* ranges = at<uint2>(bufs->image, il.ranges);
    float* final_T = at<float>(bufs->image, il.final_T);

    if ((ty0 > 0 || ty1 < gy) && !(rs->flags & GSR_FLAG_BAND_ONLY)) {
        const int npix = W * H;
        hipLaunchKernelGGL(fill_background, dim3(div_up(npix, 256)), dim3(256), 0, stream, out_color,
                           final_T, at<float>(bufs->image, il.accum), npix, rs->bg[0], rs->bg[1],
                           rs->bg[2]);
        GSR_STAGE(GSR_STAGE_MISC, hipGetLastError(), "fill_background");
    }
    uint32_t* counters = at<uint32_t>(bufs->image, il.counters);
    GSR_STAGE(GSR_STAGE_MISC, hipMemsetAsync(ranges, 0, il.ovf - il.ranges, stream), "memset ranges");

    long long K = 0;
    if (P > 0) {
        const bool full_img = ty0 == 0 && ty1 == gy;
        PreOut po{radii, depth_key, tiles, rec, at<uint4>(bufs->geom, gl.rect),
                  full_img ? at<uint32_t>(bufs->geom, gl.flags) : nullptr, counters};
        GSR_STAGE(GSR_STAGE_PREPROCESS, launch_preprocess(*cam, gauss_in(gs), ty0, ty1, po, stream), "preprocess");
        // A band ranks only its candidates (Gaussians with tiles in the band): the depth sort,
        // scan, duplicate and gather then scale with the band, not with P.
        const bool banded = ty0 > 0 || ty1 < gy;
        int NR = P;
        const uint32_t* sort_keys = depth_key;
        const uint32_t* sort_vals = nullptr;
        uint32_t cw[2 * kCountSlots];  // preprocess's count partials: candidates, then K
        uint32_t cnt[2] = {0, 0};
        auto sum_counts = [&] {
            uint64_t c = 0, k = 0;
            for (int i = 0; i < kCountSlots; ++i) c += cw[i], k += cw[kCountSlots + i];
            cnt[0] = (uint32_t)(c < UINT32_MAX ? c : UINT32_MAX);
            cnt[1] = (uint32_t)(k < UINT32_MAX ? k : UINT32_MAX);
            return 0;
        };
        GSR_CHECK_HIP(begin_read(counters, 2 * kCountSlots, stream), "read counts");
        if (banded) {
            GSR_STAGE(GSR_STAGE_DEPTH_SORT, compact_candidates(tiles, depth_key, P, at<uint32_t>(bufs->geom, gl.partials),
                                                               offsets, cand_tmp, counters + kCandCountSlot, stream),
                      "band candidates");
            GSR_STAGE(GSR_STAGE_MISC, end_read(counters, cw, 2 * kCountSlots, stream), "read counts");
            sum_counts();
            NR = (int)cnt[0];
            sort_keys = offsets;  // free until the scan
            sort_vals = cand_tmp;
            if (colour_pass_needed(*cam, gauss_in(gs), ty0, ty1))
                GSR_STAGE(GSR_STAGE_PREPROCESS, launch_colour(*cam, gauss_in(gs), cand_tmp, NR, rec, stream),
                          "band colours");
        }
        bufs->num_ranked = NR;
        int which = NR > 0 ? -1 : 1;
        GSR_STAGE(GSR_STAGE_DEPTH_SORT, radix_sort(sort_keys, sort_vals, at<uint32_t>(bufs->geom, gl.sB_k),
                                 at<uint32_t>(bufs->geom, gl.sB_v), at<uint32_t>(bufs->geom, gl.sA_k),
                                 at<uint32_t>(bufs->geom, gl.sA_v), NR, 32, at<uint32_t>(bufs->geom, gl.hist),
                                 &which, stream, true),
                      "depth sort");
        if (NR > 0 && which != 1) return fail(-12, "depth sort ended in an unexpected buffer");
        // full image: K is read here, while the depth sort runs, so the host enqueues the rest
        // of the forward without leaving the GPU idle
        if (!banded) {
            GSR_STAGE(GSR_STAGE_MISC, end_read(counters, cw, 2 * kCountSlots, stream), "read counts");
            sum_counts();
        }
        const uint32_t* gid_by_rank = at<uint32_t>(bufs->geom, gl.sA_v);
        const bool fused = scan_variant(NR) == 1;
        if (NR > 0 && !fused) {
            GSR_STAGE(GSR_STAGE_SCAN, inclusive_scan_gather(tiles, gid_by_rank, offsets, NR,
                                                at<uint32_t>(bufs->geom, gl.partials), stream),
                      "scan");
        }
        K = cnt[1];
        if (K > INT32_MAX) return fail(-3, "num_rendered overflow (%lld)", K);
        bufs->num_rendered = (int32_t)K;
        bufs->binning = alloc_binning(ctx, BinLayout(K).total);
        if (!bufs->binning) return fail(-2, "allocation failed (binning, K=%lld)", K);
        BinLayout bl(K);
        uint32_t* kA = at<uint32_t>(bufs->binning, bl.kA);
        uint32_t* vA = at<uint32_t>(bufs->binning, bl.vA);
        uint32_t* kB = at<uint32_t>(bufs->binning, bl.kB);
        uint32_t* vB = at<uint32_t>(bufs->binning, bl.vB);
        uint32_t* inst_gid = at<uint32_t>(bufs->binning, bl.inst_gid);
        if (fused) {
            GSR_STAGE(GSR_STAGE_DUPLICATE, launch_scan_duplicate(gid_by_rank, tiles, at<uint4>(bufs->geom, gl.rect), NR, gx, ty0,
                                                offsets, kA, inst_gid,
                                                at<uint32_t>(bufs->geom, gl.hist), stream),
                      "scan + duplicate");
        } else {
            GSR_STAGE(GSR_STAGE_DUPLICATE, launch_duplicate(gid_by_rank, offsets, tiles, at<uint4>(bufs->geom, gl.rect), NR, gx, ty0, ty1,
                                               kA, inst_gid, stream),
                      "duplicate");
        }
        if (K > 0) {
            int w2 = -1;
            GSR_STAGE(GSR_STAGE_TILE_SORT, radix_sort(kA, inst_gid, kB, vB, kA, vA, K, tile_bits(gx * gy),
                                     at<uint32_t>(bufs->binning, bl.hist), &w2, stream, false),
                          "tile sort");
            const bool odd = (tile_passes(gx * gy) & 1) != 0;
            if ((w2 == 0) != odd) return fail(-12, "tile sort ended in an unexpected buffer");
            GSR_STAGE(GSR_STAGE_FINALIZE, launch_finalize(odd ? kB : kA, K, ranges, stream),
                          "finalize");
        }
    } else {
        bufs->binning = alloc_binning(ctx, BinLayout(0).total);
    }
    const Views v = views(cam, P, bufs, ckt);
    GSR_STAGE(GSR_STAGE_BLEND_FWD, launch_blend_forward(*cam, rs->bg, ty0, ty1, ranges, v.sorted_gid, rec, out_color, final_T,
                                       v.accum, v.ck, stream),
                  "blend forward");
    return 0;
}

}  // extern "C"

namespace {

// One view's forward (binning variants 1 / 2), split at the host read of its instance count:
// a batch enqueues phase 1 of every view before it waits once (gsr_forward_batch).
struct FwdJob {
    const gsr_camera* cam;
    const gsr_gaussians* gs;
    const gsr_raster_settings* rs;
    float* out_color;
    int32_t* radii;
    gsr_buffers* bufs;
    int ty0 = 0, ty1 = 0, gx = 0, gy = 0, ckt = 0;
    bool full_img = true;
};

// Allocations, background / range clears, F1, then the scan (full image) or the band's
// candidate compaction.  read_counts: enqueue the D2H of F1's count partials right after F1,
// so the scan / compaction run while the host waits for them.
int fwd_phase1(FwdJob& j, gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_image, void* ctx, hipStream_t stream,
               bool debug, bool read_counts) {
    const gsr_camera* cam = j.cam;
    const gsr_gaussians* gs = j.gs;
    const gsr_raster_settings* rs = j.rs;
    gsr_buffers* bufs = j.bufs;
    const int P = gs->P, W = cam->width, H = cam->height;
    j.gx = div_up(W, kTile);
    j.gy = div_up(H, kTile);
    band(cam, rs, &j.ty0, &j.ty1);
    j.full_img = j.ty0 == 0 && j.ty1 == j.gy;
    std::memset(bufs, 0, sizeof *bufs);
    bufs->geom = alloc_geom(ctx, GeomLayout(P).total);
    j.ckt = chunked_tiles(W, j.ty0, j.ty1);
    bufs->image = alloc_image(ctx, ImgLayout(W, H, j.ckt).total);
    if (!bufs->geom || !bufs->image) return fail(-2, "allocation failed (geometry/image)");
    GeomLayout gl(P);
    ImgLayout il(W, H, j.ckt);
    uint2* ranges = at<uint2>(bufs->image, il.ranges);
    if (!j.full_img && !(rs->flags & GSR_FLAG_BAND_ONLY)) {
        const int npix = W * H;
        hipLaunchKernelGGL(fill_background, dim3(div_up(npix, 256)), dim3(256), 0, stream, j.out_color,
                           at<float>(bufs->image, il.final_T), at<float>(bufs->image, il.accum), npix, rs->bg[0],
                           rs->bg[1], rs->bg[2]);
        GSR_STAGE(GSR_STAGE_MISC, hipGetLastError(), "fill_background");
    }
    GSR_STAGE(GSR_STAGE_MISC, hipMemsetAsync(ranges, 0, il.ovf - il.ranges, stream), "memset ranges");
    if (P == 0) return 0;
    uint32_t* depth_key = at<uint32_t>(bufs->geom, gl.depth_key);
    uint32_t* tiles = at<uint32_t>(bufs->geom, gl.tiles);
    uint32_t* counters = at<uint32_t>(bufs->image, il.counters);
    uint32_t* gid_by_rank = at<uint32_t>(bufs->geom, gl.sA_v);
    PreOut po{j.radii, depth_key, tiles, at<float4>(bufs->geom, gl.rec), at<uint4>(bufs->geom, gl.rect),
              j.full_img ? at<uint32_t>(bufs->geom, gl.flags) : nullptr, counters};
    GSR_STAGE(GSR_STAGE_PREPROCESS, launch_preprocess(*cam, gauss_in(gs), j.ty0, j.ty1, po, stream), "preprocess");
    if (read_counts) GSR_CHECK_HIP(begin_read(counters, 2 * kCountSlots, stream), "read counts");
    if (!j.full_img) {
        GSR_STAGE(GSR_STAGE_DEPTH_SORT, compact_candidates(tiles, depth_key, P, at<uint32_t>(bufs->geom, gl.partials),
                                                           at<uint32_t>(bufs->geom, gl.offsets), gid_by_rank,
                                                           counters + kCandCountSlot, stream),
                  "band candidates");
    } else {
        // the scan needs no count; gid_by_rank = the identity ranking
        GSR_STAGE(GSR_STAGE_SCAN, inclusive_scan_gather(tiles, nullptr, at<uint32_t>(bufs->geom, gl.offsets), P,
                                                        at<uint32_t>(bufs->geom, gl.partials), stream, gid_by_rank),
                  "scan");
    }
    return 0;
}

// The rest, given F1's counts: band colours, binning, per-tile depth order, F6.
int fwd_phase2(FwdJob& j, uint64_t csum, uint64_t ksum, gsr_alloc_fn alloc_binning, void* ctx, hipStream_t stream,
               bool debug) {
    const gsr_camera* cam = j.cam;
    const gsr_gaussians* gs = j.gs;
    const gsr_raster_settings* rs = j.rs;
    gsr_buffers* bufs = j.bufs;
    const int P = gs->P, gx = j.gx, gy = j.gy, ty0 = j.ty0, ty1 = j.ty1;
    const bool full_img = j.full_img, scanned = j.full_img;
    const int bv = bin_variant();
    GeomLayout gl(P);
    ImgLayout il(cam->width, cam->height, j.ckt);
    uint32_t* depth_key = at<uint32_t>(bufs->geom, gl.depth_key);
    uint32_t* tiles = at<uint32_t>(bufs->geom, gl.tiles);
    float4* rec = at<float4>(bufs->geom, gl.rec);
    uint32_t* offsets = at<uint32_t>(bufs->geom, gl.offsets);
    uint32_t* counters = at<uint32_t>(bufs->image, il.counters);
    uint2* ranges = at<uint2>(bufs->image, il.ranges);
    uint32_t* gid_by_rank = at<uint32_t>(bufs->geom, gl.sA_v);
    uint32_t* tcount = bv == 2 ? at<uint32_t>(bufs->image, il.tcount) : nullptr;
    long long K = 0;
    if (P > 0) {
        int NR = P;
        if (!full_img) {
            NR = (int)(csum < (uint64_t)P ? csum : (uint64_t)P);
            if (colour_pass_needed(*cam, gauss_in(gs), ty0, ty1))
                GSR_STAGE(GSR_STAGE_PREPROCESS, launch_colour(*cam, gauss_in(gs), gid_by_rank, NR, rec, stream),
                          "band colours");
        }
        bufs->num_ranked = NR;
        K = (long long)ksum;
        if (K > INT32_MAX) return fail(-3, "num_rendered overflow (%lld)", K);
        bufs->num_rendered = (int32_t)K;
        bufs->binning = alloc_binning(ctx, BinLayout(K).total);
        if (!bufs->binning) return fail(-2, "allocation failed (binning, K=%lld)", K);
        BinLayout bl(K);
        uint32_t* kA = at<uint32_t>(bufs->binning, bl.kA);
        uint32_t* vA = at<uint32_t>(bufs->binning, bl.vA);
        uint32_t* kB = at<uint32_t>(bufs->binning, bl.kB);
        uint32_t* vB = at<uint32_t>(bufs->binning, bl.vB);
        uint32_t* inst_gid = at<uint32_t>(bufs->binning, bl.inst_gid);
        // final (tile, gid) arrays where views() expects them, and the free pair beside them
        const bool odd = (tile_passes(gx * gy) & 1) != 0;
        uint32_t* fk = odd ? kB : kA;
        uint32_t* fv = odd ? vB : vA;
        uint32_t* sk = odd ? kA : kB;
        uint32_t* sv = odd ? vA : vB;
        uint32_t* dup_key = bv == 2 ? sk : kA;  // F3's tile keys (emission order)
        // variant 1: F3 also writes each instance's depth key, the tile sort carries it, and
        // the per-tile sort reads it contiguously instead of gathering depth_key[gid]
        const bool carry = bv == 1 && carry_depth();
        uint32_t* dA = at<uint32_t>(bufs->binning, bl.dA);
        uint32_t* dB = at<uint32_t>(bufs->binning, bl.dB);
        if (NR > 0 && !scanned && scan_variant(NR) == 1) {
            GSR_STAGE(GSR_STAGE_DUPLICATE, launch_scan_duplicate(gid_by_rank, tiles, at<uint4>(bufs->geom, gl.rect), NR, gx,
                                                                 ty0, offsets, dup_key, inst_gid,
                                                                 at<uint32_t>(bufs->geom, gl.hist), stream, tcount,
                                                                 depth_key, carry ? dA : nullptr),
                      "scan + duplicate");
        } else if (NR > 0) {
            if (!scanned)
                GSR_STAGE(GSR_STAGE_SCAN, inclusive_scan_gather(tiles, gid_by_rank, offsets, NR,
                                                                at<uint32_t>(bufs->geom, gl.partials), stream),
                          "scan");
            GSR_STAGE(GSR_STAGE_DUPLICATE, launch_duplicate(gid_by_rank, offsets, tiles, at<uint4>(bufs->geom, gl.rect), NR,
                                                            gx, ty0, ty1, dup_key, inst_gid, stream, tcount,
                                                            depth_key, carry ? dA : nullptr),
                      "duplicate");
        }
        if (K > 0) {
            if (bv == 2) {
                GSR_STAGE(GSR_STAGE_TILE_SORT, launch_tile_bins(sk, inst_gid, K, ty0 * gx, (ty1 - ty0) * gx, tcount, ranges,
                                                                fk, fv, stream),
                          "tile bins");
            } else {
                int w2 = -1;
                GSR_STAGE(GSR_STAGE_TILE_SORT, radix_sort(kA, inst_gid, kB, vB, kA, vA, K, tile_bits(gx * gy),
                                                          at<uint32_t>(bufs->binning, bl.hist), &w2, stream, false,
                                                          carry ? dA : nullptr, dB, dA),
                          "tile sort");
                if ((w2 == 0) != odd) return fail(-12, "tile sort ended in an unexpected buffer");
                GSR_STAGE(GSR_STAGE_FINALIZE, launch_finalize(fk, K, ranges, stream), "finalize");
            }
            GSR_STAGE(GSR_STAGE_DEPTH_SORT, launch_tile_depth_sort(ranges, ty0 * gx, (ty1 - ty0) * gx, K, depth_key, fv,
                                                                   at<uint32_t>(bufs->image, il.ovf),
                                                                   counters + kOvfCountSlot,
                                                                   at<uint32_t>(bufs->image, il.ovf2),
                                                                   counters + kOvf2CountSlot, sk, sv, stream, bv == 1,
                                                                   carry ? (odd ? dB : dA) : nullptr),
                      "per-tile depth order");
        }
    } else {
        bufs->binning = alloc_binning(ctx, BinLayout(0).total);
    }
    const Views v = views(cam, P, bufs, j.ckt);
    GSR_STAGE(GSR_STAGE_BLEND_FWD, launch_blend_forward(*cam, rs->bg, ty0, ty1, ranges, v.sorted_gid, rec, j.out_color,
                                                        at<float>(bufs->image, il.final_T), v.accum, v.ck, stream),
              "blend forward");
    return 0;
}

// Per view of a batch: the sum of F1's 64 instance-count partials, as a u64 in two words.
struct CountPtrs {
    const uint32_t* c[GSR_MAX_BATCH];
};
__global__ __launch_bounds__(64) void batch_counts_kernel(CountPtrs p, uint32_t* __restrict__ out) {
    const uint32_t* c = p.c[blockIdx.x];
    uint32_t lo = c[kCountSlots + threadIdx.x], hi = 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {  // 64-bit sum from two 32-bit shuffles
        const uint32_t l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
        const uint32_t s = lo + l2;
        hi = hi + h2 + (s < lo ? 1u : 0u);
        lo = s;
    }
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = lo;
        out[2 * blockIdx.x + 1] = hi;
    }
}

}  // namespace

extern "C" {

int gsr_forward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                float* out_color, int32_t* radii, gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_binning,
                gsr_alloc_fn alloc_image, void* ctx, gsr_buffers* bufs, void* stream_) {
    g_err.clear();
    if (int e = validate(cam, gs, rs)) return e;
    if (!out_color || (gs->P > 0 && !radii) || !bufs || !alloc_geom || !alloc_binning || !alloc_image)
        return fail(-1, "null output / allocator");
    if (bin_variant() == 0)
        return forward_global_depth(cam, gs, rs, out_color, radii, alloc_geom, alloc_binning, alloc_image, ctx, bufs,
                                    stream_);
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    FwdJob j{cam, gs, rs, out_color, radii, bufs};
    if (int e = fwd_phase1(j, alloc_geom, alloc_image, ctx, stream, debug, true)) return e;
    uint64_t csum = 0, ksum = 0;
    if (gs->P > 0) {
        uint32_t cw[2 * kCountSlots];
        const uint32_t* counters = at<uint32_t>(bufs->image, ImgLayout(cam->width, cam->height, j.ckt).counters);
        GSR_STAGE(GSR_STAGE_MISC, end_read(counters, cw, 2 * kCountSlots, stream), "read counts");
        for (int i = 0; i < kCountSlots; ++i) csum += cw[i], ksum += cw[kCountSlots + i];
    }
    return fwd_phase2(j, csum, ksum, alloc_binning, ctx, stream, debug);
}

int gsr_forward_batch(int32_t V, const gsr_camera* cams, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                      float* const* out_colors, int32_t* const* radii, gsr_alloc_fn alloc_geom,
                      gsr_alloc_fn alloc_binning, gsr_alloc_fn alloc_image, void* ctx, gsr_buffers* bufs,
                      void* stream_) {
    g_err.clear();
    if (V < 0 || V > GSR_MAX_BATCH) return fail(-1, "batch: 0..%d views, got %d", GSR_MAX_BATCH, V);
    if (V == 0) return 0;
    if (!cams || !gs || !rs || !out_colors || !bufs || !alloc_geom || !alloc_binning || !alloc_image ||
        (gs->P > 0 && !radii))
        return fail(-1, "batch: null argument");
    if (bin_variant() == 0) return fail(-1, "batch: needs the per-tile binning (GSR_BIN_VARIANT != 0)");
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    std::vector<FwdJob> jobs;
    jobs.reserve(V);
    for (int v = 0; v < V; ++v) {
        if (int e = validate(&cams[v], gs, rs)) return e;
        if (rs->tile_y0 > 0 || rs->tile_y1 < div_up(cams[v].height, kTile))
            return fail(-1, "batch: full-image views only (view %d)", v);
        if (!out_colors[v] || (gs->P > 0 && !radii[v])) return fail(-1, "batch: null output of view %d", v);
        jobs.push_back(FwdJob{&cams[v], gs, rs, out_colors[v], gs->P > 0 ? radii[v] : nullptr, &bufs[v]});
        if (int e = fwd_phase1(jobs[v], alloc_geom, alloc_image, ctx, stream, debug, false)) return e;
    }
    std::vector<uint64_t> K(V, 0);
    if (gs->P > 0) {
        uint32_t* words = static_cast<uint32_t*>(alloc_image(ctx, 8 * (size_t)V));
        if (!words) return fail(-2, "allocation failed (batch counts)");
        CountPtrs cp{};
        for (int v = 0; v < V; ++v)
            cp.c[v] = at<uint32_t>(bufs[v].image, ImgLayout(cams[v].width, cams[v].height, jobs[v].ckt).counters);
        hipLaunchKernelGGL(batch_counts_kernel, dim3(V), dim3(64), 0, stream, cp, words);
        GSR_STAGE(GSR_STAGE_MISC, hipGetLastError(), "batch counts");
        uint32_t host[2 * GSR_MAX_BATCH];
        GSR_CHECK_HIP(begin_read(words, 2 * V, stream), "read counts");
        GSR_STAGE(GSR_STAGE_MISC, end_read(words, host, 2 * V, stream), "read counts");
        for (int v = 0; v < V; ++v) K[v] = (uint64_t)host[2 * v] | ((uint64_t)host[2 * v + 1] << 32);
    }
    for (int v = 0; v < V; ++v)
        if (int e = fwd_phase2(jobs[v], (uint64_t)gs->P, K[v], alloc_binning, ctx, stream, debug)) return e;
    return 0;
}

}  // extern "C"

extern "C" {

// SH clamp bits stored by the forward (full image), or nullptr: B2 recomputes them (band).
static const uint32_t* stored_flags(const gsr_camera* cam, const gsr_raster_settings* rs, const gsr_buffers* b,
                                    int P) {
    int ty0, ty1;
    band(cam, rs, &ty0, &ty1);
    if (ty0 != 0 || ty1 != div_up(cam->height, kTile)) return nullptr;
    return at<uint32_t>(b->geom, GeomLayout(P).flags);
}

// Per-Gaussian grad2d for all P: the gather covers the ranked Gaussians (a band's candidates);
// the rest touched no tile of the band and get zeros.
static int gather_all(const gsr_camera* cam, const gsr_raster_settings* rs, const Views& v, const gsr_buffers* bufs,
                      const float* partial, long long K, int P, float* grad2d, hipStream_t stream) {
    const int NR = bufs->num_ranked > 0 ? bufs->num_ranked : P;
    if (NR < P && !(rs->flags & GSR_FLAG_BAND_ONLY)) {
        if (hipError_t e = hipMemsetAsync(grad2d, 0, sizeof(float) * kPart * (size_t)P, stream)) return (int)e;
    }
    return launch_gather_grad2d(v.gid_by_rank, v.offsets, partial, v.rec, cam->width, cam->height, K, NR, grad2d,
                                stream);
}

static int backward_impl(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                         const gsr_buffers* bufs, const float* dL_dpix, gsr_alloc_fn alloc_scratch,
                         void* ctx, const gsr_grads* grads, float* grad2d, void* stream_) {
    if (int e = validate(cam, gs, rs)) return e;
    if (!bufs || !bufs->geom || !bufs->image || !dL_dpix) return fail(-1, "missing forward buffers / dL_dpix");
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    const int P = gs->P;
    if (P == 0) return 0;
    int ty0, ty1;
    band(cam, rs, &ty0, &ty1);
    const Views v = views(cam, P, bufs, chunked_tiles(cam->width, ty0, ty1));
    const long long K = bufs->num_rendered;
    float* partial = nullptr;
    if (K > 0) {
        if (!alloc_scratch) return fail(-1, "null scratch allocator");
        partial = static_cast<float*>(alloc_scratch(ctx, gsr_scratch_bytes((int32_t)K)));
        if (!partial) return fail(-2, "allocation failed (scratch, K=%lld)", K);
        GSR_STAGE(GSR_STAGE_MISC, launch_clear_partial(partial, K, stream), "clear partials");
        GSR_STAGE(GSR_STAGE_BLEND_BWD, launch_blend_backward(*cam, rs->bg, ty0, ty1, v.ranges, v.sorted_gid, v.rect, v.rec,
                                            v.final_T, v.accum, dL_dpix, partial, K, v.ck, stream),
                      "blend backward");
    }
    if (grad2d) {
        if (K > 0) {
            GSR_STAGE(GSR_STAGE_GATHER, gather_all(cam, rs, v, bufs, partial, K, P, grad2d, stream), "gather grad2d");
        } else {
            GSR_STAGE(GSR_STAGE_MISC, hipMemsetAsync(grad2d, 0, sizeof(float) * kPart * (size_t)P, stream), "zero grad2d");
        }
        return 0;
    }
    return 0;
}

static int check_grads(const gsr_gaussians* gs, const gsr_grads* g) {
    if (!g || !g->dL_dmeans2D || !g->dL_dopacity || !g->dL_dmeans3D) return fail(-1, "missing gradient outputs");
    if (gs->colors_precomp ? !g->dL_dcolors : !g->dL_dsh_dc) return fail(-1, "missing colour/SH gradient output");
    if (!gs->colors_precomp && gs->sh_rest && !g->dL_dsh_rest) return fail(-1, "missing sh_rest gradient output");
    if (gs->cov3D_precomp ? !g->dL_dcov3D : (!g->dL_dscales || !g->dL_drotations))
        return fail(-1, "missing cov3D / scale / rotation gradient output");
    return 0;
}

static GradOut grad_out(const gsr_grads* g) {
    GradOut o;
    o.means2D = g->dL_dmeans2D;
    o.conic = g->dL_dconic;
    o.opac = g->dL_dopacity;
    o.colors = g->dL_dcolors;
    o.means3D = g->dL_dmeans3D;
    o.sh_dc = g->dL_dsh_dc;
    o.sh_rest = g->dL_dsh_rest;
    o.scales = g->dL_dscales;
    o.rots = g->dL_drotations;
    o.cov3D = g->dL_dcov3D;
    return o;
}

int gsr_backward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                 const gsr_buffers* bufs, const float* dL_dpix, gsr_alloc_fn alloc_scratch, void* ctx,
                 const gsr_grads* grads, void* stream_) {
    g_err.clear();
    if (int e = validate(cam, gs, rs)) return e;
    if (gs->P == 0) return 0;
    if (int e = check_grads(gs, grads)) return e;
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    if (!bufs || !bufs->geom || !bufs->image || !dL_dpix) return fail(-1, "missing forward buffers / dL_dpix");
    if (!alloc_scratch) return fail(-1, "null scratch allocator");
    int ty0, ty1;
    band(cam, rs, &ty0, &ty1);
    const int P = gs->P;
    const Views v = views(cam, P, bufs, chunked_tiles(cam->width, ty0, ty1));
    const long long K = bufs->num_rendered;
    // two scratch blocks: per-instance partials (K x 48 B) and per-Gaussian grad2d (P x 48 B)
    float* partial = static_cast<float*>(alloc_scratch(ctx, gsr_scratch_bytes((int32_t)K)));
    float* grad2d = static_cast<float*>(alloc_scratch(ctx, sizeof(float) * kPart * (size_t)P));
    if (!partial || !grad2d) return fail(-2, "allocation failed (scratch, K=%lld, P=%d)", K, P);
    // full image ranked in gid order (shipped binning): gather + B2 fused, grad2d unused
    const bool fuse = K > 0 && bin_variant() != 0 && ty0 == 0 && ty1 == div_up(cam->height, kTile) &&
                      bufs->num_ranked == P && fuse_gather();
    if (K > 0) {
        GSR_STAGE(GSR_STAGE_MISC, launch_clear_partial(partial, K, stream), "clear partials");
        GSR_STAGE(GSR_STAGE_BLEND_BWD, launch_blend_backward(*cam, rs->bg, ty0, ty1, v.ranges, v.sorted_gid, v.rect, v.rec,
                                            v.final_T, v.accum, dL_dpix, partial, K, v.ck, stream),
                      "blend backward");
        if (fuse) {
            GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_gather_backward(*cam, gauss_in(gs), v.depth_key,
                                                                       stored_flags(cam, rs, bufs, P), v.offsets,
                                                                       partial, v.rec, K, grad_out(grads), stream),
                      "gather + preprocess backward");
            return 0;
        }
        GSR_STAGE(GSR_STAGE_GATHER, gather_all(cam, rs, v, bufs, partial, K, P, grad2d, stream),
                  "gather grad2d");
    } else {
        GSR_STAGE(GSR_STAGE_MISC, hipMemsetAsync(grad2d, 0, sizeof(float) * kPart * (size_t)P, stream), "zero grad2d");
    }
    GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_preprocess_backward(*cam, gauss_in(gs), 0, P, v.depth_key, stored_flags(cam, rs, bufs, P), grad2d,
                                             grad_out(grads), stream),
                  "preprocess backward");
    return 0;
}

int gsr_backward_blend(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                       const gsr_buffers* bufs, const float* dL_dpix, gsr_alloc_fn alloc_scratch, void* ctx,
                       float* grad2d, void* stream) {
    g_err.clear();
    if (!grad2d && gs && gs->P > 0) return fail(-1, "null grad2d");
    return backward_impl(cam, gs, rs, bufs, dL_dpix, alloc_scratch, ctx, nullptr, grad2d, stream);
}

int gsr_backward_preprocess_range(const gsr_camera* cam, const gsr_gaussians* gs,
                                  const gsr_raster_settings* rs, const gsr_buffers* bufs, int32_t g0,
                                  int32_t g1, const float* grad2d, const gsr_grads* grads, void* stream_) {
    g_err.clear();
    if (int e = validate(cam, gs, rs)) return e;
    if (g0 < 0 || g1 > gs->P || g0 > g1) return fail(-1, "bad Gaussian range [%d, %d) for P=%d", g0, g1, gs->P);
    if (g0 == g1) return 0;
    if (int e = check_grads(gs, grads)) return e;
    if (!bufs || !bufs->geom || !grad2d) return fail(-1, "missing forward buffers / grad2d");
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    GeomLayout gl(gs->P);
    GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_preprocess_backward(*cam, gauss_in(gs), g0, g1, at<uint32_t>(bufs->geom, gl.depth_key),
                                             stored_flags(cam, rs, bufs, gs->P), grad2d,
                                             grad_out(grads), stream),
                  "preprocess backward");
    return 0;
}

int gsr_backward_preprocess(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                            const gsr_buffers* bufs, const float* grad2d, const gsr_grads* grads,
                            void* stream) {
    if (!gs) return fail(-1, "null gaussians");
    return gsr_backward_preprocess_range(cam, gs, rs, bufs, 0, gs->P, grad2d, grads, stream);
}

int gsr_profile_enable(uint32_t stage_mask) {
    Profiler& p = prof();
    std::lock_guard<std::mutex> lk(p.mu);
    for (auto& r : p.pending) {
        hipEventSynchronize(r.b);
        p.pool.push_back(r.a);
        p.pool.push_back(r.b);
    }
    p.pending.clear();
    for (int i = 0; i < GSR_NUM_STAGES; ++i) p.ms[i] = 0.0, p.counts[i] = 0;
    __atomic_store_n(&p.mask, stage_mask, __ATOMIC_RELAXED);
    return 0;
}

int gsr_profile_read(double* ms, uint32_t* counts) {
    Profiler& p = prof();
    std::lock_guard<std::mutex> lk(p.mu);
    for (auto& r : p.pending) {
        float t = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
            p.ms[r.stage] += t;
            p.counts[r.stage] += 1;
        }
        p.pool.push_back(r.a);
        p.pool.push_back(r.b);
    }
    p.pending.clear();
    for (int i = 0; i < GSR_NUM_STAGES; ++i) {
        if (ms) ms[i] = p.ms[i];
        if (counts) counts[i] = p.counts[i];
        p.ms[i] = 0.0;
        p.counts[i] = 0;
    }
    return 0;
}

const char* gsr_stage_name(int stage) {
    static const char* names[GSR_NUM_STAGES] = {"preprocess", "depth_sort", "scan", "duplicate", "tile_sort",
                                               "finalize", "blend_fwd", "blend_bwd", "preprocess_bwd",
                                               "gather_grad2d", "misc"};
    return (stage >= 0 && stage < GSR_NUM_STAGES) ? names[stage] : "?";
}

const void* gsr_view(const gsr_camera* cam, int32_t P, const gsr_buffers* bufs, int what) {
    if (!cam || !bufs || !bufs->geom || !bufs->image) return nullptr;
    const Views v = views(cam, P, bufs);
    switch (what) {
        case GSR_VIEW_RADII_SORTED_GID: return v.sorted_gid;
        case GSR_VIEW_SORTED_TILE: return v.sorted_tile;
        case GSR_VIEW_RANGES: return v.ranges;
        case GSR_VIEW_FINAL_T: return v.final_T;
        case GSR_VIEW_N_CONTRIB: return nullptr;  // retired: B1 re-derives termination from T
        case GSR_VIEW_DEPTH_KEY: return v.depth_key;
        case GSR_VIEW_TILES_TOUCHED: return v.tiles;
        case GSR_VIEW_RECORDS: return v.rec;
        case GSR_VIEW_GID_BY_RANK: return v.gid_by_rank;
        default: return nullptr;
    }
}

}  // extern "C"

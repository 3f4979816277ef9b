// gsr_api.cpp -- the C ABI (include/gsr/gsr.h) over the CDNA4 kernels.
//
// Stage order (forward, shipped binning): F1 preprocess -> scan of tiles_touched in gid order
// (a band: compaction of its candidates first) -> ONE device->host read of K -> F3 duplicate
// -> tile-key sort (K keys) -> F5 finalize (tile ranges) -> per-tile depth sort -> F6 blend.
// Backward: B1 blend backward -> gather -> B2 preprocess backward (or B1 -> per-Gaussian grad2d
// for the multi-GPU exchange).
// No persistent allocations; every scratch buffer comes from the caller's callbacks.
#include <hip/hip_runtime.h>

#include <algorithm>
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
        if (a && b) (void)hipEventRecord(a, stream);
    }
    ~StageTimer() {
        if (!a || !b) return;
        (void)hipEventRecord(b, stream);
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

// Device pointers into the caller's buffers (layouts in gsr_internal.h).  n: Gaussians (or
// received splat slots) indexed; cap: the binning's instance capacity.
struct Views {
    uint32_t *depth_key, *tiles, *flags, *offsets, *partials, *lookback;
    bool presort;                                          // gsr_internal.h use_presort
    bool rb;                                               // gsr_internal.h use_rb_binning
    uint32_t *rb_histA, *rb_histB, *rb_status;
    uint32_t *dk0, *dv0, *dk1, *dv1, *dhist, *rtiles;      // presort only
    uint4* rrect;
    float4* rec;
    uint4* rect;
    uint2* ranges;
    uint32_t *counters, *K_dev, *ovf, *ovf2, *done, *term;
    float *final_T, *accum;
    float4* ck;  // the checkpoint pool (binning buffer)
    size_t ck_bytes;
    uint32_t *kA, *vA, *kB, *vB, *hist;
    uint8_t* mk;                         // F6's per-entry stripe masks (B1's visit filter)
    uint32_t *sorted_tile, *sorted_gid;  // where the tile sort's result lands
    uint32_t *free_k, *free_v;           // the other ping-pong pair (scratch after the sort)
};

// The layout word a forward of n entries over gx x gy tiles, `ntiles` of them binned, with a
// binning of `cap` instances writes (fwd_phase2): the row-bucketed binning where the image fits
// it and the per-tile depth order can take it, the pre-sort on dense images.
uint32_t expected_layout(long long n, int gx, int gy, long long cap, int ntiles) {
    uint32_t w = GSR_LAYOUT_TAG;
    if (use_presort(n, gx, gy)) w |= kBufPresort;
    if (use_rb_binning(n, gx, gy) && cap > 0 && cap < kRbMaxCap &&
        (GSR_RB_DEEP || tile_wave_sort_eligible(cap, ntiles)))
        w |= kBufRowBucketed;
    return w;
}

// Every use of a forward's buffers after the forward checks the layout word: missing tag (a
// struct rebuilt without the field) or bits that disagree with what the forward of these sizes
// chose would make the backward read the wrong arrays -- refused instead (ABI 4).
int check_layout(const gsr_camera* cam, int ty0, int ty1, const gsr_buffers* b) {
    if ((b->layout & GSR_LAYOUT_TAG_MASK) != GSR_LAYOUT_TAG)
        return fail(GSR_ERR_LAYOUT,
                    "gsr_buffers.layout = 0x%08x is not a forward's (ABI %d): pass the forward's gsr_buffers "
                    "unchanged",
                    b->layout, GSR_ABI_VERSION);
    const int gx = div_up(cam->width, kTile), gy = div_up(cam->height, kTile);
    const uint32_t want = expected_layout(b->n_local, gx, gy, b->capacity, (ty1 - ty0) * gx);
    if (b->layout != want)
        return fail(GSR_ERR_LAYOUT,
                    "gsr_buffers.layout = 0x%08x disagrees with the buffers (0x%08x for %d entries, capacity %d, "
                    "tile rows [%d, %d) of %d x %d)",
                    b->layout, want, b->n_local, b->capacity, ty0, ty1, gx, gy);
    return 0;
}

Views views(const gsr_camera* cam, long long n, const gsr_buffers* b) {
    Views v{};
    const GeomLayout gl(n);
    const ImgLayout il(cam->width, cam->height);
    v.depth_key = at<uint32_t>(b->geom, gl.depth_key);
    v.tiles = at<uint32_t>(b->geom, gl.tiles);
    v.flags = at<uint32_t>(b->geom, gl.flags);
    v.rec = at<float4>(b->geom, gl.rec);
    v.rect = at<uint4>(b->geom, gl.rect);
    v.offsets = at<uint32_t>(b->geom, gl.offsets);
    v.partials = at<uint32_t>(b->geom, gl.partials);
    v.lookback = at<uint32_t>(b->geom, gl.lookback);
    v.presort = use_presort(n, div_up(cam->width, kTile), div_up(cam->height, kTile));
    v.rb = (b->layout & kBufRowBucketed) != 0;  // decided by the forward (fwd_phase2), checked by check_layout
    v.rb_histA = at<uint32_t>(b->geom, gl.rb_hist);
    if (v.presort) {
        v.dk0 = at<uint32_t>(b->geom, gl.dk0);
        v.dv0 = at<uint32_t>(b->geom, gl.dv0);
        v.dk1 = at<uint32_t>(b->geom, gl.dk1);
        v.dv1 = at<uint32_t>(b->geom, gl.dv1);
        v.dhist = at<uint32_t>(b->geom, gl.dhist);
        v.rtiles = at<uint32_t>(b->geom, gl.rtiles);
        v.rrect = at<uint4>(b->geom, gl.rrect);
    }
    v.ranges = at<uint2>(b->image, il.ranges);
    v.counters = at<uint32_t>(b->image, il.counters);
    v.K_dev = v.counters + kTotalSlot;
    v.ovf = at<uint32_t>(b->image, il.ovf);
    v.ovf2 = at<uint32_t>(b->image, il.ovf2);
    v.rb_status = at<uint32_t>(b->image, il.rb_status);
    v.done = at<uint32_t>(b->image, il.done);
    v.term = at<uint32_t>(b->image, il.term);
    v.final_T = at<float>(b->image, il.final_T);
    v.accum = at<float>(b->image, il.accum);
    if (b->binning) {
        const BinLayout bl(b->capacity, (long long)ImgLayout::tile_count(cam->width, cam->height));
        v.ck = at<float4>(b->binning, bl.ck);
        v.ck_bytes = bl.ckm - bl.ck;
        v.kA = at<uint32_t>(b->binning, bl.kA);
        v.vA = at<uint32_t>(b->binning, bl.vA);
        v.kB = at<uint32_t>(b->binning, bl.kB);
        v.vB = at<uint32_t>(b->binning, bl.vB);
        v.hist = at<uint32_t>(b->binning, bl.hist);
        v.mk = at<uint8_t>(b->binning, bl.mk);
        v.rb_histB = at<uint32_t>(b->binning, bl.rb_hist);
        const int tiles = div_up(cam->width, kTile) * div_up(cam->height, kTile);
        // the radix sort ends in (kB, vB) after odd passes; the row-bucketed binning writes (kA, vA)
        const bool odd = !v.rb && (tile_passes(tiles) & 1) != 0;
        v.sorted_tile = odd ? v.kB : v.kA;
        v.sorted_gid = odd ? v.vB : v.vA;
        v.free_k = odd ? v.kA : v.kB;
        v.free_v = odd ? v.vA : v.vB;
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

// One forward, split at the (optional) host read of K so a batch can wait once for all views.
struct FwdJob {
    const gsr_camera* cam;
    const gsr_raster_settings* rs;
    float* out_color;
    gsr_buffers* bufs;
    long long n = 0;  // Gaussians (or splat slots) indexed
    int ty0 = 0, ty1 = 0, gx = 0, gy = 0;
    int vgy = 0, vh = 0;  // views mode: tile rows per view band, pixel rows per view (0: one image)
    bool rows_counted = false;  // F1 wrote the row-bucketed binning's pass-A counts (run_preprocess)
};

// Allocations (geometry from the caller when geom_ready), range / counter clears, background
// outside the band (unless band_pixels_only), then F1 via `pre` (may be empty: splats unpacked
// by the caller) and the three-kernel scan when n is large.
template <class Pre>
int fwd_phase1(FwdJob& j, gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_image, void* ctx, hipStream_t stream, bool debug,
               bool band_pixels_only, Pre&& pre) {
    const gsr_camera* cam = j.cam;
    const gsr_raster_settings* rs = j.rs;
    gsr_buffers* bufs = j.bufs;
    const int W = cam->width, H = cam->height;
    j.gx = div_up(W, kTile);
    j.gy = div_up(H, kTile);
    band(cam, rs, &j.ty0, &j.ty1);
    std::memset(bufs, 0, sizeof *bufs);
    bufs->layout = GSR_LAYOUT_TAG | (use_presort(j.n, j.gx, j.gy) ? kBufPresort : 0u);
    bufs->num_rendered = -1;
    bufs->n_local = (int32_t)j.n;
    bufs->geom = alloc_geom(ctx, GeomLayout(j.n).total);
    bufs->image = alloc_image(ctx, ImgLayout(W, H).total);
    if (!bufs->geom || !bufs->image) return fail(-2, "allocation failed (geometry/image)");
    const ImgLayout il(W, H);
    const Views v = views(cam, j.n, bufs);
    if ((j.ty0 > 0 || j.ty1 < j.gy) && !band_pixels_only) {
        const int npix = W * H;
        hipLaunchKernelGGL(fill_background, dim3(div_up(npix, 256)), dim3(256), 0, stream, j.out_color, v.final_T,
                           v.accum, npix, rs->bg[0], rs->bg[1], rs->bg[2]);
        GSR_STAGE(GSR_STAGE_MISC, hipGetLastError(), "fill_background");
    }
    GSR_STAGE(GSR_STAGE_MISC, hipMemsetAsync(v.ranges, 0, il.ovf - il.ranges, stream), "clear ranges");
    if (int e = pre(v)) return e;
    if (v.presort) {  // global (depth, gid) order, the rank-order payload and its block sums + K
        // (the lookback words, unused by the presort path, hold the block sums; F3 finishes the scan)
        GSR_STAGE(GSR_STAGE_DEPTH_SORT, launch_depth_presort(v.depth_key, v.tiles, v.rect, (int)j.n, v.dk0, v.dv0,
                                                             v.dk1, v.dv1, v.dhist, v.rtiles, v.rrect, v.lookback,
                                                             v.K_dev, stream),
                  "depth presort");
        return 0;
    }
    // the row-bucketed binning (maybe taken in phase 2) needs the scan's offsets, not the fused
    // scan + F3; when F1 summed its blocks' tiles (rows_counted), one launch scans those sums and the
    // per-Gaussian offsets are written in phase 2
    const bool rb_possible = use_rb_binning(j.n, j.gx, j.gy);
    if (rb_possible && j.rows_counted)
        GSR_STAGE(GSR_STAGE_SCAN, launch_scan_blocks(v.lookback + 16, (int)j.n, v.K_dev, stream), "scan (block sums)");
    else
        GSR_STAGE(GSR_STAGE_SCAN, launch_scan(v.tiles, (int)j.n, v.offsets, v.partials, v.K_dev, stream, !rb_possible),
                  "scan");
    return 0;
}

// The rest, given the binning capacity: F3 (with F2 when fused), tile sort, ranges, per-tile
// depth order, F6.
int fwd_phase2(FwdJob& j, long long cap, gsr_alloc_fn alloc_binning, void* ctx, hipStream_t stream, bool debug) {
    const gsr_camera* cam = j.cam;
    gsr_buffers* bufs = j.bufs;
    if (cap > INT32_MAX) return fail(-3, "num_rendered overflow (%lld)", cap);
    bufs->capacity = (int32_t)cap;
    bufs->binning = alloc_binning(ctx, BinLayout(cap, (long long)ImgLayout::tile_count(cam->width, cam->height)).total);
    if (!bufs->binning) return fail(-2, "allocation failed (binning, %lld instances)", cap);
    const int tiles = j.gx * j.gy, ntiles = (j.ty1 - j.ty0) * j.gx;
    // Row-bucketed binning when the image fits it and the register form takes the per-tile depth
    // order (it leaves a tile's entries unordered, which that form does not mind); recorded in the
    // buffers so that every later view of them (backward, accessors) finds the same arrays.
    const bool scanned = use_rb_binning(j.n, j.gx, j.gy);  // phase 1 ran the three-kernel scan
    bufs->layout = expected_layout(j.n, j.gx, j.gy, cap, ntiles);
    const Views v = views(cam, j.n, bufs);
    if (v.presort)
        GSR_STAGE(GSR_STAGE_DUPLICATE, launch_duplicate_ranked(v.rtiles, v.rrect, v.rect, (int)j.n, j.gx, j.ty0,
                                                               v.lookback, v.offsets, v.kA, v.vA, cap, stream),
                  "duplicate (rank order)");
    else if (!v.rb) {
        if (scanned && j.rows_counted)  // phase 1 scanned F1's block sums only
            GSR_STAGE(GSR_STAGE_SCAN, launch_block_offsets(v.tiles, (int)j.n, v.lookback + 16, v.offsets, stream),
                      "offsets");
        GSR_STAGE(GSR_STAGE_DUPLICATE, launch_duplicate(v.tiles, v.rect, (int)j.n, j.gx, j.ty0, v.offsets, v.lookback,
                                                        v.kA, v.vA, cap, v.K_dev, stream, scanned),
                  "duplicate");
    }
    if (cap > 0 && v.rb) {
        // F3 + the tile sort + F5 as two counting passes; the pairs ride in (kB, vB)
        // (the tile keys are left to the GSR_VIEW_SORTED_TILE accessor: nothing in the step reads them;
        // kA carries the instances' depth keys from the placement to the per-tile sort instead)
        // With the depth keys placed (rb_keys): pass A's pairs as (gid, key) over kA..vA with their
        // columns in the checkpoint pool (which F6 fills only after the sort; used when it holds cap
        // words), pass B's instances as (gid, key) over kB..vB, and the per-tile sort writes the
        // ordered gids to vA -- one 8-B store per pair / instance and no key gather in the sort.
        const bool rb_keys = GSR_RB_SORT_KEYS && !GSR_RB_TILE_KEYS && v.ck_bytes >= 4 * (size_t)cap;
        uint2* const ppair = rb_keys ? reinterpret_cast<uint2*>(v.kA) : nullptr;
        uint2* const tpair = rb_keys ? reinterpret_cast<uint2*>(v.kB) : nullptr;
        uint32_t* const pxr = rb_keys ? reinterpret_cast<uint32_t*>(v.ck) : v.vB;
        GSR_STAGE(GSR_STAGE_TILE_SORT, launch_rb_binning(v.tiles, v.rect, v.offsets, (int)j.n, j.gx, j.ty0, j.ty1,
                                                         v.rb_histA, v.rb_histB, v.rb_status, v.kB, pxr,
                                                         GSR_RB_TILE_KEYS ? v.kA : nullptr, v.vA,
                                                         v.ranges, cap, stream, j.rows_counted,
                                                         j.rows_counted ? v.lookback + 16 : nullptr, v.K_dev,
                                                         v.depth_key, ppair, tpair),
                  "row-bucketed binning");
        GSR_STAGE(GSR_STAGE_DEPTH_SORT, launch_tile_depth_sort(v.ranges, j.ty0 * j.gx, ntiles, cap, v.depth_key,
                                                               v.sorted_gid, v.ovf, v.counters + kOvfCountSlot, v.ovf2,
                                                               v.counters + kOvf2CountSlot, v.done, v.free_k,
                                                               v.free_v, stream, true, tpair),
                  "per-tile depth order");
    } else if (cap > 0) {
        int which = -1;
        GSR_STAGE(GSR_STAGE_TILE_SORT, radix_sort(v.kA, v.vA, v.kB, v.vB, v.kA, v.vA, cap, v.K_dev, tile_bits(tiles),
                                                  v.hist, &which, stream),
                  "tile sort");
        // pass 1 writes (kB, vB), the next (kA, vA): which == 0 means the result is in (kB, vB)
        if ((which == 0) != (v.sorted_tile == v.kB)) return fail(-12, "tile sort ended in an unexpected buffer");
        GSR_STAGE(GSR_STAGE_FINALIZE, launch_finalize(v.sorted_tile, cap, v.K_dev, v.ranges, stream), "finalize");
        // presort mode: the stable tile sort of rank-ordered instances is already canonical
        if (!v.presort)
            GSR_STAGE(GSR_STAGE_DEPTH_SORT, launch_tile_depth_sort(v.ranges, j.ty0 * j.gx, ntiles, cap, v.depth_key,
                                                               v.sorted_gid, v.ovf, v.counters + kOvfCountSlot, v.ovf2,
                                                               v.counters + kOvf2CountSlot, v.done, v.free_k,
                                                               v.free_v, stream),
                  "per-tile depth order");
    }
    GSR_STAGE(GSR_STAGE_BLEND_FWD, launch_blend_forward(*cam, j.rs->bg, j.ty0, j.ty1, v.ranges, v.sorted_gid, v.rec,
                                                        j.out_color, v.final_T, v.accum, v.term, v.ck, cap, stream,
                                                        j.vgy, j.vh, v.mk),
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

// F1 over Gaussians [0, P) with the count partials K is read from
int run_preprocess(const gsr_camera* cam, const gsr_gaussians* gs, int ty0, int ty1, int32_t* radii, const Views& v,
                   hipStream_t stream, bool debug) {
    if (gs->P <= 0) return 0;
    // SH clamp bits are stored by a full-image F1 only: a band's F1 evaluates the colour of its
    // own Gaussians alone, and B2 recomputes the bits (stored_flags)
    const bool full = ty0 == 0 && ty1 == div_up(cam->height, kTile);
    PreOut po{radii, v.depth_key, v.tiles, v.rec, v.rect, full ? v.flags : nullptr, v.counters};
    // the row-bucketed binning's pass-A row counts, from F1 itself (fwd_phase2 then skips them)
    if (use_rb_binning(gs->P, div_up(cam->width, kTile), div_up(cam->height, kTile))) {
        po.rb_hist = v.rb_histA;
        po.bsum = v.lookback + 16;  // the F2 scan's block partials (the lookback words are unused here)
    }
    GSR_STAGE(GSR_STAGE_PREPROCESS, launch_preprocess(*cam, gauss_in(gs), ty0, ty1, po, stream), "preprocess");
    return 0;
}

// B1 (+ the per-Gaussian gather into grad2d): shared by every backward entry point.
int blend_backward(const gsr_camera* cam, const gsr_raster_settings* rs, const gsr_buffers* bufs, const float* dL_dpix,
                   gsr_alloc_fn alloc_scratch, void* ctx, float* grad2d, hipStream_t stream, bool debug, int vgy = 0,
                   int vh = 0) {
    if (!bufs || !bufs->geom || !bufs->image || !bufs->binning || !dL_dpix) return fail(-1, "missing forward buffers / dL_dpix");
    if (!grad2d) return fail(-1, "null grad2d");
    const long long n = bufs->n_local, cap = bufs->capacity;
    if (n <= 0) return 0;
    int ty0, ty1;
    band(cam, rs, &ty0, &ty1);
    if (int e = check_layout(cam, ty0, ty1, bufs)) return e;
    const Views v = views(cam, n, bufs);
    if (!alloc_scratch) return fail(-1, "null scratch allocator");
    // band launches split each (tile, chunk) of B1 over `split` waves by stripe, one partial
    // entry per (instance, part)
    int split = b1_split(cam->width, cam->height, ty0, ty1, vgy);
    if (cap * split > (long long)UINT32_MAX) split = 1;  // entry indices are u32
    float* partial = static_cast<float*>(alloc_scratch(ctx, PartLayout(cap * split).total));
    if (!partial) return fail(-2, "allocation failed (scratch, %lld instances)", cap);
    // only the per-entry flag bytes are zeroed: the gather reads the entries B1 flagged
    GSR_STAGE(GSR_STAGE_MISC, launch_clear_flags(partial, cap * split, stream), "clear partial flags");
    GSR_STAGE(GSR_STAGE_BLEND_BWD, launch_blend_backward(*cam, rs->bg, ty0, ty1, v.ranges, v.sorted_gid, v.rect, v.rec,
                                                         v.final_T, v.accum, dL_dpix, partial, cap, v.term, v.ck,
                                                         stream, vgy, vh, v.mk, split),
              "blend backward");
    GSR_STAGE(GSR_STAGE_GATHER, launch_gather_grad2d(v.offsets, partial, v.rec, cam->width, vgy > 0 ? vh : cam->height,
                                                     cap, (int)n,
                                                     v.presort ? v.rrect : nullptr, grad2d, stream, split),
              "gather grad2d");
    return 0;
}

// SH clamp bits for B2: stored by a full-image forward, else nullptr (B2 recomputes them)
const uint32_t* stored_flags(const gsr_camera* cam, const gsr_raster_settings* rs, const uint32_t* flags) {
    int ty0, ty1;
    band(cam, rs, &ty0, &ty1);
    return (ty0 == 0 && ty1 == div_up(cam->height, kTile)) ? flags : nullptr;
}

int check_grads(const gsr_gaussians* gs, const gsr_grads* g) {
    if (!g || !g->dL_dmeans2D || !g->dL_dopacity || !g->dL_dmeans3D) return fail(-1, "missing gradient outputs");
    if (gs->colors_precomp ? !g->dL_dcolors : !g->dL_dsh_dc) return fail(-1, "missing colour/SH gradient output");
    if (!gs->colors_precomp && gs->sh_rest && !g->dL_dsh_rest) return fail(-1, "missing sh_rest gradient output");
    if (gs->cov3D_precomp ? !g->dL_dcov3D : (!g->dL_dscales || !g->dL_drotations))
        return fail(-1, "missing cov3D / scale / rotation gradient output");
    return 0;
}

GradOut grad_out(const gsr_grads* g) {
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

int band_rows_of(int32_t nbands, const int32_t* band_rows, int gy, BandRows& br) {
    if (nbands < 1 || nbands > kMaxBands) return fail(-1, "nbands must be 1..%d (got %d)", kMaxBands, nbands);
    if (!band_rows) return fail(-1, "null band_rows");
    br.n = nbands;
    for (int b = 0; b <= nbands; ++b) {
        br.row[b] = band_rows[b];
        if (band_rows[b] < 0 || band_rows[b] > gy || (b > 0 && band_rows[b] < band_rows[b - 1]))
            return fail(-1, "band_rows must be non-decreasing within [0, %d]", gy);
    }
    if (band_rows[0] != 0 || band_rows[nbands] != gy) return fail(-1, "band_rows must cover tile rows [0, %d)", gy);
    return 0;
}

// Views mode: the tall camera whose tile rows stack the V views' bands (gsr.h gsr_forward_views)
int views_camera(int32_t V, const gsr_camera* cams, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                 gsr_camera* tall) {
    if (V < 1 || V > GSR_MAX_VIEWS || V > kMaxViews) return fail(-1, "views: 1..%d views, got %d", GSR_MAX_VIEWS, V);
    if (!cams) return fail(-1, "views: null cameras");
    for (int v = 0; v < V; ++v) {
        if (int e = validate(&cams[v], gs, rs)) return e;
        if (cams[v].width != cams[0].width || cams[v].height != cams[0].height)
            return fail(-1, "views: every view must be %dx%d (view %d is %dx%d)", cams[0].width, cams[0].height, v,
                        cams[v].width, cams[v].height);
    }
    const int gy = div_up(cams[0].height, kTile);
    if (rs->tile_y0 > 0 || rs->tile_y1 < gy) return fail(-1, "views: full-image views only");
    if ((long long)V * gy >= 65535) return fail(-1, "views: %d views of %d tile rows exceed the tile grid", V, gy);
    if ((long long)V * gs->P > INT32_MAX / 2) return fail(-1, "views: V * P too large");
    *tall = cams[0];
    tall->height = V * gy * kTile;
    return 0;
}

GaussIn shard_in(const gsr_gaussians* gs) { return gauss_in(gs); }

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
size_t gsr_ck_pool_slots(int32_t capacity, int32_t w, int32_t h) {
    return ck_pool_slots(capacity, (long long)ImgLayout::tile_count(w, h));
}
size_t gsr_binning_bytes(int32_t capacity, int32_t w, int32_t h) {
    return BinLayout(capacity, (long long)ImgLayout::tile_count(w, h)).total;
}
size_t gsr_image_bytes(int32_t w, int32_t h) { return ImgLayout(w, h).total; }
size_t gsr_scratch_bytes(int32_t capacity) { return PartLayout(capacity).total; }
size_t gsr_exchange_block_bytes(int32_t pair_cap) { return exchange_block_bytes(pair_cap > 0 ? pair_cap : 0); }
size_t gsr_shard_state_bytes(int32_t P, int32_t nbands, int32_t pair_cap) {
    (void)pair_cap;
    return ShardLayout(P, nbands > 0 ? nbands : 1).total;
}

int gsr_forward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                float* out_color, int32_t* radii, gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_binning,
                gsr_alloc_fn alloc_image, void* ctx, gsr_buffers* bufs, void* stream_) {
    g_err.clear();
    if (int e = validate(cam, gs, rs)) return e;
    if (!out_color || (gs->P > 0 && !radii) || !bufs || !alloc_geom || !alloc_binning || !alloc_image)
        return fail(-1, "null output / allocator");
    if (rs->max_rendered < 0) return fail(-1, "negative max_rendered");
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    FwdJob j{cam, rs, out_color, bufs};
    j.n = gs->P;
    const bool exact = rs->max_rendered == 0;
    if (int e = fwd_phase1(j, alloc_geom, alloc_image, ctx, stream, debug, false, [&](const Views& v) {
            if (int e2 = run_preprocess(cam, gs, j.ty0, j.ty1, radii, v, stream, debug)) return e2;
            j.rows_counted = true;
            // exact sizing: F1's count partials go to the host while the scan runs
            if (exact && gs->P > 0) GSR_CHECK_HIP(begin_read(v.counters, 2 * kCountSlots, stream), "read counts");
            return 0;
        }))
        return e;
    long long cap = rs->max_rendered;
    if (exact) {
        uint64_t ksum = 0;
        if (gs->P > 0) {
            uint32_t cw[2 * kCountSlots];
            const Views v = views(cam, j.n, bufs);
            GSR_STAGE(GSR_STAGE_MISC, end_read(v.counters, cw, 2 * kCountSlots, stream), "read counts");
            for (int i = 0; i < kCountSlots; ++i) ksum += cw[kCountSlots + i];
        }
        if (ksum > (uint64_t)INT32_MAX) return fail(-3, "num_rendered overflow (%llu)", (unsigned long long)ksum);
        cap = (long long)ksum;
        bufs->num_rendered = (int32_t)ksum;
    }
    return fwd_phase2(j, cap, alloc_binning, ctx, stream, debug);
}

int gsr_read_num_rendered(const gsr_camera* cam, const gsr_buffers* bufs, int32_t* num_rendered, void* stream_) {
    g_err.clear();
    if (!cam || !bufs || !bufs->image) return fail(-1, "null camera / buffers");
    hipStream_t stream = (hipStream_t)stream_;
    const Views v = views(cam, bufs->n_local, bufs);
    uint32_t K = 0;
    if (bufs->n_local > 0) {
        if (int e = begin_read(v.K_dev, 1, stream)) return fail(-10, "read K: %s", hipGetErrorString((hipError_t)e));
        if (int e = end_read(v.K_dev, &K, 1, stream)) return fail(-10, "read K: %s", hipGetErrorString((hipError_t)e));
    }
    if (num_rendered) *num_rendered = (int32_t)(K > (uint32_t)INT32_MAX ? INT32_MAX : K);
    if (K == 0xFFFFFFFFu && bufs->capacity < INT32_MAX)
        return fail(GSR_ERR_OVERFLOW, "binning void: the row-bucketed binning's look-back did not complete "
                                      "(K marked UINT32_MAX); re-run the forward");
    if ((long long)K > (long long)bufs->capacity)
        return fail(GSR_ERR_OVERFLOW, "binning overflow: K = %u instances, capacity %d", K, bufs->capacity);
    return 0;
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
    if (rs->max_rendered < 0) return fail(-1, "negative max_rendered");
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    const bool exact = rs->max_rendered == 0;
    std::vector<FwdJob> jobs;
    jobs.reserve(V);
    for (int v = 0; v < V; ++v) {
        if (int e = validate(&cams[v], gs, rs)) return e;
        if (rs->tile_y0 > 0 || rs->tile_y1 < div_up(cams[v].height, kTile))
            return fail(-1, "batch: full-image views only (view %d)", v);
        if (!out_colors[v] || (gs->P > 0 && !radii[v])) return fail(-1, "batch: null output of view %d", v);
        jobs.push_back(FwdJob{&cams[v], rs, out_colors[v], &bufs[v]});
        jobs[v].n = gs->P;
        int32_t* rad = gs->P > 0 ? radii[v] : nullptr;
        if (int e = fwd_phase1(jobs[v], alloc_geom, alloc_image, ctx, stream, debug, false, [&](const Views& vw) {
                jobs[v].rows_counted = true;
                return run_preprocess(&cams[v], gs, jobs[v].ty0, jobs[v].ty1, rad, vw, stream, debug);
            }))
            return e;
    }
    std::vector<long long> cap(V, rs->max_rendered);
    if (exact && gs->P > 0) {
        uint32_t* words = static_cast<uint32_t*>(alloc_image(ctx, 8 * (size_t)V));
        if (!words) return fail(-2, "allocation failed (batch counts)");
        CountPtrs cp{};
        for (int v = 0; v < V; ++v) cp.c[v] = views(&cams[v], gs->P, &bufs[v]).counters;
        hipLaunchKernelGGL(batch_counts_kernel, dim3(V), dim3(64), 0, stream, cp, words);
        GSR_STAGE(GSR_STAGE_MISC, hipGetLastError(), "batch counts");
        uint32_t host[2 * GSR_MAX_BATCH];
        GSR_CHECK_HIP(begin_read(words, 2 * V, stream), "read counts");
        GSR_STAGE(GSR_STAGE_MISC, end_read(words, host, 2 * V, stream), "read counts");
        for (int v = 0; v < V; ++v) {
            const uint64_t K = (uint64_t)host[2 * v] | ((uint64_t)host[2 * v + 1] << 32);
            if (K > (uint64_t)INT32_MAX) return fail(-3, "num_rendered overflow (view %d)", v);
            cap[v] = (long long)K;
            bufs[v].num_rendered = (int32_t)K;
        }
    } else if (exact) {
        for (int v = 0; v < V; ++v) cap[v] = 0, bufs[v].num_rendered = 0;
    }
    for (int v = 0; v < V; ++v)
        if (int e = fwd_phase2(jobs[v], cap[v], alloc_binning, ctx, stream, debug)) return e;
    return 0;
}

int gsr_forward_views(int32_t V, const gsr_camera* cams, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                      float* out_color, int32_t* radii, gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_binning,
                      gsr_alloc_fn alloc_image, void* ctx, gsr_buffers* bufs, void* stream_) {
    g_err.clear();
    if (!gs || !rs) return fail(-1, "null gaussians/settings");
    gsr_camera tall;
    if (int e = views_camera(V, cams, gs, rs, &tall)) return e;
    if (!out_color || (gs->P > 0 && !radii) || !bufs || !alloc_geom || !alloc_binning || !alloc_image)
        return fail(-1, "null output / allocator");
    if (rs->max_rendered < 0) return fail(-1, "negative max_rendered");
    gsr_raster_settings rv = *rs;  // the whole tall image
    rv.tile_y0 = 0;
    rv.tile_y1 = INT32_MAX;
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    FwdJob j{&tall, &rv, out_color, bufs};
    j.n = (long long)V * gs->P;
    j.vgy = div_up(cams[0].height, kTile);
    j.vh = cams[0].height;
    const bool exact = rs->max_rendered == 0;
    if (int e = fwd_phase1(j, alloc_geom, alloc_image, ctx, stream, debug, false, [&](const Views& v) {
            if (gs->P <= 0) return 0;
            PreOut po{radii, v.depth_key, v.tiles, v.rec, v.rect, v.flags, v.counters};
            GSR_STAGE(GSR_STAGE_PREPROCESS, launch_preprocess_views(cams, V, gauss_in(gs), po, stream),
                      "preprocess (views)");
            if (exact) GSR_CHECK_HIP(begin_read(v.counters, 2 * kCountSlots, stream), "read counts");
            return 0;
        }))
        return e;
    long long cap = rs->max_rendered;
    if (exact) {
        uint64_t ksum = 0;
        if (gs->P > 0) {
            uint32_t cw[2 * kCountSlots];
            const Views v = views(&tall, j.n, bufs);
            GSR_STAGE(GSR_STAGE_MISC, end_read(v.counters, cw, 2 * kCountSlots, stream), "read counts");
            for (int i = 0; i < kCountSlots; ++i) ksum += cw[kCountSlots + i];
        }
        if (ksum > (uint64_t)INT32_MAX) return fail(-3, "num_rendered overflow (%llu)", (unsigned long long)ksum);
        cap = (long long)ksum;
        bufs->num_rendered = (int32_t)ksum;
    }
    return fwd_phase2(j, cap, alloc_binning, ctx, stream, debug);
}

int gsr_backward_views(int32_t V, const gsr_camera* cams, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                       const gsr_buffers* bufs, const float* dL_dpix, gsr_alloc_fn alloc_scratch, void* ctx,
                       const gsr_grads* grads, void* stream_) {
    g_err.clear();
    if (!gs || !rs) return fail(-1, "null gaussians/settings");
    gsr_camera tall;
    if (int e = views_camera(V, cams, gs, rs, &tall)) return e;
    if (gs->P == 0) return 0;
    if (int e = check_grads(gs, grads)) return e;
    const long long n = (long long)V * gs->P;
    if (!bufs || bufs->n_local != n) return fail(-1, "forward buffers do not match V * P view entries");
    if (int e = check_layout(&tall, 0, div_up(tall.height, kTile), bufs)) return e;
    if (!alloc_scratch) return fail(-1, "null scratch allocator");
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    gsr_raster_settings rv = *rs;
    rv.tile_y0 = 0;
    rv.tile_y1 = INT32_MAX;
    float* grad2d = static_cast<float*>(alloc_scratch(ctx, sizeof(float) * kPart * (size_t)n));
    if (!grad2d) return fail(-2, "allocation failed (grad2d, %lld entries)", n);
    if (int e = blend_backward(&tall, &rv, bufs, dL_dpix, alloc_scratch, ctx, grad2d, stream, debug,
                               div_up(cams[0].height, kTile), cams[0].height))
        return e;
    const GaussIn in = gauss_in(gs);
    const GradOut out = grad_out(grads);
    // leaf-gradient slices of views 1..V-1 (only the arrays the caller asked for)
    GradOut scratch{};
    if (V > 1) {
        const size_t P = (size_t)gs->P, k = (size_t)(V - 1) * P;
        const size_t widths[8] = {1, 3, 3, 3, 3 * (size_t)in.M_rest, 3, 4, 6};
        float* const dst[8] = {out.opac, out.colors, out.means3D, out.sh_dc, out.sh_rest, out.scales, out.rots,
                               out.cov3D};
        size_t total = 0;
        for (int a = 0; a < 8; ++a) total += dst[a] ? widths[a] * k : 0;
        float* base = static_cast<float*>(alloc_scratch(ctx, sizeof(float) * (total > 0 ? total : 1)));
        if (!base) return fail(-2, "allocation failed (per-view leaf gradients)");
        float** const slot[8] = {&scratch.opac, &scratch.colors, &scratch.means3D, &scratch.sh_dc, &scratch.sh_rest,
                                 &scratch.scales, &scratch.rots, &scratch.cov3D};
        for (int a = 0; a < 8; ++a)
            if (dst[a]) {
                *slot[a] = base;
                base += widths[a] * k;
            }
    }
    const Views v = views(&tall, n, bufs);
    GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_preprocess_backward_views(cams, V, in, v.depth_key, v.flags, grad2d, out,
                                                                         scratch, stream),
              "preprocess backward (views)");
    if (V > 1) GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_views_sum(in, V, out, scratch, stream), "views sum");
    return 0;
}

int gsr_backward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                 const gsr_buffers* bufs, const float* dL_dpix, gsr_alloc_fn alloc_scratch, void* ctx,
                 const gsr_grads* grads, void* stream_) {
    g_err.clear();
    if (int e = validate(cam, gs, rs)) return e;
    if (gs->P == 0) return 0;
    if (int e = check_grads(gs, grads)) return e;
    if (!bufs || bufs->n_local != gs->P) return fail(-1, "forward buffers do not match the Gaussians");
    {
        int ty0, ty1;
        band(cam, rs, &ty0, &ty1);
        if (int e = check_layout(cam, ty0, ty1, bufs)) return e;  // before any allocation
    }
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    if (!alloc_scratch) return fail(-1, "null scratch allocator");
    float* grad2d = static_cast<float*>(alloc_scratch(ctx, sizeof(float) * kPart * (size_t)gs->P));
    if (!grad2d) return fail(-2, "allocation failed (grad2d, P=%d)", gs->P);
    if (int e = blend_backward(cam, rs, bufs, dL_dpix, alloc_scratch, ctx, grad2d, stream, debug)) return e;
    const Views v = views(cam, gs->P, bufs);
    GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_preprocess_backward(*cam, gauss_in(gs), 0, gs->P, v.depth_key,
                                                                   stored_flags(cam, rs, v.flags), grad2d,
                                                                   grad_out(grads), stream),
              "preprocess backward");
    return 0;
}

int gsr_backward_blend(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                       const gsr_buffers* bufs, const float* dL_dpix, gsr_alloc_fn alloc_scratch, void* ctx,
                       float* grad2d, void* stream_) {
    g_err.clear();
    if (int e = validate(cam, gs, rs)) return e;
    if (gs->P == 0) return 0;
    if (!bufs || bufs->n_local != gs->P) return fail(-1, "forward buffers do not match the Gaussians");
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    return blend_backward(cam, rs, bufs, dL_dpix, alloc_scratch, ctx, grad2d, (hipStream_t)stream_, debug);
}

int gsr_backward_preprocess(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                            const gsr_buffers* bufs, const float* grad2d, const gsr_grads* grads, void* stream_) {
    g_err.clear();
    if (int e = validate(cam, gs, rs)) return e;
    if (gs->P == 0) return 0;
    if (int e = check_grads(gs, grads)) return e;
    if (!bufs || !bufs->geom || !grad2d) return fail(-1, "missing forward buffers / grad2d");
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    const GeomLayout gl(gs->P);
    GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_preprocess_backward(*cam, gauss_in(gs), 0, gs->P,
                                                                   at<uint32_t>(bufs->geom, gl.depth_key),
                                                                   stored_flags(cam, rs, at<uint32_t>(bufs->geom, gl.flags)),
                                                                   grad2d, grad_out(grads), stream),
              "preprocess backward");
    return 0;
}

// ---- multi-GPU: Gaussian shards x tile-row bands ----
int gsr_shard_forward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs, int32_t nbands,
                      const int32_t* band_rows, int32_t pair_cap, void* send, int32_t* radii, void* shard_state,
                      uint32_t* row_hist, void* stream_) {
    g_err.clear();
    if (int e = validate(cam, gs, rs)) return e;
    if (pair_cap < 0 || !send || !shard_state || (gs->P > 0 && !radii)) return fail(-1, "shard: null buffer / bad pair_cap");
    const int gy = div_up(cam->height, kTile);
    if (row_hist && gy > kMaxHistRows) return fail(-1, "shard: row histogram holds at most %d tile rows", kMaxHistRows);
    BandRows br;
    if (int e = band_rows_of(nbands, band_rows, gy, br)) return e;
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    const int P = gs->P;
    const ShardLayout sl(P, nbands);
    const GeomLayout& gl = sl.geo;
    uint32_t* depth_key = at<uint32_t>(shard_state, gl.depth_key);
    uint32_t* tiles = at<uint32_t>(shard_state, gl.tiles);
    float4* rec = at<float4>(shard_state, gl.rec);
    uint4* rect = at<uint4>(shard_state, gl.rect);
    if (P > 0) {
        PreOut po{radii, depth_key, tiles, rec, rect, at<uint32_t>(shard_state, gl.flags), nullptr};
        GSR_STAGE(GSR_STAGE_PREPROCESS, launch_preprocess(*cam, shard_in(gs), 0, gy, po, stream), "preprocess");
    }
    GSR_STAGE(GSR_STAGE_EXCHANGE, launch_pack_splats(tiles, rect, depth_key, rec, P, br,
                                                     at<uint32_t>(shard_state, sl.partials), static_cast<char*>(send),
                                                     pair_cap, at<uint32_t>(shard_state, sl.slot_of), row_hist, gy,
                                                     (rs->flags & GSR_FLAG_ROW_SPANS) != 0, stream,
                                                     at<uint32_t>(shard_state, gl.rb_hist)),
              "pack splats");
    return 0;
}

int gsr_band_forward(const gsr_camera* cam, const gsr_raster_settings* rs, int32_t nsrc, int32_t pair_cap,
                     const void* recv, float* out_color, gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_binning,
                     gsr_alloc_fn alloc_image, void* ctx, gsr_buffers* bufs, void* stream_) {
    g_err.clear();
    if (!cam || !rs) return fail(-1, "null camera / settings");
    if (nsrc < 1 || nsrc > kMaxBands || pair_cap < 0) return fail(-1, "band: bad nsrc / pair_cap");
    if (!recv || !out_color || !bufs || !alloc_geom || !alloc_binning || !alloc_image)
        return fail(-1, "band: null buffer / allocator");
    if (rs->max_rendered <= 0) return fail(-1, "band: max_rendered (the band's instance capacity) is required");
    const long long n = (long long)nsrc * pair_cap;
    if (n > INT32_MAX) return fail(-1, "band: nsrc * pair_cap too large");
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    FwdJob j{cam, rs, out_color, bufs};
    j.n = n;
    if (int e = fwd_phase1(j, alloc_geom, alloc_image, ctx, stream, debug, true, [&](const Views& v) {
            // the row-bucketed binning's pass-A counts and the F2 block sums come with the unpack
            const bool rb = use_rb_binning(j.n, j.gx, j.gy);
            GSR_STAGE(GSR_STAGE_EXCHANGE, launch_unpack_splats(static_cast<const char*>(recv), nsrc, pair_cap, j.ty0,
                                                               j.ty1, v.rec, v.depth_key, v.tiles, v.rect, stream,
                                                               rb ? v.rb_histA : nullptr, rb ? v.lookback + 16 : nullptr),
                      "unpack splats");
            j.rows_counted = rb;
            return 0;
        }))
        return e;
    return fwd_phase2(j, rs->max_rendered, alloc_binning, ctx, stream, debug);
}

int gsr_band_backward(const gsr_camera* cam, const gsr_raster_settings* rs, int32_t nsrc, int32_t pair_cap,
                      const gsr_buffers* bufs, const float* dL_dpix, gsr_alloc_fn alloc_scratch, void* ctx,
                      void* grad_send, void* stream_) {
    g_err.clear();
    if (!cam || !rs || !bufs || !grad_send) return fail(-1, "band backward: null argument");
    if ((long long)nsrc * pair_cap != bufs->n_local) return fail(-1, "band backward: nsrc * pair_cap != the forward's");
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    return blend_backward(cam, rs, bufs, dL_dpix, alloc_scratch, ctx, static_cast<float*>(grad_send),
                          (hipStream_t)stream_, debug);
}

int gsr_shard_backward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs, int32_t nbands,
                       const int32_t* band_rows, int32_t pair_cap, void* shard_state, const void* grad_recv,
                       const gsr_grads* grads, void* stream_) {
    g_err.clear();
    if (int e = validate(cam, gs, rs)) return e;
    if (gs->P == 0) return 0;
    if (int e = check_grads(gs, grads)) return e;
    if (!shard_state || !grad_recv || pair_cap < 0) return fail(-1, "shard backward: null buffer / bad pair_cap");
    BandRows br;
    if (int e = band_rows_of(nbands, band_rows, div_up(cam->height, kTile), br)) return e;
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    const int P = gs->P;
    const ShardLayout sl(P, nbands);
    const GeomLayout& gl = sl.geo;
    const uint32_t* tiles = at<uint32_t>(shard_state, gl.tiles);
    const uint4* rect = at<uint4>(shard_state, gl.rect);
    // B2 sums the bands' returned rows itself (no grad2d round trip, one launch fewer)
    BandSum bs{tiles, rect, at<uint32_t>(shard_state, sl.slot_of), static_cast<const float4*>(grad_recv), pair_cap, br};
    GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_preprocess_backward_banded(*cam, shard_in(gs),
                                                                          at<uint32_t>(shard_state, gl.depth_key),
                                                                          at<uint32_t>(shard_state, gl.flags), bs,
                                                                          grad_out(grads), stream),
              "preprocess backward (band sum)");
    return 0;
}

int gsr_band_publish(const gsr_camera* cam, const gsr_raster_settings* rs, int32_t tall, const float* out_color,
                     int32_t nbands, const void* send, int32_t pair_cap, const gsr_buffers* bufs, float* row,
                     int64_t status_off, void* stream_) {
    g_err.clear();
    if (!cam || !rs || !out_color || !send || !bufs || !bufs->image || !row) return fail(-1, "publish: null argument");
    if (cam->width <= 0 || cam->height <= 0) return fail(-1, "publish: bad image size");
    if (nbands < 1 || nbands > kMaxBands || pair_cap < 0) return fail(-1, "publish: bad nbands / pair_cap");
    int ty0, ty1;
    band(cam, rs, &ty0, &ty1);
    const int py0 = std::min(ty0 * kTile, cam->height), py1 = std::min(ty1 * kTile, cam->height);
    if (tall < py1 - py0) return fail(-1, "publish: tall (%d) below the band's %d pixel rows", tall, py1 - py0);
    if (status_off < 3LL * tall * cam->width) return fail(-1, "publish: status words overlap the pixels");
    const ImgLayout il(cam->width, cam->height);
    const uint32_t* K_dev = at<uint32_t>(bufs->image, il.counters) + kTotalSlot;
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = (rs->flags & GSR_FLAG_DEBUG) != 0;
    GSR_STAGE(GSR_STAGE_EXCHANGE, launch_band_publish(out_color, cam->width, cam->height, py0, py1, tall, row,
                                                      status_off, static_cast<const char*>(send),
                                                      exchange_block_bytes(pair_cap), nbands, K_dev, stream),
              "band publish");
    return 0;
}

int gsr_gather_finish(const gsr_camera* cam, int32_t world, const int32_t* band_rows, int32_t tall,
                      const float* gathered, int64_t row_floats, int64_t status_off, int32_t pair_cap,
                      int32_t capacity, float* image, int32_t* guard, float* zero, int64_t nzero, void* stream_) {
    g_err.clear();
    if (!cam || !gathered || !image || !guard || (nzero > 0 && !zero)) return fail(-1, "gather finish: null argument");
    if (cam->width <= 0 || cam->height <= 0) return fail(-1, "gather finish: bad image size");
    BandRows br;
    if (int e = band_rows_of(world, band_rows, div_up(cam->height, kTile), br)) return e;
    for (int r = 0; r < world; ++r)
        if (std::min(br.row[r + 1] * kTile, cam->height) - std::min(br.row[r] * kTile, cam->height) > tall)
            return fail(-1, "gather finish: band %d is taller than tall (%d)", r, tall);
    if (status_off < 3LL * tall * cam->width || status_off + world + 1 > row_floats || nzero < 0 || nzero > INT32_MAX)
        return fail(-1, "gather finish: bad row layout");
    hipStream_t stream = (hipStream_t)stream_;
    const bool debug = false;
    GSR_STAGE(GSR_STAGE_EXCHANGE, launch_gather_finish(gathered, row_floats, status_off, world, br, cam->width,
                                                       cam->height, tall, image, (uint32_t)std::max(pair_cap, 0),
                                                       (uint32_t)std::max(capacity, 0), guard, zero, (int)nzero,
                                                       stream),
              "gather finish");
    return 0;
}

int gsr_profile_enable(uint32_t stage_mask) {
    Profiler& p = prof();
    std::lock_guard<std::mutex> lk(p.mu);
    for (auto& r : p.pending) {
        (void)hipEventSynchronize(r.b);
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
                                               "gather_grad2d", "misc", "exchange"};
    return (stage >= 0 && stage < GSR_NUM_STAGES) ? names[stage] : "?";
}

const void* gsr_view(const gsr_camera* cam, int32_t P, const gsr_buffers* bufs, int what) {
    g_err.clear();
    if (!cam || !bufs || !bufs->geom || !bufs->image) return nullptr;
    if ((bufs->layout & GSR_LAYOUT_TAG_MASK) != GSR_LAYOUT_TAG) {
        fail(GSR_ERR_LAYOUT, "gsr_view: gsr_buffers.layout = 0x%08x is not a forward's", bufs->layout);
        return nullptr;
    }
    const Views v = views(cam, bufs->n_local > 0 ? bufs->n_local : P, bufs);
    switch (what) {
        case GSR_VIEW_SORTED_GID: return v.sorted_gid;
        case GSR_VIEW_SORTED_TILE:
            if (v.rb && !GSR_RB_TILE_KEYS && bufs->binning && bufs->capacity > 0) {
                // filled here from the ranges between two device-wide waits: the forward may have
                // run on any stream, blocking or not (a torch pool stream, torch.cuda.stream(s)), and
                // the null stream alone is not ordered after a non-blocking one; both
                // waits fail during a stream capture, and the accessor then returns NULL
                if (hipDeviceSynchronize() != hipSuccess ||
                    launch_tile_keys_from_ranges(v.ranges, ImgLayout::tile_count(cam->width, cam->height),
                                                 bufs->capacity, v.sorted_tile, nullptr) ||
                    hipDeviceSynchronize() != hipSuccess) {
                    fail(-10, "gsr_view(GSR_VIEW_SORTED_TILE): device synchronisation failed (stream capture?)");
                    return nullptr;
                }
            }
            return v.sorted_tile;
        case GSR_VIEW_RANGES: return v.ranges;
        case GSR_VIEW_FINAL_T: return v.final_T;
        case GSR_VIEW_N_CONTRIB: return nullptr;  // retired: B1 re-derives termination from T
        case GSR_VIEW_DEPTH_KEY: return v.depth_key;
        case GSR_VIEW_TILES_TOUCHED: return v.tiles;
        case GSR_VIEW_RECORDS: return v.rec;
        case GSR_VIEW_COUNTS: return v.K_dev;
        case GSR_VIEW_TERM: return v.term;
        case GSR_VIEW_CK_LIVE:
            if (!bufs->binning) return nullptr;
            return static_cast<const char*>(bufs->binning) +
                   BinLayout(bufs->capacity, (long long)ImgLayout::tile_count(cam->width, cam->height)).ckm;
        default: return nullptr;
    }
}

}  // extern "C"

// gsr_blend.hip -- F6 per-tile front-to-back alpha blend and B1 per-tile front-to-back
// gradient pass on gfx950.
//
// Pixel layout: a 16x16 tile is four 16x4 stripes; lane l of a wave owns column l&15 and
// row (l>>4) of each stripe it covers.  F6 runs NW waves per tile (NW = 2 shipped: wave w
// owns stripes 2w, 2w+1); B1 runs one wave per tile (all four stripes, so each record's
// per-pixel terms are reduced once).  Batches of records are gathered one record per
// thread (3 dwordx4 loads), staged in LDS with a per-record stripe mask, and swept by every
// lane; a record whose alpha >= 1/255 footprint misses a stripe is skipped for that stripe
// by a wave-uniform branch (exact: the skipped pixels fail the alpha test).
//
// Both kernels are VALU-issue-bound (a wave64 VALU op costs 4 cycles of its SIMD, exp/rcp 8;
// MI355X_MICROARCH 'vector-instruction ISSUE cost'), so the per-(pixel, record) stream is
// kept short: log2(o) is folded into the exponent (o G = exp2(power + log2 o)), the
// column-only part of the quadratic form is hoisted per record, termination is encoded in
// the sign of T (no contributor count, no separate final-T register), and B1 accumulates
// per lane only the row moments (sum sv, sum sv dy, sum sv dy^2) -- the dx factors are
// applied once per record because dx is constant along a lane's column.
//
// Workgroup -> tile mapping is XCD-aware: blocks b, b+8, ... land on one XCD (observed
// round-robin dispatch, speed only), so each XCD gets a contiguous band of tile rows and
// its L2 keeps the records those neighbouring tiles share.
//
// B1 reduces each record's 9 raw moments over the tile's 256 pixels: 4 pixels per lane in
// registers, a 2-step quad DPP reduction, then the 16 quad partials wait in LDS and are summed
// four records at a time (one (record, moment) output per lane, stored straight to HBM) --
// ~40% fewer VALU ops than a full 64-lane DPP/permlane reduction per record, and no per-batch
// moment buffer in LDS (more waves per SIMD).  It writes ONE 36-B partial per contributing
// (tile, instance) with plain stores, indexed by the instance's emission index j, and sets that
// entry's flag byte; the gather reads flagged entries only (the launcher zeroes the K flag bytes,
// never the 36-B entries), and a tile stops at the first batch whose pixels have all terminated.
//
// Measured and rejected (experiments are separate builds,
// _build.build_variant + scripts/ab.sh): packing two stripes per VGPR pair (v_pk_fma_f32 issues
// 2 FMAs in 4 cycles -- no gain over v_fma_f32 on gfx950, and the register shuffles cost extra);
// 4 waves per tile; record prefetch into registers.  The per-Gaussian sum happens later in fixed
// emission order (gsr_preprocess_bwd.hip), so gradients are deterministic and no float atomics
// are issued.
#include "gsr_kernels.h"

namespace gsr {
namespace {

constexpr int kPPL = 4;  // pixels per lane

__device__ inline int xcd_tile(int b, int nwg) {
    // bijective remap: the blocks one XCD receives (b % 8 equal) -> a contiguous tile range
    const int q = nwg / 8, r = nwg % 8;
    const int xcd = b % 8, local = b / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

template <int CTRL>
__device__ inline float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// Quad (4-lane) all-reduce of N values.  The empty asm pins each sum in the block that
// computes it: without it the compiler sinks the second add into the quad leaders' branch,
// the DPP move can no longer fuse into it, and each value costs a zero move, a DPP move and
// an add instead of one v_add_f32_dpp (2N extra VALU ops per record).
template <int N>
__device__ __forceinline__ void quad_reduce(float (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dpp_f<0xB1>(v[i]);  // quad_perm [1,0,3,2]
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dpp_f<0x4E>(v[i]);  // quad_perm [2,3,0,1]
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}



struct BlendGeom {
    int W, H, grid_x, ty0, nwg;
    // views mode (gsr_forward_views): the image is V views stacked as bands of vgy tile rows;
    // a tile's pixel y is taken relative to its view's band (records are in view coordinates)
    // and rows at or past vh inside a band are padding.  One image: vgy = all rows, vh = H.
    int vgy, vh;
    uint32_t ck_slots;  // checkpoint slots (gsr_internal.h); the live bytes follow the float4 slots
    int ck_fixed;       // 1: slot = tile * 31 + chunk - 1; 0: from the tile's start in the list
    float bg0, bg1, bg2;
    uint32_t cap;       // the binning's capacity: B1 writes partial entries j < cap only
};

// Which of the tile's four 16x4 pixel stripes (slot p = rows 4p..4p+3) can hold a pixel
// with alpha >= 1/255.  Two conservative tests, both on the record the loading lane holds:
//  1. the padded footprint box (ext_x, ext_y) must overlap the stripe;
//  2. the footprint ellipse itself must reach the stripe's pixel-centre rectangle: with the
//     PD form Q(d) = -(a' dx^2 + b' dx dy + c' dy^2) (the exponent without log2 o), a pixel
//     passes alpha >= 1/255 iff Q <= log2(255 o), so the stripe is needed iff the minimum of Q
//     over the rectangle (0 if the mean is inside, else the minimum over its four edges,
//     each a clamped 1-D quadratic) is within that bound -- padded by 2 % + 0.05 for float
//     rounding.  Records whose form is not negative definite keep the box test only.
// Exact culling: a skipped stripe has no pixel that the per-pixel test would accept, so no
// output bit changes; the ellipse test removes ~22 % of the box test's stripe evaluations
// and ~17 % of the visited records at 1M/1080p (scripts/cull_stats.py).
// min over v in [v0, v1] of a u^2 + b u v + c v^2 (c > 0), given k = -b / (2c): the minimiser
// k u clamped to the edge.  k comes from a hardware reciprocal (1 ulp), not an IEEE division
// (~11 instructions each, 16 per record): a minimiser off by a few ulp raises q by c d^2, far
// inside the 2 % + 0.05 pad, and any point of the edge bounds the minimum from above only by
// that amount, so the test stays conservative.
__device__ __forceinline__ float edge_min_q(float a, float b, float c, float k, float u, float v0, float v1) {
    const float vs = fminf(fmaxf(k * u, v0), v1);
    return fmaf(fmaf(c, vs, b * u), vs, a * u * u);
}

__device__ inline uint32_t stripe_mask(const float4 r0, const float4 r1, const float4 r2, float bx0, float by0) {
    const float ex = r2.y, ey = r2.z;
    if (!(ex >= 0.0f) || r0.x + ex < bx0 || r0.x - ex > bx0 + 15.0f) return 0u;
    const float ylo = r0.y - ey, yhi = r0.y + ey;
    // PD form coefficients (A dx^2 + B dx dy + C dy^2) and the log2-domain bound
    const float A = -r0.z, B = -r0.w, C = -r1.x;
    const bool pd = A > 0.0f && C > 0.0f && 4.0f * A * C - B * B > 0.0f;
    const float bound = fmaf(fmaxf(r2.w + 7.99435343f, 0.0f), 1.02f, 0.05f);  // log2(255 o)
    const float x0 = bx0 - r0.x, x1 = bx0 + 15.0f - r0.x;  // rect in mean-relative coords
    const float kc = -B * __builtin_amdgcn_rcpf(2.0f * C), ka = -B * __builtin_amdgcn_rcpf(2.0f * A);
    uint32_t m = 0;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const float s0 = by0 + 4.0f * p;
        bool hit = yhi >= s0 && ylo <= s0 + 3.0f;
        if (hit && pd) {
            const float y0 = s0 - r0.y, y1 = s0 + 3.0f - r0.y;
            const bool inside = x0 <= 0.0f && x1 >= 0.0f && y0 <= 0.0f && y1 >= 0.0f;
            const float q = fminf(fminf(edge_min_q(A, B, C, kc, x0, y0, y1), edge_min_q(A, B, C, kc, x1, y0, y1)),
                                  fminf(edge_min_q(C, B, A, ka, y0, x0, x1), edge_min_q(C, B, A, ka, y1, x0, x1)));
            hit = inside || q <= bound;
        }
        m |= hit ? (1u << p) : 0u;
    }
    return m;
}

// alpha of one (pixel, record) pair, with the reference's two rejections folded into the
// select: power > 0 (here: exponent above log2 o) and alpha < 1/255 give 0.
__device__ __forceinline__ float pair_alpha(float e, float L, float& oG) {
    oG = __builtin_amdgcn_exp2f(e);
    const float a = __builtin_amdgcn_fmed3f(oG, 0.0f, 0.99f);  // = min(0.99, oG): oG >= 0
    return (e <= L && oG >= (1.0f / 255.0f)) ? a : 0.0f;
}

// Same alpha, plus the keep predicate itself: keep implies alpha >= 1/255 > 0 and !keep gives
// alpha = 0, so B1 tests `keep` (an SGPR mask it already has) instead of re-comparing alpha > 0.
__device__ __forceinline__ float pair_alpha_keep(float e, float L, float& oG, bool& keep) {
    oG = __builtin_amdgcn_exp2f(e);
    keep = e <= L && oG >= (1.0f / 255.0f);
    return keep ? __builtin_amdgcn_fmed3f(oG, 0.0f, 0.99f) : 0.0f;
}

// B1 chunk size in (record, stripe) pairs it will visit (see kMaxChunks).  One pair is one
// 64-lane evaluation in B1; a tile's front 48 records with four live stripes are 192.  Measured
// at 1M / 1080p (B1 ms, F6 WRITE_SIZE MB incl. 58 MB of image): 128: 0.467, 187; 192: 0.466,
// 175; 256: 0.473, 141; 384: 0.481, ~115; 512: 0.501, 100; 768: 0.526, 87.  F6's time does not
// move with its checkpoint writes (0.253-0.259 ms across the range: they overlap the blend),
// B1's does, so the bound is set for B1.  At 5M / 1080p: 128: 0.488, 256: 0.492, 512: 0.524.
// (kChunkWork / GSR_CHUNK_WORK and the band launches' GSR_BAND_CHUNK_WORK: gsr_internal.h)

// F6.  T > 0: pixel live; T <= 0: done, |T| = final transmittance (the T after the last
// contributor -- the reference's final_T).  A pair is blended when the next transmittance
// T - alpha T (the reference's T (1 - alpha), one op shorter) is >= 1e-4; otherwise the pixel
// terminates with T unchanged (SURVEY B.3 / forward.cu renderCUDA).  The exponent is
// Horner-form: ((c' dy + b' dx) dy) + (a' dx^2 + log2 o), 3 ops per stripe with dy.
#ifndef GSR_F6_ONESYNC
#define GSR_F6_ONESYNC 1
#endif
#ifndef GSR_CK_MERGE
#define GSR_CK_MERGE 1
#endif
#ifndef GSR_CK_MERGE_BATCH_END
#define GSR_CK_MERGE_BATCH_END 0
#endif
#ifndef GSR_F6_BATCH4
#define GSR_F6_BATCH4 256
#endif
#ifndef GSR_F6_GID_AHEAD
#define GSR_F6_GID_AHEAD 1
#endif
// two-wave (full-image) F6 held to 8 waves per SIMD (64 VGPRs): the gid-ahead register would
// otherwise take it to 65 and 7 waves
#ifndef GSR_F6_WPE
#define GSR_F6_WPE 8
#endif
template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW == 2 ? GSR_F6_WPE : 1))) void blend_forward_kernel(const BlendGeom geo,
                                                                const uint2* __restrict__ ranges,
                                                                const uint32_t* __restrict__ sorted_gid,
                                                                const float4* __restrict__ rec,
                                                                float* __restrict__ out_color,
                                                                float* __restrict__ final_T,
                                                                float* __restrict__ accum,
                                                                uint32_t* __restrict__ term,
                                                                float4* __restrict__ ck,
                                                                uint8_t* __restrict__ mk) {
    constexpr int PPL = kPPL / NW;
    // records per batch: one per thread, or (GSR_F6_BATCH4 = 128) four waves sharing the two-wave
    // kernel's 128-record batches -- the same live-stripe refresh points, so the same chunks
    constexpr int BATCH = NW > 2 ? GSR_F6_BATCH4 : 64 * NW;
    static_assert(BATCH % 64 == 0 && BATCH <= 64 * NW, "F6 batch");
    constexpr int kCW = NW > 2 ? kBandChunkWork : kChunkWork;
    __shared__ float4 srec[BATCH * 3];
    __shared__ uint32_t smk[BATCH];
    __shared__ uint32_t slive[NW];
    const int tl = xcd_tile(blockIdx.x, geo.nwg);  // band-local tile index
    const int tile = tl + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const int view = ty / geo.vgy, tyl = ty - view * geo.vgy;  // tile row inside its view's band
    const float bx0 = (float)(tx * kTile), by0 = (float)(tyl * kTile);
    float pfy[PPL], T[PPL], C0[PPL], C1[PPL], C2[PPL];
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
        const int pyl = tyl * kTile + (lane >> 4) + 4 * (w * PPL + p);
        pfy[p] = (float)pyl;
        T[p] = (px < geo.W && pyl < geo.vh) ? 1.0f : -1.0f;
        C0[p] = C1[p] = C2[p] = 0.0f;
    }
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    // B1 chunk checkpoints: (T, colour sum) of every pixel where a chunk starts.  `work` counts
    // the (record, stripe) pairs of the current chunk: a record's stripe mask against the stripes
    // live (anywhere in the tile) at the start of its batch -- block-uniform, so every wave takes
    // the same chunk decisions, including a wave whose own pixels have all finished (it keeps
    // writing its final state at the later checkpoints).
    uint32_t* const table = term + (size_t)tl * kMaxChunks;  // [term, chunk 1.. starts]
    int nck = 0;   // checkpoints written
    int work = 0;  // pairs in the current chunk
    int tend = n;  // termination index: every pixel of the tile has finished before record tend
    // A stripe with no live pixel (its `live` bit clear: conservative, the bit is cleared only
    // once every T <= 0) is not written; its byte tells B1 to start it dead (T = -1), which is
    // all B1 needs of a finished pixel.
    uint8_t* const ckm = reinterpret_cast<uint8_t*>(ck + (size_t)geo.ck_slots * 256);
    auto checkpoint = [&](size_t slot, uint32_t lv) {
        float4* dst = ck + (size_t)slot * 256;
#pragma unroll
        for (int p = 0; p < PPL; ++p) {
            const bool on = (lv >> p) & 1u;  // wave-uniform
            if (on) dst[64 * (w * PPL + p) + lane] = make_float4(T[p], C0[p], C1[p], C2[p]);
            if (lane == 0) ckm[4 * (size_t)slot + w * PPL + p] = on ? 1 : 0;
        }
    };
#if GSR_CK_MERGE
    // Chunk merging.  When all kMaxChunks - 1 chunk starts are taken and the current chunk is
    // full, neighbouring chunks are merged pairwise (the even starts are kept: chunk k of the
    // merged table is chunk 2k of the old one, its checkpoint moved to slot k) and the quota
    // doubles, so B1's chunks stay within ~2x of each other in work however long the list --
    // without it the last chunk of a deep tile takes all the remaining work (after an opacity
    // reset nothing terminates: 624 of 4160 tiles at 6M / 1280x832 had a 50k-entry last chunk,
    // B1 7.9 ms of a 15.6 ms iteration).  Each thread moves exactly the checkpoint words it
    // wrote (same index map as `checkpoint`), and slot k is read (as the source of k / 2)
    // before it is overwritten, so the moves need no barrier.
    int quota = kCW;
    auto merge_chunks = [&]() {
        constexpr int kKeep = (kMaxChunks - 1) / 2;
        // a tile's chunk slots are consecutive in both layouts: chunk c at ck_slot_of(.., 1) + c - 1
        float4* const ckt = ck + ck_slot_of(geo.ck_fixed, range.x, tl, 1) * 256 - 256;
        uint8_t* const ckmt = ckm + (ck_slot_of(geo.ck_fixed, range.x, tl, 1) - 1) * 4;
#pragma unroll 1
        for (int k = 1; k <= kKeep; ++k) {
#pragma unroll 1
            for (int p = 0; p < PPL; ++p) {
                const int i = 64 * (w * PPL + p) + lane;
                ckt[256 * k + i] = ckt[512 * k + i];
                if (lane == 0) ckmt[4 * k + w * PPL + p] = ckmt[8 * k + w * PPL + p];
            }
            if (tid == 0) table[k] = table[2 * k];
        }
        nck = kKeep;
        work += quota;  // the merged current chunk: old chunk 2 kKeep (>= one quota) + the open one
        quota *= 2;
    };
#else
    constexpr int quota = kCW;
#endif
    // GSR_F6_GID_AHEAD: each batch's gid is loaded one batch ahead (one VGPR), so a batch start
    // waits for its record loads only, not for the gid load they depend on as well
    uint32_t g_next = GSR_F6_GID_AHEAD && tid < BATCH && tid < n ? sorted_gid[range.x + tid] : 0u;
    for (int base = 0; base < n; base += BATCH) {
        uint32_t live = 0;
#pragma unroll
        for (int p = 0; p < PPL; ++p) live |= __any(T[p] > 0.0f) ? (1u << p) : 0u;
        if (lane == 0) slive[w] = live << (w * PPL);
#if !GSR_F6_ONESYNC
        if (__syncthreads_or(live != 0) == 0) {
            tend = base;
            break;
        }
#endif
        if (tid < BATCH && base + tid < n) {
            const uint32_t g = GSR_F6_GID_AHEAD ? g_next : sorted_gid[range.x + base + tid];
            if (GSR_F6_GID_AHEAD && base + BATCH + tid < n) g_next = sorted_gid[range.x + base + BATCH + tid];
            const float4* r = rec + 3 * (size_t)g;
            const float4 r0 = r[0], r1 = r[1], r2 = r[2];
            srec[3 * tid + 0] = r0;
            srec[3 * tid + 1] = r1;
            srec[3 * tid + 2] = r2;
            smk[tid] = stripe_mask(r0, r1, r2, bx0, by0);
            mk[range.x + base + tid] = (uint8_t)smk[tid];  // B1's visit filter
        } else if (tid < BATCH) {
            smk[tid] = 0u;
        }
        __syncthreads();
        uint32_t tile_live = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) tile_live |= slive[i];
#if GSR_F6_ONESYNC
        // termination from the batch barrier's own slive words (__syncthreads_or is three
        // barriers); the batch just loaded is then discarded, and its mask bytes lie at or past
        // tend, where B1 never reads
        if (tile_live == 0) {
            tend = base;
            break;
        }
#endif
        const int cnt = (n - base) < BATCH ? (n - base) : BATCH;
        int visited = 0;
        for (int c0 = 0; c0 < cnt; c0 += 64) {
            const uint32_t sm = smk[c0 + lane];  // 0 past cnt
#if GSR_CK_MERGE && !GSR_CK_MERGE_BATCH_END
            // at the group boundary where a 32nd chunk would open
            if (__builtin_expect(work >= quota && nck == kMaxChunks - 1, 0)) merge_chunks();
#endif
            if (work >= quota && nck < kMaxChunks - 1) {  // chunk nck + 1 starts at base + c0
                ++nck;
                checkpoint(ck_slot_of(geo.ck_fixed, range.x, tl, nck), live);
                if (tid == 0) table[nck] = (uint32_t)(base + c0);
                work = 0;
            }
            const uint32_t tm = sm & tile_live;
            work += __popcll(__ballot(tm & 1u)) + __popcll(__ballot(tm & 2u)) + __popcll(__ballot(tm & 4u)) +
                    __popcll(__ballot(tm & 8u));
            if (!live) continue;
            const uint32_t mine = (sm >> (w * PPL)) & ((1u << PPL) - 1u);
            uint64_t todo = __ballot((mine & live) != 0u && c0 + lane < cnt);
#ifndef GSR_F6_BAND_PAIRS
#define GSR_F6_BAND_PAIRS 1
#endif
            // Band launches (NW = 4: one stripe per wave, every block resident at once) are bound
            // by one wave's dependent chain per record, not by issue: there two records are taken
            // per pass -- both alphas first (they do not depend on T), then the T / colour
            // updates in list order, so the result is bit-identical.
            if constexpr (GSR_F6_BAND_PAIRS && PPL == 1) {
                while (todo) {
                    const int ka = c0 + __builtin_ctzll(todo);
                    todo &= todo - 1;
                    const bool two = todo != 0;  // wave-uniform
                    const int kb = two ? c0 + __builtin_ctzll(todo) : ka;
                    if (two) todo &= todo - 1;
                    const float4 a0 = srec[3 * ka + 0], a1 = srec[3 * ka + 1], a2 = srec[3 * ka + 2];
                    const float4 b0 = srec[3 * kb + 0], b1 = srec[3 * kb + 1], b2 = srec[3 * kb + 2];
                    const float dxa = a0.x - pfx, dxb = b0.x - pfx;
                    const float dya = a0.y - pfy[0], dyb = b0.y - pfy[0];
                    const float ea = fmaf(fmaf(a1.x, dya, a0.w * dxa), dya, fmaf(a0.z * dxa, dxa, a2.w));
                    const float eb = fmaf(fmaf(b1.x, dyb, b0.w * dxb), dyb, fmaf(b0.z * dxb, dxb, b2.w));
                    float oGa, oGb;
                    const float aa = pair_alpha(ea, a2.w, oGa);
                    const float ab = pair_alpha(eb, b2.w, oGb);
                    {
                        const float w = aa * T[0];
                        const float tT = T[0] - w;
                        const bool ok = tT >= 0.0001f;
                        const float wgt = ok ? w : 0.0f;
                        C0[0] = fmaf(a1.z, wgt, C0[0]);
                        C1[0] = fmaf(a1.w, wgt, C1[0]);
                        C2[0] = fmaf(a2.x, wgt, C2[0]);
                        T[0] = ok ? tT : -fabsf(T[0]);
                    }
                    if (two) {
                        const float w = ab * T[0];
                        const float tT = T[0] - w;
                        const bool ok = tT >= 0.0001f;
                        const float wgt = ok ? w : 0.0f;
                        C0[0] = fmaf(b1.z, wgt, C0[0]);
                        C1[0] = fmaf(b1.w, wgt, C1[0]);
                        C2[0] = fmaf(b2.x, wgt, C2[0]);
                        T[0] = ok ? tT : -fabsf(T[0]);
                    }
                    const int before = visited;
                    visited += two ? 2 : 1;
                    if ((before >> 3) != (visited >> 3)) {
                        live = __any(T[0] > 0.0f) ? 1u : 0u;
                        if (live == 0) break;
                    }
                }
                continue;
            }
            while (todo) {
                const int kk = __builtin_ctzll(todo);
                todo &= todo - 1;
                const int k = c0 + kk;
                const float4 r0 = srec[3 * k + 0];
                const float4 r1 = srec[3 * k + 1];
                const float4 r2 = srec[3 * k + 2];
                const float dx = r0.x - pfx;
                const float bdx = r0.w * dx;
                const float K = fmaf(r0.z * dx, dx, r2.w);  // column part of the exponent + log2 o
#pragma unroll
                for (int p = 0; p < PPL; ++p) {
                    // No per-stripe branch: a culled stripe's pixels all get alpha 0 (exact test),
                    // which leaves C and T bit-for-bit unchanged, and with two waves per tile both
                    // stripes of a visited record run in one basic block -- the two chains
                    // interleave (0.257 vs 0.263 ms with the branch; with four waves a visited
                    // record always covers the wave's one stripe).  B1 keeps the branch (its
                    // culled stripes skip 28 ops, branchless 0.518 vs 0.465 ms).
                    const float dy = r0.y - pfy[p];
                    const float e = fmaf(fmaf(r1.x, dy, bdx), dy, K);
                    float oG;
                    const float a = pair_alpha(e, r2.w, oG);
                    const float w = a * T[p];
                    const float tT = T[p] - w;
                    const bool ok = tT >= 0.0001f;
                    const float wgt = ok ? w : 0.0f;
                    C0[p] = fmaf(r1.z, wgt, C0[p]);
                    C1[p] = fmaf(r1.w, wgt, C1[p]);
                    C2[p] = fmaf(r2.x, wgt, C2[p]);
                    T[p] = ok ? tT : -fabsf(T[p]);
                }
                if ((++visited & 7) == 0) {
                    uint32_t lv = 0;
#pragma unroll
                    for (int p = 0; p < PPL; ++p) lv |= __any(T[p] > 0.0f) ? (1u << p) : 0u;
                    live = lv;
                    if (live == 0) break;
                }
            }
        }
#if GSR_CK_MERGE && GSR_CK_MERGE_BATCH_END
        // at the end of the batch in which the last start was taken (outside the blend loop)
        if (nck == kMaxChunks - 1) merge_chunks();
#endif
        __syncthreads();
    }
    if (tid == 0) {
        table[0] = (uint32_t)tend;
        for (int c = nck + 1; c < kMaxChunks; ++c) table[c] = 0xFFFFFFFFu;
    }
    // per view: [3, vh, W] colour planes and a [vh, W] transmittance plane (one image: view 0)
    const size_t npix = (size_t)geo.W * geo.vh;
    float* const oc = out_color + (size_t)view * 3 * npix;
    float* const ac = accum + (size_t)view * 3 * npix;
    float* const fT = final_T + (size_t)view * npix;
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
        const int pyl = tyl * kTile + (lane >> 4) + 4 * (w * PPL + p);
        if (px < geo.W && pyl < geo.vh) {
            const size_t pix = (size_t)pyl * geo.W + px;
            const float Tf = fabsf(T[p]);
            fT[pix] = Tf;
            ac[pix] = C0[p];
            ac[npix + pix] = C1[p];
            ac[2 * npix + pix] = C2[p];
            oc[pix] = C0[p] + Tf * geo.bg0;
            oc[npix + pix] = C1[p] + Tf * geo.bg1;
            oc[2 * npix + pix] = C2[p] + Tf * geo.bg2;
        }
    }
}

// Deferred B1 reduction.  A record's 9 per-lane moments are quad-reduced by DPP; the 16 quad
// partials wait in LDS, and every kPark records one (record, moment) output per lane is summed
// from LDS in fixed quad order and stored straight to the partial arrays at the record's
// emission index j (8 moments in part8[2j..2j+1], the 9th in part1[j]).
constexpr int kPark = 4;
// Parking slot stride and the flush's lane map.  The flush reads with ds_read_b32, whose banks
// are (address / 4) mod 32 over lane groups {0-31}, {32-63} (MI355X_MICROARCH.md, LDS table).
// Flush lane l sums moment c = l >> 2 of parked slot s = l & 3 (36 lanes: c < 9), so lanes 0-31
// are (c 0-7) x (s 0-3) and read word 8 s + c + 12 i (mod 32) for quad i: 32 distinct banks when
// the slot stride is 8 mod 32 (200 = 16 quads x 12 floats + 8, 16-B aligned for the leaders'
// float4 stores).  Round 4's map (s = l / 9, c = l mod 9, stride 204 = 12 mod 32) put slots 2 / 3
// on slot 0's banks: a 2-way conflict on every flush read, the ~9.5e6 SQ_LDS_BANK_CONFLICT cycles
// per launch of profiles/r04_pmc_summary.txt (16 reads x ~6.3e5 flushes at 1M / 1080p).
constexpr int kParkSlot = 16 * 12 + 8;
static_assert(kParkSlot % 32 == 8 && kParkSlot % 4 == 0, "flush banks / float4 alignment");
// The parked records' batch indices ride in one scalar word (6 bits per slot: `kpack`); the
// flush lane of slot s reads its record's emission index from the batch's jl table (`sjl`,
// written once per batch), so a record costs no per-record readlane / LDS write for it.
__device__ __forceinline__ void park_flush(const float* qpark, const uint32_t* sjl, uint32_t kpack, int parked,
                                           float* p8f, float* p1, uint8_t* fl, int lane) {
    __syncthreads();  // one-wave block: orders the quad leaders' LDS writes before the reads
    const int slot = lane & 3, c = lane >> 2;
    if (c < 9 && slot < parked) {
        const float* q = qpark + slot * kParkSlot + c;
        // -0 is the identity of IEEE addition, so the first add of each chain folds into a move
        float t[4] = {-0.f, -0.f, -0.f, -0.f};
#pragma unroll
        for (int i = 0; i < 16; ++i) t[i & 3] += q[i * 12];
        const uint32_t j = sjl[(kpack >> (6 * slot)) & 63u];
        if (j != 0xFFFFFFFFu) {  // an entry past the capacity (binning overflow) has none
            float* dst = c < 8 ? p8f + 8 * (size_t)j + c : p1 + j;
            *dst = (t[0] + t[1]) + (t[2] + t[3]);
            if (c == 8) fl[j] = 1;  // the gather reads flagged entries only
        }
    }
    __syncthreads();
}

// B1 front to back.  With S = the forward's colour sum (no background) and the running
// Sp = sum over processed contributors of w * (c . dL/dpix), the colour behind entry k is
// (S . dL/dpix - Sp) / (1 - alpha_k) after T_k, so
//   dL/dalpha_k = T_k (c_k . dL/dpix) - R / (1 - alpha_k),
//   R = S . dL/dpix + T_final bg . dL/dpix - Sp
// (SURVEY B.4 rewritten; same value as the back-to-front recursion).  A lane keeps R itself
// (R -= w (c . dL/dpix) per contributor), one register and one op fewer than Sp and S.  T is
// recomputed with the forward's own instructions (same exponent, alpha, T - alpha T and sign
// encoding), so
// the set of contributing pairs -- and the termination point -- is exactly the forward's.
// Per record the lane accumulates sv = o G dL/dalpha moments along its column
// (sum sv, sum sv dy, sum sv dy^2) and applies dx afterwards:
//   Sx = dx sum sv, Sxx = dx^2 sum sv, Sxy = dx sum sv dy.
// B1 stores the raw tile sums (Sx, Sy, Sxx, Sxy, Syy, S0, colour x3); they are linear in the
// gradients, so gather_grad2d converts them once per Gaussian after summing over tiles.
//
// Batches: F6 stores the stripe mask of every list entry it loads (one byte each, `mk`); B1 reads
// 256 of them per step (one aligned word per lane), keeps the entries with a stripe still live
// and takes up to 64 of them, in list order, as its batch -- records that cannot touch a live
// stripe are never loaded (after an opacity reset most of a deep list is culled this way).
// Grid: one 64-lane block per (tile, chunk slot); chunk c > 0 starts where F6's chunk table
// says and resumes from F6's checkpoint, and slots the tile has no chunk for exit at once.  Each
// XCD (blocks b with equal b % 8) takes a contiguous tile range as in xcd_tile, visited
// chunk-major, so every tile's first chunk is dispatched first.
// 6 waves per SIMD: 80 VGPRs (no spills) and 6.2 KB of LDS per one-wave block.  Measured
// 0.552 ms vs 0.564 at the compiler's own 85 VGPRs (5 waves); 7 and 8 waves spill.
// Mask bytes per lane in one batch window (4: 256 entries per window; 16: 1024, for lists whose
// entries are mostly culled, e.g. after an opacity reset -- fewer serial window loads).
#ifndef GSR_B1_PAIRS
#define GSR_B1_PAIRS 0
#endif
// GSR_B1_GID_WIN: B1 loads the batch window's gids with its mask bytes (one 16-B load per lane),
// so a batch's record loads do not wait on a gid load first
#ifndef GSR_B1_GID_WIN
#define GSR_B1_GID_WIN 1
#endif
constexpr int kB1Win = GSR_B1_WIN;
static_assert(kB1Win == 4 || kB1Win == 16, "B1 window: 4 or 16 mask bytes per lane");
// SPW: the 16x4 stripes one wave owns.  4 (full images): one wave per (tile, chunk) and one
// partial entry per (tile, instance).  2 or 1 (band launches, b1_split): the (tile, chunk) is
// split over 4 / SPW one-wave blocks by stripe ("parts"), each running the same front-to-back
// loop over its own pixels only -- its own termination, its own visit filter -- and writing
// its own partial entry j * parts + part, which the gather sums with the others in part order.
// A band of 1/8 of the tiles then still fills the chip (~3.3 chunks per tile leave ~3 one-wave
// blocks per SIMD otherwise), at the price of per-record work repeated per part.
// PF (band launches, GSR_B1_BAND_PREFETCH): each visited record's LDS reads are issued before the
// previous record's work (2x unrolled, no register copies) -- with ~3 one-wave blocks per SIMD on a
// band's 1020 tiles the LDS latency per record is exposed, where on full images other waves hide
// it (round 4: the same prefetch at full occupancy measured 0.456 vs 0.447 ms).
template <int SPW, bool PF = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PF ? 4 : (SPW == 4 ? 6 : 8)))) void blend_backward_kernel(const BlendGeom geo,
                                                            const uint2* __restrict__ ranges,
                                                            const uint32_t* __restrict__ sorted_gid,
                                                            const uint4* __restrict__ rect,
                                                            const float4* __restrict__ rec,
                                                            const float* __restrict__ final_T,
                                                            const float* __restrict__ accum,
                                                            const float* __restrict__ dL_dpix,
                                                            float* __restrict__ p8f,
                                                            float* __restrict__ p1,
                                                            uint8_t* __restrict__ fl,
                                                            const uint32_t* __restrict__ term,
                                                            const float4* __restrict__ ck,
                                                            const uint8_t* __restrict__ mk) {
    // One block of LDS with srec first: the record fields then sit within the immediate offsets
    // of the record reads (8-bit dword offsets of ds_read2), so a record costs no address add.
    __shared__ struct {
        float4 srec[64 * 3];
        uint32_t sjl[64];                  // the batch's emission indices, by batch slot
        float qpark[kPark * kParkSlot];    // [slot][quad][9 of 12]
        uint32_t sidx[64];                 // the batch's entries (list offsets), in list order
        uint32_t smv[64];                  // and their stripe masks
#if GSR_B1_GID_WIN
        uint32_t sgd[64];                  // and their gids (loaded with the window's mask bytes)
#endif
    } lds;
    float4* const srec = lds.srec;
    uint32_t* const sjl = lds.sjl;
    float* const qpark = lds.qpark;
    constexpr int S = kPPL / SPW;  // parts per (tile, chunk)
    static_assert(SPW == 4 || SPW == 2 || SPW == 1, "stripes per wave");
    const int lane = threadIdx.x;
    float* const qlane = qpark + (lane >> 2) * 12;  // this quad's parking row
    int tl, chunk;
    const int part = (int)((blockIdx.x / 8) % S);  // the (tile, chunk)'s parts are neighbours
    const int sp0 = part * SPW;                      // this wave's first stripe
    {
        const int q = geo.nwg / 8, r = geo.nwg % 8, xcd = blockIdx.x % 8, local = (int)((blockIdx.x / 8) / S);
        const int t0 = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q, nt = q + (xcd < r ? 1 : 0);
        const int per = q + 1;  // padded tiles per XCD
        chunk = local / per;
        const int i = local - chunk * per;
        if (i >= nt) return;
        tl = t0 + i;
    }
    const int tile = tl + geo.ty0 * geo.grid_x;
    const uint2 range = ranges[tile];
    const int n_all = (int)(range.y - range.x);
    // F6's chunk table: [termination index, chunk 1..kMaxChunks-1 starts (UINT32_MAX: none)]
    const uint32_t* table = term + (size_t)tl * kMaxChunks;
    const uint32_t tend = table[0];
    const uint32_t start_u = chunk == 0 ? 0u : table[chunk];
    // no such chunk for this tile, or every pixel had finished before it
    if (start_u >= (uint32_t)n_all || start_u >= tend) return;
    const int start = (int)start_u;
    const uint32_t next = chunk + 1 < kMaxChunks ? table[chunk + 1] : 0xFFFFFFFFu;
    const int n = next < (uint32_t)n_all ? (int)next : n_all;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    // lane = 4 col + row: a quad holds one column's 4 rows of a stripe, so it shares dx and
    // the record's moments reduce over the quad before dx is applied (F6 lays a stripe out
    // row-major, lane = col + 16 row; B1 reads F6's checkpoints through that map)
    const int col = lane >> 2, row = lane & 3;
    const int px = tx * kTile + col;
    const float pfx = (float)px;
    const int view = ty / geo.vgy, tyl = ty - view * geo.vgy;  // tile row inside its view's band
    const float bx0 = (float)(tx * kTile), by0 = (float)(tyl * kTile);
    // F6's per-view planes (one image: view 0)
    const size_t npix = (size_t)geo.W * geo.vh;
    final_T += (size_t)view * npix;
    accum += (size_t)view * 3 * npix;
    dL_dpix += (size_t)view * 3 * npix;
    // R = S . dL/dpix - Sp + T_final bg . dL/dpix: the colour term behind the current record
    float pfy[SPW], T[SPW], R[SPW], dp0[SPW], dp1[SPW], dp2[SPW];
#pragma unroll
    for (int p = 0; p < SPW; ++p) {
        const int pyl = tyl * kTile + row + 4 * (sp0 + p);
        pfy[p] = (float)pyl;
        const bool in = px < geo.W && pyl < geo.vh;
        const size_t pix = in ? (size_t)pyl * geo.W + px : 0;
        const float Tfin = in ? final_T[pix] : 1.0f;
        dp0[p] = in ? dL_dpix[pix] : 0.0f;
        dp1[p] = in ? dL_dpix[npix + pix] : 0.0f;
        dp2[p] = in ? dL_dpix[2 * npix + pix] : 0.0f;
        const float sdp = in ? accum[pix] * dp0[p] + accum[npix + pix] * dp1[p] + accum[2 * npix + pix] * dp2[p]
                             : 0.0f;
        R[p] = sdp + Tfin * (geo.bg0 * dp0[p] + geo.bg1 * dp1[p] + geo.bg2 * dp2[p]);
        T[p] = in ? 1.0f : -1.0f;
    }
    if (chunk > 0) {  // resume from F6's checkpoint: T, and R less dL/dpix . (colour sum so far)
        const size_t slot = ck_slot_of(geo.ck_fixed, range.x, tl, chunk);
        const float4* src = ck + slot * 256;
        // F6's live-stripe bytes: a stripe it did not write had finished (start it dead)
        const uint32_t on = *reinterpret_cast<const uint32_t*>(
            reinterpret_cast<const uint8_t*>(ck + (size_t)geo.ck_slots * 256) + 4 * slot);
#pragma unroll
        for (int p = 0; p < SPW; ++p) {
            if ((on >> (8 * (sp0 + p))) & 0xFFu) {  // wave-uniform
                const float4 c4 = src[64 * (sp0 + p) + col + 16 * row];  // F6's lane of this pixel
                T[p] = c4.x;
                R[p] -= fmaf(c4.y, dp0[p], fmaf(c4.z, dp1[p], c4.w * dp2[p]));
            } else {
                T[p] = -1.0f;
            }
        }
    }
    // F6 wrote the stripe mask of every entry it loaded, all before its termination index tend;
    // past tend no pixel is live
    const int n_lim = n < (int)tend ? n : (int)tend;
    for (int base = start; base < n_lim;) {
        uint32_t live = 0;  // in stripe positions (the mask bytes' bits)
#pragma unroll
        for (int p = 0; p < SPW; ++p) live |= __any(T[p] > 0.0f) ? (1u << (sp0 + p)) : 0u;
        if (live == 0) break;
        // the batch: up to 64 entries with a live stripe among the next 256 (four mask bytes
        // per lane from one aligned word), in list order; the next batch starts after the last
        // one taken, or after the window
        constexpr int kW = kB1Win / 4;  // mask words per lane
        const uint32_t a0 = (range.x + (uint32_t)base) & ~(uint32_t)(kB1Win - 1);  // aligned window start
        uint32_t wd[kW];
        if constexpr (kW == 4) {
            const uint4 v = *reinterpret_cast<const uint4*>(mk + a0 + kB1Win * lane);
            wd[0] = v.x, wd[1] = v.y, wd[2] = v.z, wd[3] = v.w;
        } else {
            wd[0] = *reinterpret_cast<const uint32_t*>(mk + a0 + 4 * lane);
        }
#if GSR_B1_GID_WIN
        static_assert(kB1Win == 4, "gids with the mask window: 4 entries per lane");
        // the window's gids beside its mask bytes (one 16-B load per lane; the list array is
        // followed by the rest of the binning buffer, so the window's tail past the list is
        // readable and never used): the batch's record loads then wait for no gid load
        const uint4 gw = *reinterpret_cast<const uint4*>(sorted_gid + a0 + 4 * lane);
        const uint32_t gwa[4] = {gw.x, gw.y, gw.z, gw.w};
#endif
        uint32_t vis = 0;
#pragma unroll
        for (int i = 0; i < kB1Win; ++i) {
            const int e = (int)(a0 + kB1Win * lane + i - range.x);  // list offset of byte i
            const uint32_t m = (wd[i >> 2] >> (8 * (i & 3))) & 0xFu;
            if (e >= base && e < n_lim && (m & live)) vis |= 1u << i;
        }
        const uint32_t c = (uint32_t)__popc(vis);
        uint32_t incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        const uint32_t excl = incl - c;
        const uint32_t total = (uint32_t)__shfl(incl, 63, 64);
        const int cnt = total < 64u ? (int)total : 64;
        uint32_t pos = excl;
#pragma unroll
        for (int i = 0; i < kB1Win; ++i) {
            if ((vis >> i) & 1u) {
                if (pos < 64u) {
                    lds.sidx[pos] = a0 + kB1Win * lane + i - range.x;
                    lds.smv[pos] = (wd[i >> 2] >> (8 * (i & 3))) & 0xFu;
#if GSR_B1_GID_WIN
                    lds.sgd[pos] = gwa[i];
#endif
                }
                ++pos;
            }
        }
        __syncthreads();
        // next window: after the 64th taken entry when the window held more, else past it
        base = total > 64u ? (int)lds.sidx[63] + 1 : (int)(a0 + 64 * kB1Win - range.x);
        if (cnt == 0) {
            __syncthreads();
            continue;
        }
        uint32_t jl = 0, smask = 0;
        if (lane < cnt) {
#if GSR_B1_GID_WIN
            const uint32_t g = lds.sgd[lane];
#else
            const uint32_t g = sorted_gid[range.x + lds.sidx[lane]];
#endif
            const uint4 rr = rect[g];
            const int minx = rr.x & 0xFFFF, miny = rr.x >> 16, maxx = rr.y & 0xFFFF;
            const int y0 = miny > geo.ty0 ? miny : geo.ty0;
            jl = rr.z + (uint32_t)((ty - y0) * (maxx - minx) + (tx - minx));
            // past the capacity: an overflowing binning (the row-bucketed one keeps list
            // positions, not emission indices, below it) -- the entry is not written
            jl = jl >= geo.cap ? 0xFFFFFFFFu : jl * S + part;  // this part's entry
            const float4* r = rec + 3 * (size_t)g;
            srec[3 * lane + 0] = r[0];
            srec[3 * lane + 1] = r[1];
            srec[3 * lane + 2] = r[2];
            smask = lds.smv[lane];
        }
        sjl[lane] = jl;
        __syncthreads();
        uint64_t todo = __ballot(lane < cnt);
        int visited = 0, parked = 0;
        uint32_t kpack = 0;  // batch slots of the parked records, 6 bits each
        // one visited record (batch slot k): its stripes, then its moments parked / flushed;
        // true when every pixel of the tile has finished
        auto record = [&](const int k, const float4 r0, const float4 r1, const float4 r2) -> bool {
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)smask, k) & live;
            const float dx = r0.x - pfx;
            const float bdx = r0.w * dx;
            const float K = fmaf(r0.z * dx, dx, r2.w);
            // -0 is the exact identity of IEEE addition (x + -0 = x for every x, +0 included), so
            // the first stripe's adds / FMAs into these fold into plain moves / multiplies
            // without fast-math; +0 would keep them (0 + -0 = +0)
            float s0 = -0.f, sy = -0.f, syy = -0.f, g0 = -0.f, g1 = -0.f, g2 = -0.f;
            bool any = false;
            // one contributing (pixel, record) pair of stripe p into the record's moments
            auto contribute = [&](const int p, const float a, const float w, const float oG, const float dy) {
                any = true;
                const float one_m = 1.0f - a;
                const float cdp = fmaf(r1.z, dp0[p], fmaf(r1.w, dp1[p], r2.x * dp2[p]));
                R[p] = fmaf(-w, cdp, R[p]);
                const float dLda = fmaf(T[p], cdp, -R[p] * __builtin_amdgcn_rcpf(one_m));
                g0 = fmaf(w, dp0[p], g0);
                g1 = fmaf(w, dp1[p], g1);
                g2 = fmaf(w, dp2[p], g2);
                const float sv = oG * dLda;
                s0 += sv;
                const float svy = sv * dy;
                sy += svy;
                syy = fmaf(svy, dy, syy);
            };
#if GSR_B1_PAIRS
            if constexpr (SPW >= 2) {
                // Stripes in pairs (2q, 2q + 1): the two alpha / transmittance chains of a visited
                // pair in one block, interleaved (the exp latency of one covers the other), the
                // contributions still behind exec-mask branches.  A stripe of the pair that the
                // record does not visit runs with L = -inf: keep is false, so alpha = 0, T stays
                // (live T >= 1e-4, dead T < 0) and nothing is added -- bit-identical to skipping it.
#pragma unroll
                for (int q = 0; q < SPW / 2; ++q) {
                    const int pa = 2 * q, pb = 2 * q + 1;
                    const uint32_t pm = (m >> (sp0 + pa)) & 3u;
                    if (!pm) continue;  // wave-uniform
                    const float La = (pm & 1u) ? r2.w : -INFINITY, Lb = (pm & 2u) ? r2.w : -INFINITY;
                    const float dya = r0.y - pfy[pa], dyb = r0.y - pfy[pb];
                    const float ea = fmaf(fmaf(r1.x, dya, bdx), dya, K);
                    const float eb = fmaf(fmaf(r1.x, dyb, bdx), dyb, K);
                    float oGa, oGb;
                    bool keepa, keepb;
                    const float aa = pair_alpha_keep(ea, La, oGa, keepa);
                    const float ab = pair_alpha_keep(eb, Lb, oGb, keepb);
                    const float wa = aa * T[pa], wb = ab * T[pb];
                    const float tTa = T[pa] - wa, tTb = T[pb] - wb;
                    const bool oka = tTa >= 0.0001f, okb = tTb >= 0.0001f;
                    if (oka && keepa) contribute(pa, aa, wa, oGa, dya);
                    T[pa] = oka ? tTa : -fabsf(T[pa]);
                    if (okb && keepb) contribute(pb, ab, wb, oGb, dyb);
                    T[pb] = okb ? tTb : -fabsf(T[pb]);
                }
            } else
#endif
            {
#pragma unroll
                for (int p = 0; p < SPW; ++p) {
                    if (!(m & (1u << (sp0 + p)))) continue;  // wave-uniform
                    const float dy = r0.y - pfy[p];
                    const float e = fmaf(fmaf(r1.x, dy, bdx), dy, K);
                    float oG;
                    bool keep;
                    const float a = pair_alpha_keep(e, r2.w, oG, keep);
                    const float w = a * T[p];
                    const float tT = T[p] - w;
                    const bool ok = tT >= 0.0001f;
                    if (ok && keep) contribute(p, a, w, oG, dy);
                    T[p] = ok ? tT : -fabsf(T[p]);
                }
            }
            if (__any(any)) {
                // the quad shares dx: reduce the six column sums (12 DPP adds, not 18 for the
                // nine dx-weighted moments of a row-major quad), then apply dx once
                float u[6] = {s0, sy, syy, g0, g1, g2};
                quad_reduce(u);
                const float sx = u[0] * dx;
                float v[9] = {sx, u[1], sx * dx, u[1] * dx, u[2], u[0], u[3], u[4], u[5]};
                if ((lane & 3) == 0) {
                    float* dst = qlane + parked * kParkSlot;
                    *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
                    *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
                    dst[8] = v[8];
                }
                kpack |= (uint32_t)k << (6 * parked);
                if (++parked == kPark) {
                    park_flush(qpark, sjl, kpack, parked, p8f, p1, fl, lane);
                    parked = 0;
                    kpack = 0;
                }
            }
            if ((++visited & 7) == 0) {
                uint32_t lv = 0;
#pragma unroll
                for (int p = 0; p < SPW; ++p) lv |= __any(T[p] > 0.0f) ? (1u << (sp0 + p)) : 0u;
                live = lv;
                if (live == 0) return true;
            }
            return false;
        };
        if constexpr (PF) {
            if (todo) {
                int ka = __builtin_ctzll(todo);
                todo &= todo - 1;
                float4 a0 = srec[3 * ka + 0], a1 = srec[3 * ka + 1], a2 = srec[3 * ka + 2];
                float4 b0, b1, b2;
                while (true) {
                    const int kb = todo ? __builtin_ctzll(todo) : -1;  // wave-uniform
                    if (kb >= 0) {
                        todo &= todo - 1;
                        b0 = srec[3 * kb + 0];
                        b1 = srec[3 * kb + 1];
                        b2 = srec[3 * kb + 2];
                    }
                    if (record(ka, a0, a1, a2) || kb < 0) break;
                    ka = todo ? __builtin_ctzll(todo) : -1;
                    if (ka >= 0) {
                        todo &= todo - 1;
                        a0 = srec[3 * ka + 0];
                        a1 = srec[3 * ka + 1];
                        a2 = srec[3 * ka + 2];
                    }
                    if (record(kb, b0, b1, b2) || ka < 0) break;
                }
            }
        } else {
            while (todo) {
                const int k = __builtin_ctzll(todo);
                todo &= todo - 1;
                if (record(k, srec[3 * k + 0], srec[3 * k + 1], srec[3 * k + 2])) break;
            }
        }
        if (parked) park_flush(qpark, sjl, kpack, parked, p8f, p1, fl, lane);
        __syncthreads();  // srec / qpark are rewritten by the next batch
    }
}
}  // namespace

// Waves per F6 tile: 2 for a full image (wave w owns stripes 2w, 2w + 1), 4 when the launch
// has too few tiles to fill the chip (multi-GPU bands).  Measured at 1M/1080p with the
// branchless stripe pair: 2 waves 0.258 ms, 1 wave 0.269 (with branches) / 0.343 (branchless,
// 4 stripes), 4 waves 0.299.
#ifndef GSR_F6_BAND_TILES
#define GSR_F6_BAND_TILES 4096
#endif
constexpr int kF6FullWaves = 2, kF6BandWaves = 4, kF6BandTiles = GSR_F6_BAND_TILES;

static BlendGeom make_geo(const gsr_camera& cam, const float bg[3], int ty0, int ty1, long long cap, int vgy, int vh) {
    BlendGeom g;
    g.W = cam.width;
    g.H = cam.height;
    g.vgy = vgy > 0 ? vgy : div_up(cam.height, kTile);
    g.vh = vgy > 0 ? vh : cam.height;
    g.grid_x = div_up(cam.width, kTile);
    g.ty0 = ty0;
    g.nwg = (ty1 - ty0) * g.grid_x;
    const long long full_tiles = (long long)div_up(cam.height, kTile) * g.grid_x;
    g.ck_slots = (uint32_t)ck_pool_slots(cap, full_tiles);  // = BinLayout's
    g.ck_fixed = ck_fixed_layout(cap, full_tiles) ? 1 : 0;
    g.bg0 = bg[0];
    g.bg1 = bg[1];
    g.bg2 = bg[2];
    g.cap = cap > 0 ? (uint32_t)cap : 0u;
    return g;
}

int launch_blend_forward(const gsr_camera& cam, const float bg[3], int ty0, int ty1,
                         const uint2* ranges, const uint32_t* sorted_gid, const float4* rec,
                         float* out_color, float* final_T, float* accum, uint32_t* term, float4* ck, long long cap,
                         hipStream_t s, int vgy, int vh, uint8_t* mk) {
    const BlendGeom geo = make_geo(cam, bg, ty0, ty1, cap, vgy, vh);
    if (geo.nwg <= 0) return 0;
    // the variant (and with it the B1 chunk work) follows the tiles of ONE image: views mode then
    // chunks every tile as a per-view call does, which keeps its gradients bit-identical
    const long long sel = vgy > 0 ? (long long)geo.vgy * geo.grid_x : geo.nwg;
    if (sel >= kF6BandTiles)
        hipLaunchKernelGGL(blend_forward_kernel<kF6FullWaves>, dim3(geo.nwg), dim3(64 * kF6FullWaves), 0, s, geo,
                           ranges, sorted_gid, rec, out_color, final_T, accum, term, ck, mk);
    else
        hipLaunchKernelGGL(blend_forward_kernel<kF6BandWaves>, dim3(geo.nwg), dim3(64 * kF6BandWaves), 0, s, geo,
                           ranges, sorted_gid, rec, out_color, final_T, accum, term, ck, mk);
    return (int)hipGetLastError();
}

// B1 parts per (tile, chunk) (blend_backward_kernel's 4 / SPW) on launches of fewer than
// GSR_B1_SPLIT_TILES tiles of one image (multi-GPU bands).  Measured at 1M / 1080p, N = 8
// (rehearsal kernel trace, mean band B1 / gather; profiles/r06_experiments/b1_split_1m_w8.txt):
// 1 part 101.8 / 24.7 us, 2 parts 101.4 / 50.9, 4 parts 130.0 / 115.4 -- a part repeats the
// record's set-up, batch loads and reduction for fewer stripes, and the per-chunk chain is set
// by that per-record work, not by the stripes; so the split is built but off (1).
#ifndef GSR_B1_SPLIT_TILES
#define GSR_B1_SPLIT_TILES 4096
#endif
#ifndef GSR_B1_BAND_PREFETCH
#define GSR_B1_BAND_PREFETCH 1
#endif
#ifndef GSR_B1_BAND_SPLIT
#define GSR_B1_BAND_SPLIT 1
#endif
int b1_split(int W, int H, int ty0, int ty1, int vgy) {
    (void)H;
    const long long gx = div_up(W, kTile);
    const long long sel = vgy > 0 ? (long long)vgy * gx : (long long)(ty1 - ty0) * gx;  // one image's tiles
    return sel < GSR_B1_SPLIT_TILES ? GSR_B1_BAND_SPLIT : 1;
}

int launch_blend_backward(const gsr_camera& cam, const float bg[3], int ty0, int ty1,
                          const uint2* ranges, const uint32_t* sorted_gid, const uint4* rect,
                          const float4* rec, const float* final_T,
                          const float* accum, const float* dL_dpix, float* partial, long long cap,
                          const uint32_t* term, const float4* ck, hipStream_t s, int vgy, int vh,
                          const uint8_t* mk, int split) {
    const BlendGeom geo = make_geo(cam, bg, ty0, ty1, cap, vgy, vh);
    if (geo.nwg <= 0) return 0;
    if (split != 1 && split != 2 && split != 4) return (int)hipErrorInvalidValue;
    const PartLayout pl(cap * split);  // one entry per (instance, part)
    char* base = reinterpret_cast<char*>(partial);
    const int blocks = 8 * (geo.nwg / 8 + 1) * kMaxChunks * split;
    auto* p8 = reinterpret_cast<float*>(base + pl.p8);
    auto* p1 = reinterpret_cast<float*>(base + pl.p1);
    auto* fl = reinterpret_cast<uint8_t*>(base + pl.fl);
    const long long sel = vgy > 0 ? (long long)geo.vgy * geo.grid_x : geo.nwg;  // one image's tiles
    if (split == 1 && GSR_B1_BAND_PREFETCH && sel < kF6BandTiles)
        hipLaunchKernelGGL((blend_backward_kernel<4, true>), dim3(blocks), dim3(64), 0, s, geo, ranges, sorted_gid,
                           rect, rec, final_T, accum, dL_dpix, p8, p1, fl, term, ck, mk);
    else if (split == 1)
        hipLaunchKernelGGL(blend_backward_kernel<4>, dim3(blocks), dim3(64), 0, s, geo, ranges, sorted_gid, rect, rec,
                           final_T, accum, dL_dpix, p8, p1, fl, term, ck, mk);
    else if (split == 2)
        hipLaunchKernelGGL(blend_backward_kernel<2>, dim3(blocks), dim3(64), 0, s, geo, ranges, sorted_gid, rect, rec,
                           final_T, accum, dL_dpix, p8, p1, fl, term, ck, mk);
    else
        hipLaunchKernelGGL(blend_backward_kernel<1>, dim3(blocks), dim3(64), 0, s, geo, ranges, sorted_gid, rect, rec,
                           final_T, accum, dL_dpix, p8, p1, fl, term, ck, mk);
    return (int)hipGetLastError();
}

int launch_clear_flags(float* partial, long long cap, hipStream_t s) {
    if (cap <= 0) return 0;
    const PartLayout pl(cap);
    return (int)hipMemsetAsync(reinterpret_cast<char*>(partial) + pl.fl, 0, (size_t)cap, s);
}

}  // namespace gsr

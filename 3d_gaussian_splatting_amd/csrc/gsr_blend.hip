// gsr_blend.hip -- F6 per-tile front-to-back alpha blend and B1 per-tile back-to-front
// gradient pass on gfx950.
//
// One wave64 per 16x16 tile, 4 pixels per lane (lane l: column l&15, rows (l>>4)+4p).  A
// whole tile in one wave means: the "all pixels done" early-out is one ballot (no block
// barrier), and each LDS-staged record (3 x ds_read_b128, broadcast) feeds 4 pixel
// evaluations instead of 1, which keeps the loop VALU-bound rather than LDS-bound.
// Batches of 64 records are gathered by the wave's 64 lanes (one record per lane: 3
// dwordx4 loads from the record array), staged in LDS, then swept by every lane.
//
// Workgroup -> tile mapping is XCD-aware: blocks b, b+8, ... land on one XCD (observed
// round-robin dispatch, speed only), so each XCD gets a contiguous band of tile rows and
// its L2 keeps the records those neighbouring tiles share.
//
// B1 reduces each record's 9 gradient terms over the tile's 256 pixels in registers
// (4 pixels per lane, then a 6-step DPP wave reduction) and writes ONE 48-B partial per
// (tile, instance) with plain stores, indexed by the instance's emission index j.  The
// per-Gaussian sum happens later in fixed emission order (gsr_preprocess_bwd.hip), so
// gradients are deterministic and no float atomics are issued (at 1M/1080p, 9 scattered
// atomics per instance would run at the ~0.08 TB/s scattered-atomic rate).
//
// Roofline: VALU-bound (exp + ~20 flops per pixel x record pair); HBM traffic per tile is
// the gathered 48-B records + per-pixel I/O.
#include <cstdlib>

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

// Row-level (16-lane) all-reduce of N independent values, step-interleaved so consecutive
// DPP reads never hit the VGPR written by the instruction right before (no s_nop hazards).
template <int N>
__device__ inline void row_reduce(float (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dpp_f<0xB1>(v[i]);   // quad_perm [1,0,3,2]
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dpp_f<0x4E>(v[i]);   // quad_perm [2,3,0,1]
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dpp_f<0x141>(v[i]);  // row_half_mirror
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += dpp_f<0x140>(v[i]);  // row_mirror
}

__device__ inline float fsum_pair(uint2 r) { return __uint_as_float(r.x) + __uint_as_float(r.y); }

// gfx950 reduce-scatter of four row-reduced values: afterwards lanes of row 0/1/2/3 hold the
// 64-lane totals of a/b/c/d.  v_permlane16_swap swaps VDST rows 1,3 with VSRC rows 0,2;
// v_permlane32_swap swaps VDST lanes 32-63 with VSRC lanes 0-31.
__device__ inline float scatter4(float a, float b, float c, float d) {
    auto ab = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    auto cd = __builtin_amdgcn_permlane16_swap(__float_as_uint(c), __float_as_uint(d), false, false);
    const float x = __uint_as_float(ab[0]) + __uint_as_float(ab[1]);  // rows: a01 b01 a23 b23
    const float y = __uint_as_float(cd[0]) + __uint_as_float(cd[1]);  // rows: c01 d01 c23 d23
    auto xy = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
    return __uint_as_float(xy[0]) + __uint_as_float(xy[1]);           // rows: a b c d
}

// full 64-lane all-reduce of a row-reduced value (every lane gets the total)
__device__ inline float allreduce_rows(float a) {
    auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
    const float x = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
    auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
}

__device__ inline uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(x, o, 64);
        x = x > y ? x : y;
    }
    return x;
}

struct BlendGeom {
    int W, H, grid_x, ty0, nwg;
    float bg0, bg1, bg2;
};

// Which of the tile's four 16x4 pixel stripes (slot p = rows 4p..4p+3) the record's
// alpha >= 1/255 footprint box can touch.  Exact culling: a pixel outside the (padded) box
// fails the alpha test, so skipping it changes no output bit.
__device__ inline uint32_t stripe_mask(const float4 r0, const float4 r2, float bx0, float by0) {
    const float ex = r2.y, ey = r2.z;
    if (!(ex >= 0.0f) || r0.x + ex < bx0 || r0.x - ex > bx0 + 15.0f) return 0u;
    const float ylo = r0.y - ey, yhi = r0.y + ey;
    uint32_t m = 0;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const float s0 = by0 + 4.0f * p;
        m |= (yhi >= s0 && ylo <= s0 + 3.0f) ? (1u << p) : 0u;
    }
    return m;
}

// SLOT_CULL: skip culled 16x4 stripes with a wave-uniform branch (fewer VALU ops) or
// evaluate all four stripes predicated (independent chains the scheduler can interleave).
template <bool SLOT_CULL>
__global__ __launch_bounds__(64) void blend_forward_kernel(const BlendGeom geo,
                                                           const uint2* __restrict__ ranges,
                                                           const uint32_t* __restrict__ sorted_gid,
                                                           const float4* __restrict__ rec,
                                                           float* __restrict__ out_color,
                                                           float* __restrict__ final_T,
                                                           uint32_t* __restrict__ n_contrib,
                                                           float* __restrict__ accum) {
    __shared__ float4 srec[64 * 3];
    const int tile = xcd_tile(blockIdx.x, geo.nwg) + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
    float pfy[kPPL], T[kPPL], C0[kPPL], C1[kPPL], C2[kPPL];
    uint32_t last[kPPL];
    bool done[kPPL];
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        pfy[p] = (float)py;
        T[p] = 1.0f;
        C0[p] = C1[p] = C2[p] = 0.0f;
        last[p] = 0;
        done[p] = !(px < geo.W && py < geo.H);
    }
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    for (int base = 0; base < n; base += 64) {
        uint32_t live = 0;  // stripes with at least one unfinished pixel (wave-uniform)
#pragma unroll
        for (int p = 0; p < kPPL; ++p) live |= __all(done[p]) ? 0u : (1u << p);
        if (live == 0) break;
        uint32_t smask = 0;
        if (base + lane < n) {
            const uint32_t g = sorted_gid[range.x + base + lane];
            const float4* r = rec + 3 * (size_t)g;
            const float4 r0 = r[0], r1 = r[1], r2 = r[2];
            srec[3 * lane + 0] = r0;
            srec[3 * lane + 1] = r1;
            srec[3 * lane + 2] = r2;
            smask = stripe_mask(r0, r2, bx0, by0);
        }
        __syncthreads();
        uint64_t todo = __ballot((smask & live) != 0u);
        int visited = 0;
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)smask, k) & live;
            const float4 r0 = srec[3 * k + 0];  // x, y, a', b'
            const float4 r1 = srec[3 * k + 1];  // c', opacity, r, g
            const float rb = srec[3 * k + 2].x; // b
            const uint32_t idx = (uint32_t)(base + k + 1);
#pragma unroll
            for (int p = 0; p < kPPL; ++p) {
                if (SLOT_CULL && !(m & (1u << p))) continue;  // wave-uniform
                const float dx = r0.x - pfx, dy = r0.y - pfy[p];
                const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
                const float alpha = fminf(0.99f, r1.y * __builtin_amdgcn_exp2f(pw));
                const bool valid = (SLOT_CULL || (m & (1u << p))) && !done[p] && pw <= 0.0f &&
                                   alpha >= (1.0f / 255.0f);
                const float tT = T[p] * (1.0f - alpha);
                const bool term = valid && tT < 0.0001f;
                const bool contrib = valid && !term;
                done[p] = done[p] || term;
                const float w = contrib ? alpha * T[p] : 0.0f;
                C0[p] = fmaf(r1.z, w, C0[p]);
                C1[p] = fmaf(r1.w, w, C1[p]);
                C2[p] = fmaf(rb, w, C2[p]);
                T[p] = contrib ? tT : T[p];
                last[p] = contrib ? idx : last[p];
            }
            if ((++visited & 7) == 0) {
                uint32_t lv = 0;
#pragma unroll
                for (int p = 0; p < kPPL; ++p) lv |= __all(done[p]) ? 0u : (1u << p);
                live = lv;
                if (live == 0) break;
            }
        }
        __syncthreads();
    }
    const size_t npix = (size_t)geo.W * geo.H;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        if (px < geo.W && py < geo.H) {
            const size_t pix = (size_t)py * geo.W + px;
            final_T[pix] = T[p];
            n_contrib[pix] = last[p];
            accum[pix] = C0[p];
            accum[npix + pix] = C1[p];
            accum[2 * npix + pix] = C2[p];
            out_color[pix] = C0[p] + T[p] * geo.bg0;
            out_color[npix + pix] = C1[p] + T[p] * geo.bg1;
            out_color[2 * npix + pix] = C2[p] + T[p] * geo.bg2;
        }
    }
}

template <bool SLOT_CULL>
__global__ __launch_bounds__(64) void blend_backward_kernel(const BlendGeom geo,
                                                            const uint2* __restrict__ ranges,
                                                            const uint32_t* __restrict__ sorted_gid,
                                                            const uint32_t* __restrict__ inst_start,
                                                            const uint2* __restrict__ rect,
                                                            const float4* __restrict__ rec,
                                                            const float* __restrict__ final_T,
                                                            const uint32_t* __restrict__ n_contrib,
                                                            const float* __restrict__ dL_dpix,
                                                            float* __restrict__ partial) {
    __shared__ float4 srec[64 * 3];
    __shared__ float smom[64 * 12];  // per batch entry: Sx Sy Sxx Sxy | Syy S0 gr gg | gb - - -
    const int tile = xcd_tile(blockIdx.x, geo.nwg) + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
    const size_t npix = (size_t)geo.W * geo.H;
    const float hw = 0.5f * (float)geo.W, hh = 0.5f * (float)geo.H;
    // per-pixel state (4 pixels per lane)
    float T[kPPL], dp0[kPPL], dp1[kPPL], dp2[kPPL], cbg[kPPL];
    float ac0[kPPL], ac1[kPPL], ac2[kPPL], lc0[kPPL], lc1[kPPL], lc2[kPPL], la[kPPL];
    uint32_t lastc[kPPL];
    uint32_t maxlast = 0;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        const bool in = px < geo.W && py < geo.H;
        const size_t pix = in ? (size_t)py * geo.W + px : 0;
        const float Tf = in ? final_T[pix] : 1.0f;
        T[p] = Tf;
        lastc[p] = in ? n_contrib[pix] : 0u;
        dp0[p] = in ? dL_dpix[pix] : 0.0f;
        dp1[p] = in ? dL_dpix[npix + pix] : 0.0f;
        dp2[p] = in ? dL_dpix[2 * npix + pix] : 0.0f;
        cbg[p] = -Tf * (geo.bg0 * dp0[p] + geo.bg1 * dp1[p] + geo.bg2 * dp2[p]);
        ac0[p] = ac1[p] = ac2[p] = lc0[p] = lc1[p] = lc2[p] = la[p] = 0.0f;
        maxlast = maxlast > lastc[p] ? maxlast : lastc[p];
    }
    maxlast = wave_max_u32(maxlast);
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    const int row = lane >> 4;
    for (int top = n; top > 0; top -= 64) {
        const int lo = top > 64 ? top - 64 : 0;
        const int cnt = top - lo;
        const int e_l = top - 1 - lane;  // this lane's entry (descending)
        uint32_t jl = 0, smask = 0;
        float4 q0 = make_float4(0.f, 0.f, 0.f, 0.f), q1 = q0;  // this lane's record (conic)
        if (lane < cnt) {
            const uint32_t g = sorted_gid[range.x + e_l];
            // emission index of (g, this tile): g's first instance + row-major offset in its
            // band-clipped rect (the order duplicate emitted them in)
            const uint2 rr = rect[g];
            const int minx = rr.x & 0xFFFF, miny = rr.x >> 16, maxx = rr.y & 0xFFFF;
            const int y0 = miny > geo.ty0 ? miny : geo.ty0;
            jl = inst_start[g] + (uint32_t)((ty - y0) * (maxx - minx) + (tx - minx));
            if (e_l < (int)maxlast) {
                const float4* r = rec + 3 * (size_t)g;
                q0 = r[0];
                q1 = r[1];
                const float4 r2 = r[2];
                srec[3 * lane + 0] = q0;
                srec[3 * lane + 1] = q1;
                srec[3 * lane + 2] = r2;
                smask = stripe_mask(q0, r2, bx0, by0);
            }
        }
#pragma unroll
        for (int c = 0; c < 12; ++c) smom[lane * 12 + c] = 0.0f;
        __syncthreads();
        uint64_t todo = __ballot(smask != 0u);
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)smask, k);
            const uint32_t e = (uint32_t)(top - 1 - k);
            const float4 r0 = srec[3 * k + 0];  // x, y, a', b'
            const float4 r1 = srec[3 * k + 1];  // c', o, r, g
            const float rb = srec[3 * k + 2].x;
            // moments of s = G * o * dL/dalpha over the tile's pixels (+ colour sums)
            float v[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            bool any = false;
#pragma unroll
            for (int p = 0; p < kPPL; ++p) {
                if (SLOT_CULL && !(m & (1u << p))) continue;  // wave-uniform
                const float dx = r0.x - pfx, dy = r0.y - (by0 + (float)(row + 4 * p));
                const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
                const float G = __builtin_amdgcn_exp2f(pw);
                const float alpha = fminf(0.99f, r1.y * G);
                const bool valid = (SLOT_CULL || (m & (1u << p))) && e < lastc[p] && pw <= 0.0f &&
                                   alpha >= (1.0f / 255.0f);
                if (valid) {
                    any = true;
                    const float inv = __builtin_amdgcn_rcpf(1.0f - alpha);
                    T[p] = T[p] * inv;
                    const float dch = alpha * T[p];
                    ac0[p] = fmaf(la[p], lc0[p] - ac0[p], ac0[p]);
                    ac1[p] = fmaf(la[p], lc1[p] - ac1[p], ac1[p]);
                    ac2[p] = fmaf(la[p], lc2[p] - ac2[p], ac2[p]);
                    lc0[p] = r1.z;
                    lc1[p] = r1.w;
                    lc2[p] = rb;
                    la[p] = alpha;
                    float dLda = (r1.z - ac0[p]) * dp0[p];
                    dLda = fmaf(r1.w - ac1[p], dp1[p], dLda);
                    dLda = fmaf(rb - ac2[p], dp2[p], dLda);
                    v[6] = fmaf(dch, dp0[p], v[6]);
                    v[7] = fmaf(dch, dp1[p], v[7]);
                    v[8] = fmaf(dch, dp2[p], v[8]);
                    dLda = fmaf(dLda, T[p], cbg[p] * inv);
                    const float GdL = G * dLda;
                    v[5] += GdL;
                    const float sv = r1.y * GdL;
                    const float sx = sv * dx, sy = sv * dy;
                    v[0] += sx;
                    v[1] += sy;
                    v[2] = fmaf(sx, dx, v[2]);
                    v[3] = fmaf(sx, dy, v[3]);
                    v[4] = fmaf(sy, dy, v[4]);
                }
            }
            if (__any(any)) {
                row_reduce(v);
                const float t0 = scatter4(v[0], v[1], v[2], v[3]);  // rows: Sx Sy Sxx Sxy
                const float t1 = scatter4(v[4], v[5], v[6], v[7]);  // rows: Syy S0 gr gg
                const float t2 = allreduce_rows(v[8]);              // gb everywhere
                if ((lane & 15) == 0) {
                    smom[k * 12 + row] = t0;
                    smom[k * 12 + 4 + row] = t1;
                    if (row == 0) smom[k * 12 + 8] = t2;
                }
            }
        }
        __syncthreads();
        if (lane < cnt) {
            // raw moments -> 2D gradients with this entry's own conic
            const float* mo = smom + lane * 12;
            const float Sx = mo[0], Sy = mo[1], Sxx = mo[2], Sxy = mo[3], Syy = mo[4], S0 = mo[5];
            const float A = -2.0f * kLn2 * q0.z, B = -kLn2 * q0.w, C = -2.0f * kLn2 * q1.x;
            float4* dst = reinterpret_cast<float4*>(partial + (size_t)kPart * jl);
            dst[0] = make_float4((-A * Sx - B * Sy) * hw, (-C * Sy - B * Sx) * hh, -0.5f * Sxx, -Sxy);
            dst[1] = make_float4(-0.5f * Syy, S0, mo[6], mo[7]);
            dst[2] = make_float4(mo[8], 0.f, 0.f, 0.f);
        }
        __syncthreads();
    }
}


// Forward, SALU-light body: every predicate is a v_cmp feeding a v_cndmask (no s_and/s_or
// of lane masks per pixel); finished pixels carry T = 0 so they contribute nothing, with the
// transmittance after their last contribution kept in Tf.
__global__ __launch_bounds__(64) void blend_forward_v2_kernel(const BlendGeom geo,
                                                              const uint2* __restrict__ ranges,
                                                              const uint32_t* __restrict__ sorted_gid,
                                                              const float4* __restrict__ rec,
                                                              float* __restrict__ out_color,
                                                              float* __restrict__ final_T,
                                                              uint32_t* __restrict__ n_contrib,
                                                              float* __restrict__ accum) {
    __shared__ float4 srec[64 * 3];
    const int tile = xcd_tile(blockIdx.x, geo.nwg) + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
    float pfy[kPPL], T[kPPL], Tf[kPPL], C0[kPPL], C1[kPPL], C2[kPPL];
    uint32_t last[kPPL];
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        pfy[p] = (float)py;
        T[p] = (px < geo.W && py < geo.H) ? 1.0f : 0.0f;
        Tf[p] = 1.0f;
        C0[p] = C1[p] = C2[p] = 0.0f;
        last[p] = 0;
    }
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    for (int base = 0; base < n; base += 64) {
        uint32_t live = 0;
#pragma unroll
        for (int p = 0; p < kPPL; ++p) live |= __all(T[p] == 0.0f) ? 0u : (1u << p);
        if (live == 0) break;
        uint32_t smask = 0;
        if (base + lane < n) {
            const uint32_t g = sorted_gid[range.x + base + lane];
            const float4* r = rec + 3 * (size_t)g;
            const float4 r0 = r[0], r1 = r[1], r2 = r[2];
            srec[3 * lane + 0] = r0;
            srec[3 * lane + 1] = r1;
            srec[3 * lane + 2] = r2;
            smask = stripe_mask(r0, r2, bx0, by0);
        }
        __syncthreads();
        uint64_t todo = __ballot((smask & live) != 0u);
        int visited = 0;
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)smask, k) & live;
            const float4 r0 = srec[3 * k + 0];
            const float4 r1 = srec[3 * k + 1];
            const float rb = srec[3 * k + 2].x;
            const uint32_t idx = (uint32_t)(base + k + 1);
#pragma unroll
            for (int p = 0; p < kPPL; ++p) {
                if (!(m & (1u << p))) continue;  // wave-uniform
                const float dx = r0.x - pfx, dy = r0.y - pfy[p];
                const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
                float a = fminf(0.99f, r1.y * __builtin_amdgcn_exp2f(pw));
                a = pw <= 0.0f ? a : 0.0f;
                a = a >= (1.0f / 255.0f) ? a : 0.0f;
                const float tT = T[p] * (1.0f - a);
                const bool ok = tT >= 0.0001f;
                const float w = ok ? a * T[p] : 0.0f;
                C0[p] = fmaf(r1.z, w, C0[p]);
                C1[p] = fmaf(r1.w, w, C1[p]);
                C2[p] = fmaf(rb, w, C2[p]);
                const bool used = w > 0.0f;
                last[p] = used ? idx : last[p];
                Tf[p] = used ? tT : Tf[p];
                T[p] = a > 0.0f ? (ok ? tT : 0.0f) : T[p];
            }
            if ((++visited & 7) == 0) {
                uint32_t lv = 0;
#pragma unroll
                for (int p = 0; p < kPPL; ++p) lv |= __all(T[p] == 0.0f) ? 0u : (1u << p);
                live = lv;
                if (live == 0) break;
            }
        }
        __syncthreads();
    }
    const size_t npix = (size_t)geo.W * geo.H;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        if (px < geo.W && py < geo.H) {
            const size_t pix = (size_t)py * geo.W + px;
            final_T[pix] = Tf[p];
            n_contrib[pix] = last[p];
            accum[pix] = C0[p];
            accum[npix + pix] = C1[p];
            accum[2 * npix + pix] = C2[p];
            out_color[pix] = C0[p] + Tf[p] * geo.bg0;
            out_color[npix + pix] = C1[p] + Tf[p] * geo.bg1;
            out_color[2 * npix + pix] = C2[p] + Tf[p] * geo.bg2;
        }
    }
}

// B1 front to back.  With S = the forward's colour sum (no background) and the running
// Sp = sum over processed contributors of w * (c . dL/dpix), the colour behind entry k is
// (S . dL/dpix - Sp) / (1 - alpha_k) after T_k, so
//   dL/dalpha_k = T_k (c_k . dL/dpix) - (S . dL/dpix - Sp + T_final bg . dL/dpix) / (1 - alpha_k)
// (SURVEY B.4 rewritten; same value as the back-to-front recursion).  Per-pixel state is two
// floats (T, Sp) and T is recomputed with the forward's own T * (1 - alpha) -- no divisions.
template <bool SLOT_CULL>
__global__ __launch_bounds__(64) void blend_backward_f2b_kernel(const BlendGeom geo,
                                                                const uint2* __restrict__ ranges,
                                                                const uint32_t* __restrict__ sorted_gid,
                                                                const uint32_t* __restrict__ inst_start,
                                                                const uint2* __restrict__ rect,
                                                                const float4* __restrict__ rec,
                                                                const float* __restrict__ final_T,
                                                                const uint32_t* __restrict__ n_contrib,
                                                                const float* __restrict__ accum,
                                                                const float* __restrict__ dL_dpix,
                                                                float* __restrict__ partial) {
    __shared__ float4 srec[64 * 3];
    __shared__ float smom[64 * 12];
    const int tile = xcd_tile(blockIdx.x, geo.nwg) + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
    const size_t npix = (size_t)geo.W * geo.H;
    const float hw = 0.5f * (float)geo.W, hh = 0.5f * (float)geo.H;
    const int row = lane >> 4;
    float T[kPPL], Sp[kPPL], cb[kPPL], dp0[kPPL], dp1[kPPL], dp2[kPPL];
    uint32_t lastc[kPPL];
    uint32_t maxlast = 0;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + row + 4 * p;
        const bool in = px < geo.W && py < geo.H;
        const size_t pix = in ? (size_t)py * geo.W + px : 0;
        const float Tfin = in ? final_T[pix] : 1.0f;
        lastc[p] = in ? n_contrib[pix] : 0u;
        dp0[p] = in ? dL_dpix[pix] : 0.0f;
        dp1[p] = in ? dL_dpix[npix + pix] : 0.0f;
        dp2[p] = in ? dL_dpix[2 * npix + pix] : 0.0f;
        const float sdp = in ? accum[pix] * dp0[p] + accum[npix + pix] * dp1[p] + accum[2 * npix + pix] * dp2[p]
                             : 0.0f;
        cb[p] = sdp + Tfin * (geo.bg0 * dp0[p] + geo.bg1 * dp1[p] + geo.bg2 * dp2[p]);
        T[p] = 1.0f;
        Sp[p] = 0.0f;
        maxlast = maxlast > lastc[p] ? maxlast : lastc[p];
    }
    maxlast = wave_max_u32(maxlast);
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    for (int base = 0; base < n; base += 64) {
        const int cnt = (n - base) < 64 ? (n - base) : 64;
        const int e_l = base + lane;
        uint32_t jl = 0, smask = 0;
        float4 q0 = make_float4(0.f, 0.f, 0.f, 0.f), q1 = q0;
        if (lane < cnt) {
            const uint32_t g = sorted_gid[range.x + e_l];
            const uint2 rr = rect[g];
            const int minx = rr.x & 0xFFFF, miny = rr.x >> 16, maxx = rr.y & 0xFFFF;
            const int y0 = miny > geo.ty0 ? miny : geo.ty0;
            jl = inst_start[g] + (uint32_t)((ty - y0) * (maxx - minx) + (tx - minx));
            if (e_l < (int)maxlast) {
                const float4* r = rec + 3 * (size_t)g;
                q0 = r[0];
                q1 = r[1];
                const float4 r2 = r[2];
                srec[3 * lane + 0] = q0;
                srec[3 * lane + 1] = q1;
                srec[3 * lane + 2] = r2;
                smask = stripe_mask(q0, r2, bx0, by0);
            }
        }
#pragma unroll
        for (int c = 0; c < 12; ++c) smom[lane * 12 + c] = 0.0f;
        __syncthreads();
        uint64_t todo = __ballot(smask != 0u);
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)smask, k);
            const uint32_t e = (uint32_t)(base + k);
            const float4 r0 = srec[3 * k + 0];
            const float4 r1 = srec[3 * k + 1];
            const float rb = srec[3 * k + 2].x;
            float v[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            bool any = false;
#pragma unroll
            for (int p = 0; p < kPPL; ++p) {
                if (SLOT_CULL && !(m & (1u << p))) continue;  // wave-uniform
                const float dx = r0.x - pfx, dy = r0.y - (by0 + (float)(row + 4 * p));
                const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
                const float G = __builtin_amdgcn_exp2f(pw);
                const float oG = r1.y * G;
                const float alpha = fminf(0.99f, oG);
                const bool valid = (SLOT_CULL || (m & (1u << p))) && e < lastc[p] && pw <= 0.0f &&
                                   alpha >= (1.0f / 255.0f);
                if (valid) {
                    any = true;
                    const float w = alpha * T[p];
                    const float cdp = fmaf(r1.z, dp0[p], fmaf(r1.w, dp1[p], rb * dp2[p]));
                    Sp[p] = fmaf(w, cdp, Sp[p]);
                    const float one_m = 1.0f - alpha;
                    const float dLda = fmaf(T[p], cdp, -(cb[p] - Sp[p]) * __builtin_amdgcn_rcpf(one_m));
                    T[p] = T[p] * one_m;
                    v[6] = fmaf(w, dp0[p], v[6]);
                    v[7] = fmaf(w, dp1[p], v[7]);
                    v[8] = fmaf(w, dp2[p], v[8]);
                    v[5] = fmaf(G, dLda, v[5]);
                    const float sv = oG * dLda;
                    const float sx = sv * dx, sy = sv * dy;
                    v[0] += sx;
                    v[1] += sy;
                    v[2] = fmaf(sx, dx, v[2]);
                    v[3] = fmaf(sx, dy, v[3]);
                    v[4] = fmaf(sy, dy, v[4]);
                }
            }
            if (__any(any)) {
                row_reduce(v);
                const float t0 = scatter4(v[0], v[1], v[2], v[3]);
                const float t1 = scatter4(v[4], v[5], v[6], v[7]);
                const float t2 = allreduce_rows(v[8]);
                if ((lane & 15) == 0) {
                    smom[k * 12 + row] = t0;
                    smom[k * 12 + 4 + row] = t1;
                    if (row == 0) smom[k * 12 + 8] = t2;
                }
            }
        }
        __syncthreads();
        if (lane < cnt) {
            const float* mo = smom + lane * 12;
            const float Sx = mo[0], Sy = mo[1], Sxx = mo[2], Sxy = mo[3], Syy = mo[4], S0 = mo[5];
            const float A = -2.0f * kLn2 * q0.z, B = -kLn2 * q0.w, C = -2.0f * kLn2 * q1.x;
            float4* dst = reinterpret_cast<float4*>(partial + (size_t)kPart * jl);
            dst[0] = make_float4((-A * Sx - B * Sy) * hw, (-C * Sy - B * Sx) * hh, -0.5f * Sxx, -Sxy);
            dst[1] = make_float4(-0.5f * Syy, S0, mo[6], mo[7]);
            dst[2] = make_float4(mo[8], 0.f, 0.f, 0.f);
        }
        __syncthreads();
    }
}


// Forward with the record gathers software-pipelined: batch b+1's records (and batch b+2's
// Gaussian ids) are loaded into registers while batch b is blended from LDS, so the
// gather latency (L2 / Infinity Cache / HBM, 500-900 cycles) is off the critical path.
__global__ __launch_bounds__(64) void blend_forward_v3_kernel(const BlendGeom geo,
                                                              const uint2* __restrict__ ranges,
                                                              const uint32_t* __restrict__ sorted_gid,
                                                              const float4* __restrict__ rec,
                                                              float* __restrict__ out_color,
                                                              float* __restrict__ final_T,
                                                              uint32_t* __restrict__ n_contrib,
                                                              float* __restrict__ accum) {
    __shared__ float4 srec[64 * 3];
    const int tile = xcd_tile(blockIdx.x, geo.nwg) + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
    float pfy[kPPL], T[kPPL], Tf[kPPL], C0[kPPL], C1[kPPL], C2[kPPL];
    uint32_t last[kPPL];
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        pfy[p] = (float)py;
        T[p] = (px < geo.W && py < geo.H) ? 1.0f : 0.0f;
        Tf[p] = 1.0f;
        C0[p] = C1[p] = C2[p] = 0.0f;
        last[p] = 0;
    }
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    // prologue: ids of batches 0 and 1, records of batch 0
    uint32_t g_next = (64 + lane < n) ? sorted_gid[range.x + 64 + lane] : 0u;
    float4 p0 = make_float4(0.f, 0.f, 0.f, 0.f), p1 = p0, p2 = p0;
    if (lane < n) {
        const float4* r = rec + 3 * (size_t)sorted_gid[range.x + lane];
        p0 = r[0];
        p1 = r[1];
        p2 = r[2];
    }
    for (int base = 0; base < n; base += 64) {
        uint32_t live = 0;
#pragma unroll
        for (int p = 0; p < kPPL; ++p) live |= __all(T[p] == 0.0f) ? 0u : (1u << p);
        if (live == 0) break;
        uint32_t smask = 0;
        if (base + lane < n) {
            srec[3 * lane + 0] = p0;
            srec[3 * lane + 1] = p1;
            srec[3 * lane + 2] = p2;
            smask = stripe_mask(p0, p2, bx0, by0);
        }
        __syncthreads();
        // prefetch: records of batch base+64, id of batch base+128
        if (base + 64 + lane < n) {
            const float4* r = rec + 3 * (size_t)g_next;
            p0 = r[0];
            p1 = r[1];
            p2 = r[2];
        }
        g_next = (base + 128 + lane < n) ? sorted_gid[range.x + base + 128 + lane] : 0u;
        uint64_t todo = __ballot((smask & live) != 0u);
        int visited = 0;
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)smask, k) & live;
            const float4 r0 = srec[3 * k + 0];
            const float4 r1 = srec[3 * k + 1];
            const float rb = srec[3 * k + 2].x;
            const uint32_t idx = (uint32_t)(base + k + 1);
#pragma unroll
            for (int p = 0; p < kPPL; ++p) {
                if (!(m & (1u << p))) continue;  // wave-uniform
                const float dx = r0.x - pfx, dy = r0.y - pfy[p];
                const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
                float a = fminf(0.99f, r1.y * __builtin_amdgcn_exp2f(pw));
                a = pw <= 0.0f ? a : 0.0f;
                a = a >= (1.0f / 255.0f) ? a : 0.0f;
                const float tT = T[p] * (1.0f - a);
                const bool ok = tT >= 0.0001f;
                const float w = ok ? a * T[p] : 0.0f;
                C0[p] = fmaf(r1.z, w, C0[p]);
                C1[p] = fmaf(r1.w, w, C1[p]);
                C2[p] = fmaf(rb, w, C2[p]);
                const bool used = w > 0.0f;
                last[p] = used ? idx : last[p];
                Tf[p] = used ? tT : Tf[p];
                T[p] = a > 0.0f ? (ok ? tT : 0.0f) : T[p];
            }
            if ((++visited & 7) == 0) {
                uint32_t lv = 0;
#pragma unroll
                for (int p = 0; p < kPPL; ++p) lv |= __all(T[p] == 0.0f) ? 0u : (1u << p);
                live = lv;
                if (live == 0) break;
            }
        }
        __syncthreads();
    }
    const size_t npix = (size_t)geo.W * geo.H;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        if (px < geo.W && py < geo.H) {
            const size_t pix = (size_t)py * geo.W + px;
            final_T[pix] = Tf[p];
            n_contrib[pix] = last[p];
            accum[pix] = C0[p];
            accum[npix + pix] = C1[p];
            accum[2 * npix + pix] = C2[p];
            out_color[pix] = C0[p] + Tf[p] * geo.bg0;
            out_color[npix + pix] = C1[p] + Tf[p] * geo.bg1;
            out_color[2 * npix + pix] = C2[p] + Tf[p] * geo.bg2;
        }
    }
}

template <bool SLOT_CULL>
__global__ __launch_bounds__(64) void blend_backward_f2b_pf_kernel(const BlendGeom geo,
                                                                const uint2* __restrict__ ranges,
                                                                const uint32_t* __restrict__ sorted_gid,
                                                                const uint32_t* __restrict__ inst_start,
                                                                const uint2* __restrict__ rect,
                                                                const float4* __restrict__ rec,
                                                                const float* __restrict__ final_T,
                                                                const uint32_t* __restrict__ n_contrib,
                                                                const float* __restrict__ accum,
                                                                const float* __restrict__ dL_dpix,
                                                                float* __restrict__ partial) {
    __shared__ float4 srec[64 * 3];
    __shared__ float smom[64 * 12];
    const int tile = xcd_tile(blockIdx.x, geo.nwg) + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
    const size_t npix = (size_t)geo.W * geo.H;
    const float hw = 0.5f * (float)geo.W, hh = 0.5f * (float)geo.H;
    const int row = lane >> 4;
    float T[kPPL], Sp[kPPL], cb[kPPL], dp0[kPPL], dp1[kPPL], dp2[kPPL];
    uint32_t lastc[kPPL];
    uint32_t maxlast = 0;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + row + 4 * p;
        const bool in = px < geo.W && py < geo.H;
        const size_t pix = in ? (size_t)py * geo.W + px : 0;
        const float Tfin = in ? final_T[pix] : 1.0f;
        lastc[p] = in ? n_contrib[pix] : 0u;
        dp0[p] = in ? dL_dpix[pix] : 0.0f;
        dp1[p] = in ? dL_dpix[npix + pix] : 0.0f;
        dp2[p] = in ? dL_dpix[2 * npix + pix] : 0.0f;
        const float sdp = in ? accum[pix] * dp0[p] + accum[npix + pix] * dp1[p] + accum[2 * npix + pix] * dp2[p]
                             : 0.0f;
        cb[p] = sdp + Tfin * (geo.bg0 * dp0[p] + geo.bg1 * dp1[p] + geo.bg2 * dp2[p]);
        T[p] = 1.0f;
        Sp[p] = 0.0f;
        maxlast = maxlast > lastc[p] ? maxlast : lastc[p];
    }
    maxlast = wave_max_u32(maxlast);
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    // prologue: batch 0's id, rect, inst_start and record; batch 1's id (software pipeline)
    uint32_t g_cur = lane < n ? sorted_gid[range.x + lane] : 0u;
    uint32_t g_next = (64 + lane < n) ? sorted_gid[range.x + 64 + lane] : 0u;
    uint2 rr_p = make_uint2(0u, 0u);
    uint32_t is_p = 0;
    float4 p0 = make_float4(0.f, 0.f, 0.f, 0.f), p1 = p0, p2 = p0;
    if (lane < n) {
        rr_p = rect[g_cur];
        is_p = inst_start[g_cur];
        if (lane < (int)maxlast) {
            const float4* r = rec + 3 * (size_t)g_cur;
            p0 = r[0];
            p1 = r[1];
            p2 = r[2];
        }
    }
    for (int base = 0; base < n; base += 64) {
        const int cnt = (n - base) < 64 ? (n - base) : 64;
        const int e_l = base + lane;
        uint32_t jl = 0, smask = 0;
        const float4 q0 = p0, q1 = p1;
        if (lane < cnt) {
            const int minx = rr_p.x & 0xFFFF, miny = rr_p.x >> 16, maxx = rr_p.y & 0xFFFF;
            const int y0 = miny > geo.ty0 ? miny : geo.ty0;
            jl = is_p + (uint32_t)((ty - y0) * (maxx - minx) + (tx - minx));
            if (e_l < (int)maxlast) {
                srec[3 * lane + 0] = p0;
                srec[3 * lane + 1] = p1;
                srec[3 * lane + 2] = p2;
                smask = stripe_mask(p0, p2, bx0, by0);
            }
        }
        // prefetch batch base+64 (rect, inst_start, record) and the id of batch base+128
        {
            const int e_n = base + 64 + lane;
            if (e_n < n) {
                rr_p = rect[g_next];
                is_p = inst_start[g_next];
                if (e_n < (int)maxlast) {
                    const float4* r = rec + 3 * (size_t)g_next;
                    p0 = r[0];
                    p1 = r[1];
                    p2 = r[2];
                }
            }
            g_next = (base + 128 + lane < n) ? sorted_gid[range.x + base + 128 + lane] : 0u;
        }
#pragma unroll
        for (int c = 0; c < 12; ++c) smom[lane * 12 + c] = 0.0f;
        __syncthreads();
        uint64_t todo = __ballot(smask != 0u);
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)smask, k);
            const uint32_t e = (uint32_t)(base + k);
            const float4 r0 = srec[3 * k + 0];
            const float4 r1 = srec[3 * k + 1];
            const float rb = srec[3 * k + 2].x;
            float v[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            bool any = false;
#pragma unroll
            for (int p = 0; p < kPPL; ++p) {
                if (SLOT_CULL && !(m & (1u << p))) continue;  // wave-uniform
                const float dx = r0.x - pfx, dy = r0.y - (by0 + (float)(row + 4 * p));
                const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
                const float G = __builtin_amdgcn_exp2f(pw);
                const float oG = r1.y * G;
                const float alpha = fminf(0.99f, oG);
                const bool valid = (SLOT_CULL || (m & (1u << p))) && e < lastc[p] && pw <= 0.0f &&
                                   alpha >= (1.0f / 255.0f);
                if (valid) {
                    any = true;
                    const float w = alpha * T[p];
                    const float cdp = fmaf(r1.z, dp0[p], fmaf(r1.w, dp1[p], rb * dp2[p]));
                    Sp[p] = fmaf(w, cdp, Sp[p]);
                    const float one_m = 1.0f - alpha;
                    const float dLda = fmaf(T[p], cdp, -(cb[p] - Sp[p]) * __builtin_amdgcn_rcpf(one_m));
                    T[p] = T[p] * one_m;
                    v[6] = fmaf(w, dp0[p], v[6]);
                    v[7] = fmaf(w, dp1[p], v[7]);
                    v[8] = fmaf(w, dp2[p], v[8]);
                    v[5] = fmaf(G, dLda, v[5]);
                    const float sv = oG * dLda;
                    const float sx = sv * dx, sy = sv * dy;
                    v[0] += sx;
                    v[1] += sy;
                    v[2] = fmaf(sx, dx, v[2]);
                    v[3] = fmaf(sx, dy, v[3]);
                    v[4] = fmaf(sy, dy, v[4]);
                }
            }
            if (__any(any)) {
                row_reduce(v);
                const float t0 = scatter4(v[0], v[1], v[2], v[3]);
                const float t1 = scatter4(v[4], v[5], v[6], v[7]);
                const float t2 = allreduce_rows(v[8]);
                if ((lane & 15) == 0) {
                    smom[k * 12 + row] = t0;
                    smom[k * 12 + 4 + row] = t1;
                    if (row == 0) smom[k * 12 + 8] = t2;
                }
            }
        }
        __syncthreads();
        if (lane < cnt) {
            const float* mo = smom + lane * 12;
            const float Sx = mo[0], Sy = mo[1], Sxx = mo[2], Sxy = mo[3], Syy = mo[4], S0 = mo[5];
            const float A = -2.0f * kLn2 * q0.z, B = -kLn2 * q0.w, C = -2.0f * kLn2 * q1.x;
            float4* dst = reinterpret_cast<float4*>(partial + (size_t)kPart * jl);
            dst[0] = make_float4((-A * Sx - B * Sy) * hw, (-C * Sy - B * Sx) * hh, -0.5f * Sxx, -Sxy);
            dst[1] = make_float4(-0.5f * Syy, S0, mo[6], mo[7]);
            dst[2] = make_float4(mo[8], 0.f, 0.f, 0.f);
        }
        __syncthreads();
    }
}


// ---- mask-specialised bodies: every active stripe of a record in ONE basic block ----
struct FwdState {
    float T[kPPL], Tf[kPPL], C0[kPPL], C1[kPPL], C2[kPPL];
    uint32_t last[kPPL];
};

template <uint32_t M>
__device__ __forceinline__ void fwd_record(FwdState& st, const float (&pfy)[kPPL], float pfx, const float4 r0,
                                           const float4 r1, float rb, uint32_t idx) {
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        {
            if (!((M >> p) & 1u)) continue;
            const float dx = r0.x - pfx, dy = r0.y - pfy[p];
            const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
            float a = fminf(0.99f, r1.y * __builtin_amdgcn_exp2f(pw));
            a = pw <= 0.0f ? a : 0.0f;
            a = a >= (1.0f / 255.0f) ? a : 0.0f;
            const float tT = st.T[p] * (1.0f - a);
            const bool ok = tT >= 0.0001f;
            const float w = ok ? a * st.T[p] : 0.0f;
            st.C0[p] = fmaf(r1.z, w, st.C0[p]);
            st.C1[p] = fmaf(r1.w, w, st.C1[p]);
            st.C2[p] = fmaf(rb, w, st.C2[p]);
            const bool used = w > 0.0f;
            st.last[p] = used ? idx : st.last[p];
            st.Tf[p] = used ? tT : st.Tf[p];
            st.T[p] = a > 0.0f ? (ok ? tT : 0.0f) : st.T[p];
        }
    }
}

__device__ __forceinline__ void fwd_dispatch(uint32_t m, FwdState& st, const float (&pfy)[kPPL], float pfx,
                                             const float4 r0, const float4 r1, float rb, uint32_t idx) {
    switch (m) {
#define GSR_FWD_CASE(M) \
    case M: fwd_record<M>(st, pfy, pfx, r0, r1, rb, idx); break;
        GSR_FWD_CASE(1) GSR_FWD_CASE(2) GSR_FWD_CASE(3) GSR_FWD_CASE(4) GSR_FWD_CASE(5)
        GSR_FWD_CASE(6) GSR_FWD_CASE(7) GSR_FWD_CASE(8) GSR_FWD_CASE(9) GSR_FWD_CASE(10)
        GSR_FWD_CASE(11) GSR_FWD_CASE(12) GSR_FWD_CASE(13) GSR_FWD_CASE(14) GSR_FWD_CASE(15)
#undef GSR_FWD_CASE
        default: break;
    }
}

__global__ __launch_bounds__(64) void blend_forward_v4_kernel(const BlendGeom geo,
                                                              const uint2* __restrict__ ranges,
                                                              const uint32_t* __restrict__ sorted_gid,
                                                              const float4* __restrict__ rec,
                                                              float* __restrict__ out_color,
                                                              float* __restrict__ final_T,
                                                              uint32_t* __restrict__ n_contrib,
                                                              float* __restrict__ accum) {
    __shared__ float4 srec[64 * 3];
    const int tile = xcd_tile(blockIdx.x, geo.nwg) + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
    float pfy[kPPL];
    FwdState st;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        pfy[p] = (float)py;
        st.T[p] = (px < geo.W && py < geo.H) ? 1.0f : 0.0f;
        st.Tf[p] = 1.0f;
        st.C0[p] = st.C1[p] = st.C2[p] = 0.0f;
        st.last[p] = 0;
    }
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    for (int base = 0; base < n; base += 64) {
        uint32_t live = 0;
#pragma unroll
        for (int p = 0; p < kPPL; ++p) live |= __all(st.T[p] == 0.0f) ? 0u : (1u << p);
        if (live == 0) break;
        uint32_t smask = 0;
        if (base + lane < n) {
            const uint32_t g = sorted_gid[range.x + base + lane];
            const float4* r = rec + 3 * (size_t)g;
            const float4 r0 = r[0], r1 = r[1], r2 = r[2];
            srec[3 * lane + 0] = r0;
            srec[3 * lane + 1] = r1;
            srec[3 * lane + 2] = r2;
            smask = stripe_mask(r0, r2, bx0, by0);
        }
        __syncthreads();
        uint64_t todo = __ballot((smask & live) != 0u);
        int visited = 0;
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)smask, k) & live;
            const float4 r0 = srec[3 * k + 0];
            const float4 r1 = srec[3 * k + 1];
            const float rb = srec[3 * k + 2].x;
            fwd_dispatch(m, st, pfy, pfx, r0, r1, rb, (uint32_t)(base + k + 1));
            if ((++visited & 7) == 0) {
                uint32_t lv = 0;
#pragma unroll
                for (int p = 0; p < kPPL; ++p) lv |= __all(st.T[p] == 0.0f) ? 0u : (1u << p);
                live = lv;
                if (live == 0) break;
            }
        }
        __syncthreads();
    }
    const size_t npix = (size_t)geo.W * geo.H;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        if (px < geo.W && py < geo.H) {
            const size_t pix = (size_t)py * geo.W + px;
            final_T[pix] = st.Tf[p];
            n_contrib[pix] = st.last[p];
            accum[pix] = st.C0[p];
            accum[npix + pix] = st.C1[p];
            accum[2 * npix + pix] = st.C2[p];
            out_color[pix] = st.C0[p] + st.Tf[p] * geo.bg0;
            out_color[npix + pix] = st.C1[p] + st.Tf[p] * geo.bg1;
            out_color[2 * npix + pix] = st.C2[p] + st.Tf[p] * geo.bg2;
        }
    }
}

// ---- backward, mask-specialised ----
struct BwdState {
    float T[kPPL], Sp[kPPL], cb[kPPL], dp0[kPPL], dp1[kPPL], dp2[kPPL];
    uint32_t lastc[kPPL];
};

template <uint32_t M>
__device__ __forceinline__ bool bwd_record(BwdState& st, float (&v)[9], float pfx, float by0, int row,
                                           const float4 r0, const float4 r1, float rb, uint32_t e) {
    bool any = false;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        if (!((M >> p) & 1u)) continue;
        const float dx = r0.x - pfx, dy = r0.y - (by0 + (float)(row + 4 * p));
        const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
        const float G = __builtin_amdgcn_exp2f(pw);
        const float oG = r1.y * G;
        const float alpha = fminf(0.99f, oG);
        const bool valid = e < st.lastc[p] && pw <= 0.0f && alpha >= (1.0f / 255.0f);
        // predicated (no divergent branch): invalid pairs contribute exact zeros
        const float a = valid ? alpha : 0.0f;
        const float w = a * st.T[p];
        const float cdp = fmaf(r1.z, st.dp0[p], fmaf(r1.w, st.dp1[p], rb * st.dp2[p]));
        st.Sp[p] = fmaf(w, cdp, st.Sp[p]);
        const float one_m = 1.0f - a;
        const float dLda = fmaf(st.T[p], cdp, -(st.cb[p] - st.Sp[p]) * __builtin_amdgcn_rcpf(one_m));
        st.T[p] = st.T[p] * one_m;
        v[6] = fmaf(w, st.dp0[p], v[6]);
        v[7] = fmaf(w, st.dp1[p], v[7]);
        v[8] = fmaf(w, st.dp2[p], v[8]);
        const float Gv = valid ? G : 0.0f;
        v[5] = fmaf(Gv, dLda, v[5]);
        const float sv = r1.y * Gv * dLda;
        const float sx = sv * dx, sy = sv * dy;
        v[0] += sx;
        v[1] += sy;
        v[2] = fmaf(sx, dx, v[2]);
        v[3] = fmaf(sx, dy, v[3]);
        v[4] = fmaf(sy, dy, v[4]);
        any = any || valid;
    }
    return any;
}

__device__ __forceinline__ bool bwd_dispatch(uint32_t m, BwdState& st, float (&v)[9], float pfx, float by0,
                                             int row, const float4 r0, const float4 r1, float rb, uint32_t e) {
    switch (m) {
#define GSR_BWD_CASE(M) \
    case M: return bwd_record<M>(st, v, pfx, by0, row, r0, r1, rb, e);
        GSR_BWD_CASE(1) GSR_BWD_CASE(2) GSR_BWD_CASE(3) GSR_BWD_CASE(4) GSR_BWD_CASE(5)
        GSR_BWD_CASE(6) GSR_BWD_CASE(7) GSR_BWD_CASE(8) GSR_BWD_CASE(9) GSR_BWD_CASE(10)
        GSR_BWD_CASE(11) GSR_BWD_CASE(12) GSR_BWD_CASE(13) GSR_BWD_CASE(14) GSR_BWD_CASE(15)
#undef GSR_BWD_CASE
        default: return false;
    }
}

__global__ __launch_bounds__(64) void blend_backward_v4_kernel(const BlendGeom geo,
                                                               const uint2* __restrict__ ranges,
                                                               const uint32_t* __restrict__ sorted_gid,
                                                               const uint32_t* __restrict__ inst_start,
                                                               const uint2* __restrict__ rect,
                                                               const float4* __restrict__ rec,
                                                               const float* __restrict__ final_T,
                                                               const uint32_t* __restrict__ n_contrib,
                                                               const float* __restrict__ accum,
                                                               const float* __restrict__ dL_dpix,
                                                               float* __restrict__ partial) {
    __shared__ float4 srec[64 * 3];
    __shared__ float smom[64 * 12];
    const int tile = xcd_tile(blockIdx.x, geo.nwg) + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
    const size_t npix = (size_t)geo.W * geo.H;
    const float hw = 0.5f * (float)geo.W, hh = 0.5f * (float)geo.H;
    const int row = lane >> 4;
    BwdState st;
    uint32_t maxlast = 0;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + row + 4 * p;
        const bool in = px < geo.W && py < geo.H;
        const size_t pix = in ? (size_t)py * geo.W + px : 0;
        const float Tfin = in ? final_T[pix] : 1.0f;
        st.lastc[p] = in ? n_contrib[pix] : 0u;
        st.dp0[p] = in ? dL_dpix[pix] : 0.0f;
        st.dp1[p] = in ? dL_dpix[npix + pix] : 0.0f;
        st.dp2[p] = in ? dL_dpix[2 * npix + pix] : 0.0f;
        const float sdp = in ? accum[pix] * st.dp0[p] + accum[npix + pix] * st.dp1[p] +
                                   accum[2 * npix + pix] * st.dp2[p]
                             : 0.0f;
        st.cb[p] = sdp + Tfin * (geo.bg0 * st.dp0[p] + geo.bg1 * st.dp1[p] + geo.bg2 * st.dp2[p]);
        st.T[p] = 1.0f;
        st.Sp[p] = 0.0f;
        maxlast = maxlast > st.lastc[p] ? maxlast : st.lastc[p];
    }
    maxlast = wave_max_u32(maxlast);
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    for (int base = 0; base < n; base += 64) {
        const int cnt = (n - base) < 64 ? (n - base) : 64;
        const int e_l = base + lane;
        uint32_t jl = 0, smask = 0;
        float4 q0 = make_float4(0.f, 0.f, 0.f, 0.f), q1 = q0;
        if (lane < cnt) {
            const uint32_t g = sorted_gid[range.x + e_l];
            const uint2 rr = rect[g];
            const int minx = rr.x & 0xFFFF, miny = rr.x >> 16, maxx = rr.y & 0xFFFF;
            const int y0 = miny > geo.ty0 ? miny : geo.ty0;
            jl = inst_start[g] + (uint32_t)((ty - y0) * (maxx - minx) + (tx - minx));
            if (e_l < (int)maxlast) {
                const float4* r = rec + 3 * (size_t)g;
                q0 = r[0];
                q1 = r[1];
                const float4 r2 = r[2];
                srec[3 * lane + 0] = q0;
                srec[3 * lane + 1] = q1;
                srec[3 * lane + 2] = r2;
                smask = stripe_mask(q0, r2, bx0, by0);
            }
        }
#pragma unroll
        for (int c = 0; c < 12; ++c) smom[lane * 12 + c] = 0.0f;
        __syncthreads();
        uint64_t todo = __ballot(smask != 0u);
        while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)smask, k);
            const float4 r0 = srec[3 * k + 0];
            const float4 r1 = srec[3 * k + 1];
            const float rb = srec[3 * k + 2].x;
            float v[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            const bool any = bwd_dispatch(m, st, v, pfx, by0, row, r0, r1, rb, (uint32_t)(base + k));
            if (__any(any)) {
                row_reduce(v);
                const float t0 = scatter4(v[0], v[1], v[2], v[3]);
                const float t1 = scatter4(v[4], v[5], v[6], v[7]);
                const float t2 = allreduce_rows(v[8]);
                if ((lane & 15) == 0) {
                    smom[k * 12 + row] = t0;
                    smom[k * 12 + 4 + row] = t1;
                    if (row == 0) smom[k * 12 + 8] = t2;
                }
            }
        }
        __syncthreads();
        if (lane < cnt) {
            const float* mo = smom + lane * 12;
            const float Sx = mo[0], Sy = mo[1], Sxx = mo[2], Sxy = mo[3], Syy = mo[4], S0 = mo[5];
            const float A = -2.0f * kLn2 * q0.z, B = -kLn2 * q0.w, C = -2.0f * kLn2 * q1.x;
            float4* dst = reinterpret_cast<float4*>(partial + (size_t)kPart * jl);
            dst[0] = make_float4((-A * Sx - B * Sy) * hw, (-C * Sy - B * Sx) * hh, -0.5f * Sxx, -Sxy);
            dst[1] = make_float4(-0.5f * Syy, S0, mo[6], mo[7]);
            dst[2] = make_float4(mo[8], 0.f, 0.f, 0.f);
        }
        __syncthreads();
    }
}


// Forward with NW waves per 16x16 tile (PPL = 4/NW pixels per lane; wave w owns rows
// [w*16/NW, (w+1)*16/NW)).  The block stages 64*NW records per batch (one per thread) and
// their per-stripe masks in LDS; each wave sweeps the records touching its own stripes.
template <int NW>
__global__ __launch_bounds__(64 * NW) void blend_forward_nw_kernel(const BlendGeom geo,
                                                                   const uint2* __restrict__ ranges,
                                                                   const uint32_t* __restrict__ sorted_gid,
                                                                   const float4* __restrict__ rec,
                                                                   float* __restrict__ out_color,
                                                                   float* __restrict__ final_T,
                                                                   uint32_t* __restrict__ n_contrib,
                                                                   float* __restrict__ accum) {
    constexpr int PPL = kPPL / NW;
    constexpr int BATCH = 64 * NW;
    __shared__ float4 srec[BATCH * 3];
    __shared__ uint32_t smk[BATCH];
    const int tile = xcd_tile(blockIdx.x, geo.nwg) + geo.ty0 * geo.grid_x;
    const int tx = tile % geo.grid_x, ty = tile / geo.grid_x;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int px = tx * kTile + (lane & 15);
    const float pfx = (float)px;
    const float bx0 = (float)(tx * kTile), by0 = (float)(ty * kTile);
    // wave w owns global stripes [w*PPL, (w+1)*PPL)
    float pfy[PPL], T[PPL], Tf[PPL], C0[PPL], C1[PPL], C2[PPL];
    uint32_t last[PPL];
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * (w * PPL + p);
        pfy[p] = (float)py;
        T[p] = (px < geo.W && py < geo.H) ? 1.0f : 0.0f;
        Tf[p] = 1.0f;
        C0[p] = C1[p] = C2[p] = 0.0f;
        last[p] = 0;
    }
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    for (int base = 0; base < n; base += BATCH) {
        uint32_t live = 0;
#pragma unroll
        for (int p = 0; p < PPL; ++p) live |= __all(T[p] == 0.0f) ? 0u : (1u << p);
        if (__syncthreads_or(live != 0) == 0) break;
        if (base + tid < n) {
            const uint32_t g = sorted_gid[range.x + base + tid];
            const float4* r = rec + 3 * (size_t)g;
            const float4 r0 = r[0], r1 = r[1], r2 = r[2];
            srec[3 * tid + 0] = r0;
            srec[3 * tid + 1] = r1;
            srec[3 * tid + 2] = r2;
            smk[tid] = stripe_mask(r0, r2, bx0, by0);
        } else {
            smk[tid] = 0u;
        }
        __syncthreads();
        const int cnt = (n - base) < BATCH ? (n - base) : BATCH;
        int visited = 0;
        for (int c0 = 0; c0 < cnt && live; c0 += 64) {
            const uint32_t mine = (smk[c0 + lane] >> (w * PPL)) & ((1u << PPL) - 1u);
            uint64_t todo = __ballot((mine & live) != 0u && c0 + lane < cnt);
            while (todo) {
                const int kk = __builtin_ctzll(todo);
                todo &= todo - 1;
                const int k = c0 + kk;
                const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)mine, kk) & live;
                const float4 r0 = srec[3 * k + 0];
                const float4 r1 = srec[3 * k + 1];
                const float rb = srec[3 * k + 2].x;
                const uint32_t idx = (uint32_t)(base + k + 1);
#pragma unroll
                for (int p = 0; p < PPL; ++p) {
                    if (!(m & (1u << p))) continue;  // wave-uniform
                    const float dx = r0.x - pfx, dy = r0.y - pfy[p];
                    const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
                    float a = fminf(0.99f, r1.y * __builtin_amdgcn_exp2f(pw));
                    a = pw <= 0.0f ? a : 0.0f;
                    a = a >= (1.0f / 255.0f) ? a : 0.0f;
                    const float tT = T[p] * (1.0f - a);
                    const bool ok = tT >= 0.0001f;
                    const float wgt = ok ? a * T[p] : 0.0f;
                    C0[p] = fmaf(r1.z, wgt, C0[p]);
                    C1[p] = fmaf(r1.w, wgt, C1[p]);
                    C2[p] = fmaf(rb, wgt, C2[p]);
                    const bool used = wgt > 0.0f;
                    last[p] = used ? idx : last[p];
                    Tf[p] = used ? tT : Tf[p];
                    T[p] = a > 0.0f ? (ok ? tT : 0.0f) : T[p];
                }
                if ((++visited & 7) == 0) {
                    uint32_t lv = 0;
#pragma unroll
                    for (int p = 0; p < PPL; ++p) lv |= __all(T[p] == 0.0f) ? 0u : (1u << p);
                    live = lv;
                    if (live == 0) break;
                }
            }
        }
        __syncthreads();
    }
    const size_t npix = (size_t)geo.W * geo.H;
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * (w * PPL + p);
        if (px < geo.W && py < geo.H) {
            const size_t pix = (size_t)py * geo.W + px;
            final_T[pix] = Tf[p];
            n_contrib[pix] = last[p];
            accum[pix] = C0[p];
            accum[npix + pix] = C1[p];
            accum[2 * npix + pix] = C2[p];
            out_color[pix] = C0[p] + Tf[p] * geo.bg0;
            out_color[npix + pix] = C1[p] + Tf[p] * geo.bg1;
            out_color[2 * npix + pix] = C2[p] + Tf[p] * geo.bg2;
        }
    }
}

}  // namespace

// Kernel-variant selector for A/B timing (bench/ablation only; default = shipped variant).
static int variant(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
}

static BlendGeom make_geo(const gsr_camera& cam, const float bg[3], int ty0, int ty1) {
    BlendGeom g;
    g.W = cam.width;
    g.H = cam.height;
    g.grid_x = div_up(cam.width, kTile);
    g.ty0 = ty0;
    g.nwg = (ty1 - ty0) * g.grid_x;
    g.bg0 = bg[0];
    g.bg1 = bg[1];
    g.bg2 = bg[2];
    return g;
}

int launch_blend_forward(const gsr_camera& cam, const float bg[3], int ty0, int ty1,
                         const uint2* ranges, const uint32_t* sorted_gid, const float4* rec,
                         float* out_color, float* final_T, uint32_t* n_contrib, float* accum,
                         hipStream_t s) {
    const BlendGeom geo = make_geo(cam, bg, ty0, ty1);
    if (geo.nwg <= 0) return 0;
    const int v = variant("GSR_FWD_VARIANT", 5);
    if (v == 5)
        hipLaunchKernelGGL(blend_forward_nw_kernel<2>, dim3(geo.nwg), dim3(128), 0, s, geo, ranges, sorted_gid,
                           rec, out_color, final_T, n_contrib, accum);
    else if (v == 6)
        hipLaunchKernelGGL(blend_forward_nw_kernel<4>, dim3(geo.nwg), dim3(256), 0, s, geo, ranges, sorted_gid,
                           rec, out_color, final_T, n_contrib, accum);
    else if (v == 7)
        hipLaunchKernelGGL(blend_forward_nw_kernel<1>, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid,
                           rec, out_color, final_T, n_contrib, accum);
    else if (v == 4)
        hipLaunchKernelGGL(blend_forward_v4_kernel, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid, rec,
                           out_color, final_T, n_contrib, accum);
    else if (v == 3)
        hipLaunchKernelGGL(blend_forward_v3_kernel, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid, rec,
                           out_color, final_T, n_contrib, accum);
    else if (v == 2)
        hipLaunchKernelGGL(blend_forward_v2_kernel, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid, rec,
                           out_color, final_T, n_contrib, accum);
    else if (v == 1)
        hipLaunchKernelGGL(blend_forward_kernel<false>, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid,
                           rec, out_color, final_T, n_contrib, accum);
    else
        hipLaunchKernelGGL(blend_forward_kernel<true>, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid,
                           rec, out_color, final_T, n_contrib, accum);
    return (int)hipGetLastError();
}

int launch_blend_backward(const gsr_camera& cam, const float bg[3], int ty0, int ty1,
                          const uint2* ranges, const uint32_t* sorted_gid, const uint32_t* inst_start,
                          const uint2* rect, const float4* rec, const float* final_T,
                          const uint32_t* n_contrib, const float* accum, const float* dL_dpix,
                          float* partial, hipStream_t s) {
    const BlendGeom geo = make_geo(cam, bg, ty0, ty1);
    if (geo.nwg <= 0) return 0;
    const int v = variant("GSR_BWD_VARIANT", 2);
    if (v == 4)
        hipLaunchKernelGGL(blend_backward_v4_kernel, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid,
                           inst_start, rect, rec, final_T, n_contrib, accum, dL_dpix, partial);
    else if (v == 3)
        hipLaunchKernelGGL(blend_backward_f2b_pf_kernel<true>, dim3(geo.nwg), dim3(64), 0, s, geo, ranges,
                           sorted_gid, inst_start, rect, rec, final_T, n_contrib, accum, dL_dpix, partial);
    else if (v == 2)
        hipLaunchKernelGGL(blend_backward_f2b_kernel<true>, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid,
                           inst_start, rect, rec, final_T, n_contrib, accum, dL_dpix, partial);
    else if (v == 1)
        hipLaunchKernelGGL(blend_backward_kernel<false>, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid,
                           inst_start, rect, rec, final_T, n_contrib, dL_dpix, partial);
    else
        hipLaunchKernelGGL(blend_backward_kernel<true>, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid,
                           inst_start, rect, rec, final_T, n_contrib, dL_dpix, partial);
    return (int)hipGetLastError();
}

}  // namespace gsr

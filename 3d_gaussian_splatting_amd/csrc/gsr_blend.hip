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

template <int CTRL, int ROW_MASK = 0xF>
__device__ inline float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROW_MASK, 0xF, false));
}

// sum over the 64 lanes (every lane must be active); result is wave-uniform
__device__ inline float wave_sum(float x) {
    x += dpp_f<0xB1>(x);         // quad_perm [1,0,3,2]
    x += dpp_f<0x4E>(x);         // quad_perm [2,3,0,1]
    x += dpp_f<0x141>(x);        // row_half_mirror
    x += dpp_f<0x140>(x);        // row_mirror
    x += dpp_f<0x142, 0xA>(x);   // row_bcast:15
    x += dpp_f<0x143, 0xC>(x);   // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
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

__global__ __launch_bounds__(64) void blend_forward_kernel(const BlendGeom geo,
                                                           const uint2* __restrict__ ranges,
                                                           const uint32_t* __restrict__ sorted_gid,
                                                           const float4* __restrict__ rec,
                                                           float* __restrict__ out_color,
                                                           float* __restrict__ final_T,
                                                           uint32_t* __restrict__ n_contrib) {
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
                if (!(m & (1u << p))) continue;  // wave-uniform
                const float dx = r0.x - pfx, dy = r0.y - pfy[p];
                const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
                const float alpha = fminf(0.99f, r1.y * __builtin_amdgcn_exp2f(pw));
                const bool valid = !done[p] && pw <= 0.0f && alpha >= (1.0f / 255.0f);
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
            out_color[pix] = C0[p] + T[p] * geo.bg0;
            out_color[npix + pix] = C1[p] + T[p] * geo.bg1;
            out_color[2 * npix + pix] = C2[p] + T[p] * geo.bg2;
        }
    }
}

__global__ __launch_bounds__(64) void blend_backward_kernel(const BlendGeom geo,
                                                            const uint2* __restrict__ ranges,
                                                            const uint32_t* __restrict__ sorted_gid,
                                                            const uint32_t* __restrict__ sorted_j,
                                                            const float4* __restrict__ rec,
                                                            const float* __restrict__ final_T,
                                                            const uint32_t* __restrict__ n_contrib,
                                                            const float* __restrict__ dL_dpix,
                                                            float* __restrict__ partial) {
    __shared__ float4 srec[64 * 3];
    __shared__ float4 sout[64 * 3];
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
    for (int top = n; top > 0; top -= 64) {
        const int lo = top > 64 ? top - 64 : 0;
        const int cnt = top - lo;
        const int e_l = top - 1 - lane;  // this lane's entry (descending)
        uint32_t jl = 0, smask = 0;
        if (lane < cnt) {
            jl = sorted_j[range.x + e_l];
            if (e_l < (int)maxlast) {
                const uint32_t g = sorted_gid[range.x + e_l];
                const float4* r = rec + 3 * (size_t)g;
                const float4 r0 = r[0], r1 = r[1], r2 = r[2];
                srec[3 * lane + 0] = r0;
                srec[3 * lane + 1] = r1;
                srec[3 * lane + 2] = r2;
                smask = stripe_mask(r0, r2, bx0, by0);
            }
        }
        sout[3 * lane + 0] = make_float4(0.f, 0.f, 0.f, 0.f);
        sout[3 * lane + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
        sout[3 * lane + 2] = make_float4(0.f, 0.f, 0.f, 0.f);
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
            // moments of s = G * o * dL/dalpha over the tile's pixels
            float Sx = 0.f, Sy = 0.f, Sxx = 0.f, Sxy = 0.f, Syy = 0.f, S0 = 0.f, gr = 0.f, gg = 0.f, gb = 0.f;
            bool any = false;
#pragma unroll
            for (int p = 0; p < kPPL; ++p) {
                if (!(m & (1u << p))) continue;  // wave-uniform
                const float dx = r0.x - pfx, dy = r0.y - (by0 + (float)((lane >> 4) + 4 * p));
                const float pw = fmaf(r0.z * dx, dx, fmaf(r0.w * dx, dy, r1.x * dy * dy));
                const float G = __builtin_amdgcn_exp2f(pw);
                const float alpha = fminf(0.99f, r1.y * G);
                const bool valid = e < lastc[p] && pw <= 0.0f && alpha >= (1.0f / 255.0f);
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
                    gr = fmaf(dch, dp0[p], gr);
                    gg = fmaf(dch, dp1[p], gg);
                    gb = fmaf(dch, dp2[p], gb);
                    dLda = fmaf(dLda, T[p], cbg[p] * inv);
                    const float GdL = G * dLda;
                    S0 += GdL;
                    const float s = r1.y * GdL;
                    const float sx = s * dx, sy = s * dy;
                    Sx += sx;
                    Sy += sy;
                    Sxx = fmaf(sx, dx, Sxx);
                    Sxy = fmaf(sx, dy, Sxy);
                    Syy = fmaf(sy, dy, Syy);
                }
            }
            if (__any(any)) {
                Sx = wave_sum(Sx);
                Sy = wave_sum(Sy);
                Sxx = wave_sum(Sxx);
                Sxy = wave_sum(Sxy);
                Syy = wave_sum(Syy);
                S0 = wave_sum(S0);
                gr = wave_sum(gr);
                gg = wave_sum(gg);
                gb = wave_sum(gb);
                if (lane == 0) {
                    const float A = -2.0f * kLn2 * r0.z, B = -kLn2 * r0.w, C = -2.0f * kLn2 * r1.x;
                    sout[3 * k + 0] = make_float4((-A * Sx - B * Sy) * hw, (-C * Sy - B * Sx) * hh, -0.5f * Sxx, -Sxy);
                    sout[3 * k + 1] = make_float4(-0.5f * Syy, S0, gr, gg);
                    sout[3 * k + 2] = make_float4(gb, 0.f, 0.f, 0.f);
                }
            }
        }
        __syncthreads();
        if (lane < cnt) {
            float4* dst = reinterpret_cast<float4*>(partial + (size_t)kPart * jl);
            dst[0] = sout[3 * lane + 0];
            dst[1] = sout[3 * lane + 1];
            dst[2] = sout[3 * lane + 2];
        }
        __syncthreads();
    }
}

}  // namespace

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
                         float* out_color, float* final_T, uint32_t* n_contrib, hipStream_t s) {
    const BlendGeom geo = make_geo(cam, bg, ty0, ty1);
    if (geo.nwg <= 0) return 0;
    hipLaunchKernelGGL(blend_forward_kernel, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid, rec,
                       out_color, final_T, n_contrib);
    return (int)hipGetLastError();
}

int launch_blend_backward(const gsr_camera& cam, const float bg[3], int ty0, int ty1,
                          const uint2* ranges, const uint32_t* sorted_gid, const uint32_t* sorted_j,
                          const float4* rec, const float* final_T, const uint32_t* n_contrib,
                          const float* dL_dpix, float* partial, hipStream_t s) {
    const BlendGeom geo = make_geo(cam, bg, ty0, ty1);
    if (geo.nwg <= 0) return 0;
    hipLaunchKernelGGL(blend_backward_kernel, dim3(geo.nwg), dim3(64), 0, s, geo, ranges, sorted_gid,
                       sorted_j, rec, final_T, n_contrib, dL_dpix, partial);
    return (int)hipGetLastError();
}

}  // namespace gsr

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
        bool alldone = true;
#pragma unroll
        for (int p = 0; p < kPPL; ++p) alldone &= done[p];
        if (__all(alldone)) break;
        if (base + lane < n) {
            const uint32_t g = sorted_gid[range.x + base + lane];
            const float4* r = rec + 3 * (size_t)g;
            srec[3 * lane + 0] = r[0];
            srec[3 * lane + 1] = r[1];
            srec[3 * lane + 2] = r[2];
        }
        __syncthreads();
        const int cnt = (n - base) < 64 ? (n - base) : 64;
        for (int k = 0; k < cnt; ++k) {
            const float4 r0 = srec[3 * k + 0];  // x, y, A, B
            const float4 r1 = srec[3 * k + 1];  // C, opacity, r, g
            const float4 r2 = srec[3 * k + 2];  // b, depth, rect
#pragma unroll
            for (int p = 0; p < kPPL; ++p) {
                if (done[p]) continue;
                const float dx = r0.x - pfx, dy = r0.y - pfy[p];
                const float power = -0.5f * (r0.z * dx * dx + r1.x * dy * dy) - r0.w * dx * dy;
                if (power > 0.0f) continue;
                const float alpha = fminf(0.99f, r1.y * __expf(power));
                if (alpha < 1.0f / 255.0f) continue;
                const float test_T = T[p] * (1.0f - alpha);
                if (test_T < 0.0001f) {
                    done[p] = true;
                    continue;
                }
                const float w = alpha * T[p];
                C0[p] += r1.z * w;
                C1[p] += r1.w * w;
                C2[p] += r2.x * w;
                T[p] = test_T;
                last[p] = (uint32_t)(base + k + 1);
            }
            if ((k & 7) == 7) {
                bool ad = true;
#pragma unroll
                for (int p = 0; p < kPPL; ++p) ad &= done[p];
                if (__all(ad)) break;
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
    const size_t npix = (size_t)geo.W * geo.H;
    const float ddelx_dx = 0.5f * (float)geo.W, ddely_dy = 0.5f * (float)geo.H;
    float pfy[kPPL], T[kPPL], Tf[kPPL], dp0[kPPL], dp1[kPPL], dp2[kPPL], bgd[kPPL];
    float ac0[kPPL], ac1[kPPL], ac2[kPPL], lc0[kPPL], lc1[kPPL], lc2[kPPL], la[kPPL];
    uint32_t lastc[kPPL];
    uint32_t maxlast = 0;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const int py = ty * kTile + (lane >> 4) + 4 * p;
        pfy[p] = (float)py;
        const bool in = px < geo.W && py < geo.H;
        const size_t pix = in ? (size_t)py * geo.W + px : 0;
        Tf[p] = in ? final_T[pix] : 1.0f;
        T[p] = Tf[p];
        lastc[p] = in ? n_contrib[pix] : 0u;
        dp0[p] = in ? dL_dpix[pix] : 0.0f;
        dp1[p] = in ? dL_dpix[npix + pix] : 0.0f;
        dp2[p] = in ? dL_dpix[2 * npix + pix] : 0.0f;
        bgd[p] = geo.bg0 * dp0[p] + geo.bg1 * dp1[p] + geo.bg2 * dp2[p];
        ac0[p] = ac1[p] = ac2[p] = lc0[p] = lc1[p] = lc2[p] = la[p] = 0.0f;
        maxlast = maxlast > lastc[p] ? maxlast : lastc[p];
    }
    maxlast = wave_max_u32(maxlast);
    const uint2 range = ranges[tile];
    const int n = (int)(range.y - range.x);
    for (int top = n; top > 0; top -= 64) {
        const int lo = top > 64 ? top - 64 : 0;
        const int cnt = top - lo;
        const int e_l = top - 1 - lane;  // entry of this lane's batch slot (descending)
        uint32_t jl = 0;
        if (lane < cnt) {
            jl = sorted_j[range.x + e_l];
            if (e_l < (int)maxlast) {
                const uint32_t g = sorted_gid[range.x + e_l];
                const float4* r = rec + 3 * (size_t)g;
                srec[3 * lane + 0] = r[0];
                srec[3 * lane + 1] = r[1];
                srec[3 * lane + 2] = r[2];
            }
        }
        sout[3 * lane + 0] = make_float4(0.f, 0.f, 0.f, 0.f);
        sout[3 * lane + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
        sout[3 * lane + 2] = make_float4(0.f, 0.f, 0.f, 0.f);
        __syncthreads();
        if (lo < (int)maxlast) {
            const int kstart = top > (int)maxlast ? top - (int)maxlast : 0;
            for (int k = kstart; k < cnt; ++k) {
                const uint32_t e = (uint32_t)(top - 1 - k);
                const float4 r0 = srec[3 * k + 0];
                const float4 r1 = srec[3 * k + 1];
                const float4 r2 = srec[3 * k + 2];
                float gmx = 0.f, gmy = 0.f, gA = 0.f, gB = 0.f, gC = 0.f, go = 0.f, gr = 0.f, gg = 0.f,
                      gb = 0.f;
                bool any = false;
#pragma unroll
                for (int p = 0; p < kPPL; ++p) {
                    if (e >= lastc[p]) continue;
                    const float dx = r0.x - pfx, dy = r0.y - pfy[p];
                    const float power = -0.5f * (r0.z * dx * dx + r1.x * dy * dy) - r0.w * dx * dy;
                    if (power > 0.0f) continue;
                    const float G = __expf(power);
                    const float alpha = fminf(0.99f, r1.y * G);
                    if (alpha < 1.0f / 255.0f) continue;
                    any = true;
                    const float one_m = 1.0f - alpha;
                    T[p] = T[p] / one_m;
                    const float dchannel = alpha * T[p];
                    ac0[p] = la[p] * lc0[p] + (1.0f - la[p]) * ac0[p];
                    ac1[p] = la[p] * lc1[p] + (1.0f - la[p]) * ac1[p];
                    ac2[p] = la[p] * lc2[p] + (1.0f - la[p]) * ac2[p];
                    lc0[p] = r1.z;
                    lc1[p] = r1.w;
                    lc2[p] = r2.x;
                    float dL_dalpha = (r1.z - ac0[p]) * dp0[p] + (r1.w - ac1[p]) * dp1[p] + (r2.x - ac2[p]) * dp2[p];
                    gr += dchannel * dp0[p];
                    gg += dchannel * dp1[p];
                    gb += dchannel * dp2[p];
                    dL_dalpha *= T[p];
                    la[p] = alpha;
                    dL_dalpha += (-Tf[p] / one_m) * bgd[p];
                    const float dL_dG = r1.y * dL_dalpha;
                    const float gdx = G * dx, gdy = G * dy;
                    gmx += dL_dG * (-gdx * r0.z - gdy * r0.w) * ddelx_dx;
                    gmy += dL_dG * (-gdy * r1.x - gdx * r0.w) * ddely_dy;
                    gA += -0.5f * gdx * dx * dL_dG;
                    gB += -gdx * dy * dL_dG;
                    gC += -0.5f * gdy * dy * dL_dG;
                    go += G * dL_dalpha;
                }
                if (__any(any)) {
                    gmx = wave_sum(gmx);
                    gmy = wave_sum(gmy);
                    gA = wave_sum(gA);
                    gB = wave_sum(gB);
                    gC = wave_sum(gC);
                    go = wave_sum(go);
                    gr = wave_sum(gr);
                    gg = wave_sum(gg);
                    gb = wave_sum(gb);
                    if (lane == 0) {
                        sout[3 * k + 0] = make_float4(gmx, gmy, gA, gB);
                        sout[3 * k + 1] = make_float4(gC, go, gr, gg);
                        sout[3 * k + 2] = make_float4(gb, 0.f, 0.f, 0.f);
                    }
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

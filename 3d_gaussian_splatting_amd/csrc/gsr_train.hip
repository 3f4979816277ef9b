// gsr_train.hip -- training-step kernels around the rasterizer (include/gsr/gsr_train.h,
// SURVEY.md §8f rows 1-2) on gfx950.
//
//  * activate_kernel      exp / normalize / sigmoid of the raw leaves (the reference's getters,
//                         src/scene/gaussian_model.cpp:270-298), one thread per Gaussian.
//  * ssim_forward_kernel  L1 + SSIM terms of one 64 x 16 output tile per block: the raw tile
//                         plus a 5-pixel halo is staged in LDS, blurred horizontally (5 moment
//                         maps) into LDS and vertically in registers (each pass slides the
//                         11-tap window over 4 outputs per thread); writes the three SSIM
//                         derivative maps the backward blurs, and one (sum S, sum |x - y|)
//                         partial per block (fixed-order sums, no atomics).
//  * ssim_backward_kernel the adjoint: blur of the three maps (same separable window) combined
//                         with x and y, plus the L1 sign term -> dL/dimg.
//  * adam_kernel          one launch for all six parameter groups (multi-tensor): activation
//                         backward, moments, bias-corrected update; float4 per thread.
//  * densify_stats_kernel max_radii2D / grad accumulation / denom for radii > 0.
//  * compact_* + gather_rows_kernel  mask -> ascending index list (wave64 ballot counts,
//                         block-local scan) and a multi-tensor row gather (prune / clone).
//
// All of these are HBM-bound streams (DESIGN.md §11 gives bytes per element); none is
// GEMM-shaped, so nothing here goes near MFMA.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstring>

#include "../../include/gsr/gsr_train.h"

namespace gsr {
// defined in gsr_api.cpp: sets the thread-local error text read by gsr_last_error()
int set_error(int code, const char* msg);
}  // namespace gsr

namespace gsr {
namespace {

// ---------------------------------------------------------------- activations
__global__ __launch_bounds__(256) void activate_kernel(const float* __restrict__ s_raw, const float4* __restrict__ q_raw,
                                                       const float* __restrict__ o_raw, int P, float* __restrict__ s,
                                                       float4* __restrict__ q, float* __restrict__ o) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= P) return;
    if (s) {
#pragma unroll
        for (int k = 0; k < 3; ++k) s[3 * g + k] = expf(s_raw[3 * g + k]);
    }
    if (q) {
        const float4 r = q_raw[g];
        const float n = fmaxf(sqrtf(r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w), 1e-12f);
        q[g] = make_float4(r.x / n, r.y / n, r.z / n, r.w / n);
    }
    if (o) o[g] = 1.0f / (1.0f + expf(-o_raw[g]));
}

// ---------------------------------------------------------------- SSIM + L1
constexpr int kWin = 11, kRad = 5;
constexpr int kTX = 64, kTY = 16;                              // output tile
constexpr int kRX = kTX + 2 * kRad, kRY = kTY + 2 * kRad;      // 74 x 26 staged tile
constexpr int kRXP = kRX + 1;                                  // LDS row pitch
constexpr float kC1 = 0.01f * 0.01f, kC2 = 0.03f * 0.03f;

struct Window {
    float w[kWin];
};

__device__ __forceinline__ void block_sum2(float& a, float& b, float* red) {
    // fixed-order block reduction of two values (256 threads)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[2 * wv] = a;
        red[2 * wv + 1] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = (red[0] + red[2]) + (red[4] + red[6]);
        b = (red[1] + red[3]) + (red[5] + red[7]);
    }
}

// maps: A | B | Cm planes of C*H*W floats, scaled by g = -lambda / (C H W) (dL/dS per pixel):
//   A = g dS/dmu_x, B = g dS/dE[x^2], Cm = g dS/dE[xy]
__global__ __launch_bounds__(256) void ssim_forward_kernel(const float* __restrict__ img, const float* __restrict__ gt,
                                                           int H, int W, const Window win, float gscale,
                                                           float* __restrict__ maps, float2* __restrict__ part) {
    __shared__ float sx[kRY * kRXP], sy[kRY * kRXP];
    __shared__ float hs[5][kRY * kTX];
    __shared__ float red[8];
    const int c = blockIdx.z, x0 = blockIdx.x * kTX, y0 = blockIdx.y * kTY, tid = threadIdx.x;
    const size_t plane = (size_t)H * W;
    const float* X = img + c * plane;
    const float* Y = gt + c * plane;
    for (int i = tid; i < kRY * kRX; i += 256) {
        const int r = i / kRX, cc = i - r * kRX;
        const int gy = y0 - kRad + r, gx = x0 - kRad + cc;
        const bool in = gx >= 0 && gx < W && gy >= 0 && gy < H;
        const size_t o = in ? (size_t)gy * W + gx : 0;
        sx[r * kRXP + cc] = in ? X[o] : 0.0f;
        sy[r * kRXP + cc] = in ? Y[o] : 0.0f;
    }
    __syncthreads();
    // horizontal pass: a thread slides the window over 4 adjacent columns of one row (14 LDS reads
    // of x and y for 4 outputs instead of 44); each output still sums its taps in k order
    for (int i = tid; i < kRY * (kTX / 4); i += 256) {
        const int r = i / (kTX / 4), c0 = 4 * (i - r * (kTX / 4));
        float m[4][5];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 5; ++q) m[j][q] = 0.f;
#pragma unroll
        for (int t = 0; t < kWin + 3; ++t) {
            const float a = sx[r * kRXP + c0 + t], b = sy[r * kRXP + c0 + t];
            const float aa = a * a, bb = b * b, ab = a * b;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = t - j;
                if (k < 0 || k >= kWin) continue;
                const float w = win.w[k];
                m[j][0] = fmaf(w, a, m[j][0]);
                m[j][1] = fmaf(w, b, m[j][1]);
                m[j][2] = fmaf(w, aa, m[j][2]);
                m[j][3] = fmaf(w, bb, m[j][3]);
                m[j][4] = fmaf(w, ab, m[j][4]);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 5; ++q) hs[q][r * kTX + c0 + j] = m[j][q];
    }
    __syncthreads();
    float ssum = 0.f, l1sum = 0.f;
    const size_t all = (size_t)gridDim.z * plane;
    float* A = maps;
    float* B = maps + all;
    float* Cm = maps + 2 * all;
    // vertical pass: thread (column cc, row group rg) slides over rows 4 rg .. 4 rg + 3 (14 LDS
    // reads per moment for 4 outputs instead of 44), taps summed in k order as before
    const int cc = tid & (kTX - 1), r0 = 4 * (tid >> 6);
    float mv[4][5];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 5; ++q) mv[j][q] = 0.f;
#pragma unroll
    for (int t = 0; t < kWin + 3; ++t) {
        float h[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) h[q] = hs[q][(r0 + t) * kTX + cc];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = t - j;
            if (k < 0 || k >= kWin) continue;
            const float w = win.w[k];
#pragma unroll
            for (int q = 0; q < 5; ++q) mv[j][q] = fmaf(w, h[q], mv[j][q]);
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int r = r0 + j;
        const int gx = x0 + cc, gy = y0 + r;
        const float* m = mv[j];
        if (gx >= W || gy >= H) continue;
        const float mu1 = m[0], mu2 = m[1];
        const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu12 = mu1 * mu2;
        const float s1 = m[2] - mu1_sq, s2 = m[3] - mu2_sq, s12 = m[4] - mu12;
        const float N1 = 2.0f * mu12 + kC1, N2 = 2.0f * s12 + kC2;
        const float D1 = mu1_sq + mu2_sq + kC1, D2 = s1 + s2 + kC2;
        const float den = D1 * D2;
        const float S = (N1 * N2) / den;
        const float iD1 = 1.0f / D1, iD2 = 1.0f / D2;
        const float dmu = 2.0f * mu2 * (N2 - N1) / den - 2.0f * mu1 * S * (iD1 - iD2);
        const float dxx = -S * iD2;
        const float dxy = 2.0f * N1 / den;
        const size_t o = c * plane + (size_t)gy * W + gx;
        A[o] = gscale * dmu;
        B[o] = gscale * dxx;
        Cm[o] = gscale * dxy;
        ssum += S;
        l1sum += fabsf(sx[(r + kRad) * kRXP + cc + kRad] - sy[(r + kRad) * kRXP + cc + kRad]);
    }
    block_sum2(ssum, l1sum, red);
    if (tid == 0) part[(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = make_float2(ssum, l1sum);
}

__global__ __launch_bounds__(256) void loss_finalize_kernel(const float2* __restrict__ part, int nparts, double inv_n,
                                                            float lambda, float* __restrict__ stats) {
    __shared__ double rs[256], rl[256];
    double s = 0.0, l = 0.0;
    for (int i = threadIdx.x; i < nparts; i += 256) {
        const float2 p = part[i];
        s += (double)p.x;
        l += (double)p.y;
    }
    rs[threadIdx.x] = s;
    rl[threadIdx.x] = l;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            rs[threadIdx.x] += rs[threadIdx.x + o];
            rl[threadIdx.x] += rl[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float ssim = (float)(rs[0] * inv_n), l1 = (float)(rl[0] * inv_n);
        stats[0] = (1.0f - lambda) * l1 + lambda * (1.0f - ssim);
        stats[1] = l1;
        stats[2] = ssim;
    }
}

__global__ __launch_bounds__(256) void ssim_backward_kernel(const float* __restrict__ img, const float* __restrict__ gt,
                                                            int H, int W, const Window win, float l1scale,
                                                            const float* __restrict__ maps, float* __restrict__ dimg) {
    __shared__ float sm[3][kRY * kRXP];
    __shared__ float hs[3][kRY * kTX];
    const int c = blockIdx.z, x0 = blockIdx.x * kTX, y0 = blockIdx.y * kTY, tid = threadIdx.x;
    const size_t plane = (size_t)H * W, all = (size_t)gridDim.z * plane;
    for (int i = tid; i < kRY * kRX; i += 256) {
        const int r = i / kRX, cc = i - r * kRX;
        const int gy = y0 - kRad + r, gx = x0 - kRad + cc;
        const bool in = gx >= 0 && gx < W && gy >= 0 && gy < H;
        const size_t o = c * plane + (in ? (size_t)gy * W + gx : 0);
#pragma unroll
        for (int q = 0; q < 3; ++q) sm[q][r * kRXP + cc] = in ? maps[q * all + o] : 0.0f;
    }
    __syncthreads();
    for (int i = tid; i < kRY * (kTX / 4); i += 256) {  // horizontal, 4 columns per thread
        const int r = i / (kTX / 4), c0 = 4 * (i - r * (kTX / 4));
        float m[4][3];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) m[j][q] = 0.f;
#pragma unroll
        for (int t = 0; t < kWin + 3; ++t) {
            float v[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) v[q] = sm[q][r * kRXP + c0 + t];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = t - j;
                if (k < 0 || k >= kWin) continue;
                const float w = win.w[k];
#pragma unroll
                for (int q = 0; q < 3; ++q) m[j][q] = fmaf(w, v[q], m[j][q]);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) hs[q][r * kTX + c0 + j] = m[j][q];
    }
    __syncthreads();
    const int cc = tid & (kTX - 1), r0 = 4 * (tid >> 6);  // vertical, 4 rows per thread
    float mv[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) mv[j][q] = 0.f;
#pragma unroll
    for (int t = 0; t < kWin + 3; ++t) {
        float h[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) h[q] = hs[q][(r0 + t) * kTX + cc];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = t - j;
            if (k < 0 || k >= kWin) continue;
            const float w = win.w[k];
#pragma unroll
            for (int q = 0; q < 3; ++q) mv[j][q] = fmaf(w, h[q], mv[j][q]);
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int gx = x0 + cc, gy = y0 + r0 + j;
        if (gx >= W || gy >= H) continue;
        const size_t o = c * plane + (size_t)gy * W + gx;
        const float x = img[o], y = gt[o];
        const float d = x - y;
        const float sgn = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
        dimg[o] = fmaf(l1scale, sgn, mv[j][0] + 2.0f * x * mv[j][1] + y * mv[j][2]);
    }
}

// ---------------------------------------------------------------- Adam
struct AdamArgs {
    gsr_adam_group g[GSR_ADAM_MAX_GROUPS];
    int blk_start[GSR_ADAM_MAX_GROUPS + 1];
    float step_size[GSR_ADAM_MAX_GROUPS];  // lr / (1 - beta1^step)
    float bc2_sqrt[GSR_ADAM_MAX_GROUPS];   // sqrt(1 - beta2^step)
    int ngroups;
    float b1, b2, eps, omb1, omb2;          // omb = 1 - beta (rounded once, as libtorch's alpha)
    const uint32_t* guard_k;                // skip the whole step when *guard_k > guard_cap
    uint32_t guard_cap;
};

// The device-side step guard: a render under a binning bound whose true instance count K (the
// scan's device counter) exceeded the bound was truncated; the optimizer step / statistics of
// that iteration are then dropped here, on the device, with no host wait (the host learns of
// the overflow one iteration later from its pinned copy and re-sizes).
__device__ __forceinline__ bool guard_tripped(const uint32_t* k, uint32_t cap) {
    return k != nullptr && *k > cap;  // written by an earlier kernel of the stream
}
// Streaming (non-temporal) loads / stores: parameters, gradients and moments are touched once per
// step, so they should not displace the L2 / MALL lines the rasterizer reuses.  Measured in the
// configs[4] loop (6M Gaussians, 1280x832, 4000 iterations): 89.8 vs 87.2 iters/s; two float4
// columns per thread: 87.6 (profiles/r04_experiments/loop_ab_4k.txt).
#ifndef GSR_ADAM_NT
#define GSR_ADAM_NT 1
#endif
constexpr int kAdamBlock = 256, kAdamVec = 1, kAdamPerBlock = 4 * kAdamVec * kAdamBlock;
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld4(const float* p) {
#if GSR_ADAM_NT
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *reinterpret_cast<const float4*>(p);
#endif
}
__device__ __forceinline__ void st4(float* p, float4 v) {
#if GSR_ADAM_NT
    const f32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<f32x4*>(p));
#else
    *reinterpret_cast<float4*>(p) = v;
#endif
}

__device__ __forceinline__ float adam_one(float& p, float g, float& m, float& v, float ss, float b2s, const AdamArgs& a) {
    m = fmaf(a.omb1, g, m * a.b1);
    v = fmaf(a.omb2 * g, g, v * a.b2);
    const float denom = sqrtf(v) / b2s + a.eps;
    p = fmaf(-ss, m / denom, p);
    return p;
}

__device__ __forceinline__ void adam_act_grad(int act, float (&p)[4], float (&g)[4]) {
    // activation backward: gradient w.r.t. the raw leaf
    if (act == GSR_ACT_EXP) {
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] = g[k] * expf(p[k]);
    } else if (act == GSR_ACT_SIGMOID) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float s = 1.0f / (1.0f + expf(-p[k]));
            g[k] = g[k] * (1.0f - s) * s;
        }
    } else if (act == GSR_ACT_NORMALIZE4) {  // one row of 4 (n % 4 == 0 checked on the host)
        const float nr = sqrtf(p[0] * p[0] + p[1] * p[1] + p[2] * p[2] + p[3] * p[3]);
        const float n = fmaxf(nr, 1e-12f);
        const float dot = g[0] * p[0] + g[1] * p[1] + g[2] * p[2] + g[3] * p[3];
        // d/dx of x / max(|x|, eps): g / n - (g . x) / n^2 * d|x|/dx (the clamp passes no
        // gradient when it is active)
        const float c = nr > 1e-12f ? dot / (n * n) / nr : 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] = g[k] / n - c * p[k];
    }
}

// kAdamVec float4 columns per thread (column u of a block is coalesced); all loads of the
// thread are issued before any update so that its bytes are in flight together.
__global__ __launch_bounds__(kAdamBlock) void adam_kernel(const AdamArgs a) {
    if (guard_tripped(a.guard_k, a.guard_cap)) return;
    int gi = 0;
    while (gi + 1 < a.ngroups && (int)blockIdx.x >= a.blk_start[gi + 1]) ++gi;  // wave-uniform
    const gsr_adam_group& G = a.g[gi];
    const float ss = a.step_size[gi], b2s = a.bc2_sqrt[gi];
    float p[kAdamVec][4], g[kAdamVec][4], m[kAdamVec][4], v[kAdamVec][4];
    long long e0[kAdamVec];
    int cnt[kAdamVec];
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
        e0[u] = (((long long)(blockIdx.x - a.blk_start[gi]) * kAdamVec + u) * kAdamBlock + threadIdx.x) * 4;
        const long long left = G.n - e0[u];
        cnt[u] = left <= 0 ? 0 : (left < 4 ? (int)left : 4);
        if (cnt[u] == 4) {
            const float4 P4 = ld4(G.param + e0[u]);
            const float4 G4 = ld4(G.grad + e0[u]);
            const float4 M4 = ld4(G.exp_avg + e0[u]);
            const float4 V4 = ld4(G.exp_avg_sq + e0[u]);
            p[u][0] = P4.x, p[u][1] = P4.y, p[u][2] = P4.z, p[u][3] = P4.w;
            g[u][0] = G4.x, g[u][1] = G4.y, g[u][2] = G4.z, g[u][3] = G4.w;
            m[u][0] = M4.x, m[u][1] = M4.y, m[u][2] = M4.z, m[u][3] = M4.w;
            v[u][0] = V4.x, v[u][1] = V4.y, v[u][2] = V4.z, v[u][3] = V4.w;
        } else {
            for (int k = 0; k < 4; ++k) {
                const bool in = k < cnt[u];
                p[u][k] = in ? G.param[e0[u] + k] : 0.f;
                g[u][k] = in ? G.grad[e0[u] + k] : 0.f;
                m[u][k] = in ? G.exp_avg[e0[u] + k] : 0.f;
                v[u][k] = in ? G.exp_avg_sq[e0[u] + k] : 0.f;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
        if (cnt[u] == 0) continue;
        adam_act_grad(G.act, p[u], g[u]);
#pragma unroll
        for (int k = 0; k < 4; ++k) adam_one(p[u][k], g[u][k], m[u][k], v[u][k], ss, b2s, a);
        if (cnt[u] == 4) {
            st4(G.param + e0[u], make_float4(p[u][0], p[u][1], p[u][2], p[u][3]));
            st4(G.exp_avg + e0[u], make_float4(m[u][0], m[u][1], m[u][2], m[u][3]));
            st4(G.exp_avg_sq + e0[u], make_float4(v[u][0], v[u][1], v[u][2], v[u][3]));
        } else {
            for (int k = 0; k < cnt[u]; ++k) {
                G.param[e0[u] + k] = p[u][k];
                G.exp_avg[e0[u] + k] = m[u][k];
                G.exp_avg_sq[e0[u] + k] = v[u][k];
            }
        }
    }
}

// ---------------------------------------------------------------- densification statistics
__global__ __launch_bounds__(256) void densify_stats_kernel(const int* __restrict__ radii, const float* __restrict__ dm2,
                                                            int P, float* __restrict__ maxr, float* __restrict__ acc,
                                                            float* __restrict__ den, const uint32_t* guard_k,
                                                            uint32_t guard_cap) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= P || guard_tripped(guard_k, guard_cap)) return;
    const int r = radii[g];
    if (r <= 0) return;
    maxr[g] = fmaxf(maxr[g], (float)r);
    const float gx = dm2[3 * g], gy = dm2[3 * g + 1];
    acc[g] += sqrtf(gx * gx + gy * gy);
    den[g] += 1.0f;
}

// ---------------------------------------------------------------- compaction
constexpr int kCmpBlock = 256, kCmpPer = 4 * kCmpBlock;

__device__ __forceinline__ int thread_flags(const uint8_t* mask, int n, int base, bool f[4]) {
    int c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[k] = base + k < n && mask[base + k] != 0;
        c += f[k] ? 1 : 0;
    }
    return c;
}

__global__ __launch_bounds__(kCmpBlock) void compact_count_kernel(const uint8_t* __restrict__ mask, int n,
                                                                  int* __restrict__ counts) {
    __shared__ int red[4];
    bool f[4];
    int c = thread_flags(mask, n, (blockIdx.x * kCmpBlock + threadIdx.x) * 4, f);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// exclusive scan of the block counts in one block (chunks of 1024), total -> *total
__global__ __launch_bounds__(1024) void compact_scan_kernel(int* __restrict__ counts, int nb, int* __restrict__ total) {
    __shared__ int s[1024];
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += 1024) {
        const int i = b0 + threadIdx.x;
        const int v = i < nb ? counts[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const int t = (int)threadIdx.x >= o ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < nb) counts[i] = carry + s[threadIdx.x] - v;
        carry += s[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(kCmpBlock) void compact_scatter_kernel(const uint8_t* __restrict__ mask, int n,
                                                                    const int* __restrict__ offs,
                                                                    int* __restrict__ idx) {
    __shared__ int wsum[4];
    bool f[4];
    const int base = (blockIdx.x * kCmpBlock + threadIdx.x) * 4;
    const int c = thread_flags(mask, n, base, f);
    // inclusive wave prefix of c (Hillis-Steele over 64 lanes)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(x, o);
        if (lane >= o) x += t;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int before = offs[blockIdx.x] + x - c;
    for (int w = 0; w < wv; ++w) before += wsum[w];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (f[k]) idx[before++] = base + k;
}

// ---------------------------------------------------------------- multi-tensor row gather
struct GatherArgs {
    gsr_row_copy c[GSR_GATHER_MAX];
};

__global__ __launch_bounds__(256) void gather_rows_kernel(const GatherArgs a, const int* __restrict__ idx, int n_out) {
    const gsr_row_copy& C = a.c[blockIdx.y];
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long tot = (long long)n_out * C.width;
    if (e >= tot) return;
    const int row = (int)(e / C.width), col = (int)(e - (long long)row * C.width);
    C.dst[e] = C.src[(long long)idx[row] * C.width + col];
}

Window ssim_window() {
    // torch: gauss = Tensor([exp(-(x - 5)^2 / (2 sigma^2)) for x in range(11)]) (double exp,
    // stored f32), then gauss / gauss.sum() in f32
    Window w;
    float g[kWin], sum = 0.0f;
    for (int x = 0; x < kWin; ++x) g[x] = (float)std::exp(-(double)((x - kRad) * (x - kRad)) / (2.0 * 1.5 * 1.5));
    for (int x = 0; x < kWin; ++x) sum += g[x];
    for (int x = 0; x < kWin; ++x) w.w[x] = g[x] / sum;
    return w;
}

size_t align256(size_t x) { return (x + 255) / 256 * 256; }

int check_image(const float* img, const float* gt, int C, int H, int W) {
    if (!img || !gt) return set_error(-1, "loss: null image");
    if (C <= 0 || H <= 0 || W <= 0) return set_error(-1, "loss: bad image shape");
    return 0;
}

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

int gsr_activate(const float* scale_raw, const float* rot_raw, const float* opac_raw, int32_t P, float* scales,
                 float* rots, float* opacs, void* stream) {
    if (P < 0) return set_error(-1, "activate: negative P");
    if (P == 0) return 0;
    if ((scales && !scale_raw) || (rots && !rot_raw) || (opacs && !opac_raw)) return set_error(-1, "activate: null input");
    if ((rots && (reinterpret_cast<uintptr_t>(rots) & 15)) || (rot_raw && (reinterpret_cast<uintptr_t>(rot_raw) & 15)))
        return set_error(-1, "activate: rotations must be 16-byte aligned");
    hipLaunchKernelGGL(activate_kernel, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, scale_raw,
                       reinterpret_cast<const float4*>(rot_raw), opac_raw, P, scales, reinterpret_cast<float4*>(rots),
                       opacs);
    return (int)hipGetLastError();
}

size_t gsr_loss_scratch_bytes(int32_t C, int32_t H, int32_t W) {
    const size_t n = (size_t)(C > 0 ? C : 0) * (H > 0 ? H : 0) * (W > 0 ? W : 0);
    const size_t nb = (size_t)((W + kTX - 1) / kTX) * ((H + kTY - 1) / kTY) * (C > 0 ? C : 0);
    return align256(3 * n * sizeof(float)) + align256(nb * sizeof(float2));
}

int gsr_loss_forward(const float* img, const float* gt, int32_t C, int32_t H, int32_t W, float lambda_dssim,
                     void* maps, float* stats, void* stream) {
    if (int e = check_image(img, gt, C, H, W)) return e;
    if (!maps || !stats) return set_error(-1, "loss: null scratch / stats");
    const dim3 grid((W + kTX - 1) / kTX, (H + kTY - 1) / kTY, C);
    const size_t n = (size_t)C * H * W;
    float* m = static_cast<float*>(maps);
    float2* part = reinterpret_cast<float2*>(static_cast<char*>(maps) + align256(3 * n * sizeof(float)));
    const float gscale = (float)(-(double)lambda_dssim / (double)n);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(ssim_forward_kernel, grid, dim3(256), 0, s, img, gt, H, W, ssim_window(), gscale, m, part);
    const int nparts = (int)(grid.x * grid.y * grid.z);
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, part, nparts, 1.0 / (double)n, lambda_dssim,
                       stats);
    return (int)hipGetLastError();
}

int gsr_loss_backward(const float* img, const float* gt, int32_t C, int32_t H, int32_t W, float lambda_dssim,
                      const void* maps, float* dL_dimg, void* stream) {
    if (int e = check_image(img, gt, C, H, W)) return e;
    if (!maps || !dL_dimg) return set_error(-1, "loss: null scratch / output");
    const dim3 grid((W + kTX - 1) / kTX, (H + kTY - 1) / kTY, C);
    const size_t n = (size_t)C * H * W;
    const float l1scale = (float)((1.0 - (double)lambda_dssim) / (double)n);
    hipLaunchKernelGGL(ssim_backward_kernel, grid, dim3(256), 0, (hipStream_t)stream, img, gt, H, W, ssim_window(),
                       l1scale, static_cast<const float*>(maps), dL_dimg);
    return (int)hipGetLastError();
}

int gsr_adam_step(const gsr_adam_group* groups, int32_t ngroups, float beta1, float beta2, float eps, void* stream) {
    return gsr_adam_step_guarded(groups, ngroups, beta1, beta2, eps, nullptr, 0, stream);
}

int gsr_adam_step_guarded(const gsr_adam_group* groups, int32_t ngroups, float beta1, float beta2, float eps,
                          const uint32_t* guard_k, uint32_t guard_cap, void* stream) {
    if (ngroups < 0 || ngroups > GSR_ADAM_MAX_GROUPS) return set_error(-1, "adam: 0..8 groups");
    if (ngroups == 0) return 0;
    if (!groups) return set_error(-1, "adam: null groups");
    AdamArgs a;
    std::memset(&a, 0, sizeof a);
    a.ngroups = ngroups;
    a.b1 = beta1;
    a.b2 = beta2;
    a.eps = eps;
    a.omb1 = (float)(1.0 - (double)beta1);
    a.omb2 = (float)(1.0 - (double)beta2);
    a.guard_k = guard_k;
    a.guard_cap = guard_cap;
    long long blocks = 0;
    for (int i = 0; i < ngroups; ++i) {
        const gsr_adam_group& g = groups[i];
        if (g.n < 0) return set_error(-1, "adam: negative group size");
        if (g.n > 0 && (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq)) return set_error(-1, "adam: null tensor");
        if (g.step < 1) return set_error(-1, "adam: step must be >= 1");
        if (g.act < GSR_ACT_NONE || g.act > GSR_ACT_NORMALIZE4) return set_error(-1, "adam: bad activation");
        if (g.act == GSR_ACT_NORMALIZE4 && g.n % 4) return set_error(-1, "adam: normalize group needs rows of 4");
        for (const void* p : {(const void*)g.param, (const void*)g.grad, (const void*)g.exp_avg, (const void*)g.exp_avg_sq})
            if (reinterpret_cast<uintptr_t>(p) & 15) return set_error(-1, "adam: tensors must be 16-byte aligned");
        a.g[i] = g;
        a.blk_start[i] = (int)blocks;
        blocks += (g.n + kAdamPerBlock - 1) / kAdamPerBlock;
        // libtorch adam.cpp: bias corrections in double, scalars cast to the tensor type
        const double bc1 = 1.0 - std::pow((double)beta1, (double)g.step);
        const double bc2 = 1.0 - std::pow((double)beta2, (double)g.step);
        a.step_size[i] = (float)((double)g.lr / bc1);
        a.bc2_sqrt[i] = (float)std::sqrt(bc2);
    }
    if (blocks > INT32_MAX / 2) return set_error(-1, "adam: too many elements");
    a.blk_start[ngroups] = (int)blocks;
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(kAdamBlock), 0, (hipStream_t)stream, a);
    return (int)hipGetLastError();
}

int gsr_densify_stats(const int32_t* radii, const float* dmeans2D, int32_t P, float* max_radii2D, float* grad_accum,
                      float* denom, void* stream) {
    return gsr_densify_stats_guarded(radii, dmeans2D, P, max_radii2D, grad_accum, denom, nullptr, 0, stream);
}

int gsr_densify_stats_guarded(const int32_t* radii, const float* dmeans2D, int32_t P, float* max_radii2D,
                              float* grad_accum, float* denom, const uint32_t* guard_k, uint32_t guard_cap,
                              void* stream) {
    if (P < 0) return set_error(-1, "densify_stats: negative P");
    if (P == 0) return 0;
    if (!radii || !dmeans2D || !max_radii2D || !grad_accum || !denom) return set_error(-1, "densify_stats: null tensor");
    hipLaunchKernelGGL(densify_stats_kernel, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, radii, dmeans2D, P,
                       max_radii2D, grad_accum, denom, guard_k, guard_cap);
    return (int)hipGetLastError();
}

size_t gsr_compact_scratch_bytes(int32_t n) {
    const size_t nb = (size_t)((n > 0 ? n : 0) + kCmpPer - 1) / kCmpPer;
    return align256((nb + 1) * sizeof(int));
}

int gsr_compact_index(const uint8_t* mask, int32_t n, int32_t* idx_out, int32_t* count_out, void* scratch, void* stream) {
    if (n < 0) return set_error(-1, "compact: negative n");
    if (!count_out || !scratch || (n > 0 && (!mask || !idx_out))) return set_error(-1, "compact: null pointer");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) return (int)hipMemsetAsync(count_out, 0, sizeof(int32_t), s);
    const int nb = (n + kCmpPer - 1) / kCmpPer;
    int* counts = static_cast<int*>(scratch);
    hipLaunchKernelGGL(compact_count_kernel, dim3(nb), dim3(kCmpBlock), 0, s, mask, n, counts);
    hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, s, counts, nb, count_out);
    hipLaunchKernelGGL(compact_scatter_kernel, dim3(nb), dim3(kCmpBlock), 0, s, mask, n, counts, idx_out);
    return (int)hipGetLastError();
}

int gsr_gather_rows(const gsr_row_copy* copies, int32_t ncopies, const int32_t* idx, int32_t n_out, void* stream) {
    if (ncopies < 0 || ncopies > GSR_GATHER_MAX) return set_error(-1, "gather_rows: 0..24 copies");
    if (n_out < 0) return set_error(-1, "gather_rows: negative n_out");
    if (ncopies == 0 || n_out == 0) return 0;
    if (!copies || !idx) return set_error(-1, "gather_rows: null pointer");
    GatherArgs a;
    std::memset(&a, 0, sizeof a);
    long long maxw = 0;
    for (int i = 0; i < ncopies; ++i) {
        if (!copies[i].src || !copies[i].dst || copies[i].width <= 0) return set_error(-1, "gather_rows: bad copy");
        if (copies[i].src == copies[i].dst) return set_error(-1, "gather_rows: dst aliases src");
        a.c[i] = copies[i];
        maxw = copies[i].width > maxw ? copies[i].width : maxw;
    }
    const long long blocks = ((long long)n_out * maxw + 255) / 256;
    if (blocks > INT32_MAX) return set_error(-1, "gather_rows: too large");
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)blocks, ncopies), dim3(256), 0, (hipStream_t)stream, a, idx,
                       n_out);
    return (int)hipGetLastError();
}

}  // extern "C"

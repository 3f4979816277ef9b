// gsr_preprocess_bwd.hip -- B2: per-Gaussian chain rule from the 2D gradients (mean2D, conic,
// opacity, colour) to the leaves (means3D, SH, scales, rotations, or the precomputed colour /
// cov3D), on gfx950.  One thread per Gaussian; every output element is written (zeros for
// culled Gaussians) so the caller can hand in uninitialised tensors.
//
// The per-Gaussian 2D gradient (grad2d) is the sum of its per-(tile, instance) partials in
// emission order (rect row-major), read from the contiguous range [inst_start[g], +tiles[g])
// by gather_grad2d_kernel -- a fixed order, so results are bitwise reproducible run to run.
//
// Derivation (restated; same formulas as oracle/gsr_oracle.c
// preprocess_backward_one): conic (A,B,C) = inv([[a,b],[b,c]]), cov2D = T Sigma T^T with
// T = J W, J the EWA Jacobian (x/y terms zeroed outside the 1.3 tan(fov) clamp), Sigma = L L^T,
// L = R(q) diag(mod s) (src/utils/general_utils.cpp:24-37,91-97), SH basis derivatives w.r.t.
// the normalised view direction, NDC mean through the homogeneous divide.
//
// Roofline: HBM-bound (V*(80+12M) + N*(60+12M) bytes).
#include "gsr_kernels.h"

namespace gsr {
namespace {

__constant__ float kC2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                             -1.0925484305920792f, 0.5462742152960396f};
__constant__ float kC3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                             0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                             -0.5900435899266435f};
constexpr float kC0 = 0.28209479177387814f;
constexpr float kC1 = 0.4886025119029199f;

// Per-Gaussian sum of its per-(tile, instance) partials in emission order.  A block owns 256
// consecutive Gaussians; their segments [offsets[g-1], offsets[g]) tile one contiguous
// stretch of the partial arrays, which the block streams through LDS in coalesced windows of
// kGatherWin entries.  Only entries B1 flagged (records that changed a pixel) are loaded; the
// rest count as zeros, so the partial block itself is never cleared and entries of records past
// a tile's termination are never read.  Each thread then adds the part of its own segment that
// lies in the window, in order, from LDS.  The partials are B1's raw tile moments (Sx, Sy, Sxx,
// Sxy, Syy, S0, colour x3, gsr_blend.hip); they are linear in the 2D gradients, so the
// conversion runs once on the per-Gaussian sum, with the Gaussian's own conic and opacity from
// its blend record.  The 48-B result lands at grad2d[gid].
constexpr int kGatherWin = 512;
#ifndef GSR_GATHER_FLAG_AHEAD
#define GSR_GATHER_FLAG_AHEAD 1
#endif
#ifndef GSR_GATHER_DATA_AHEAD
#define GSR_GATHER_DATA_AHEAD 1
#endif

// rrect (presort mode): index i is a depth rank whose emission range the rank-order offsets give;
// its Gaussian (record read, grad2d row written) is rrect[i].z.  nullptr: i is the gid itself.
__global__ __launch_bounds__(256) void gather_grad2d_kernel(const uint32_t* __restrict__ offsets,
                                                            const float4* __restrict__ p8,
                                                            const float* __restrict__ p1,
                                                            const uint8_t* __restrict__ fl,
                                                            const float4* __restrict__ rec, float hw, float hh,
                                                            int P, uint32_t cap, const uint4* __restrict__ rrect,
                                                            float* __restrict__ grad2d, uint32_t split) {
    __shared__ float4 w8[2 * kGatherWin];
    __shared__ float w1[kGatherWin];
    __shared__ uint32_t wv[kGatherWin / 4];
    const int g0 = blockIdx.x * 256, g = g0 + threadIdx.x;
    const int gl = (P - g0 < 256 ? P - g0 : 256) + g0;  // one past the block's last Gaussian
    // emission indices past the binning's capacity were never emitted (overflow): clamped; a
    // split B1 (band launches) wrote `split` consecutive entries per instance, summed in order
    auto off = [&](int i) { const uint32_t o = offsets[i]; return (o < cap ? o : cap) * split; };
    const uint32_t J0 = g0 ? off(g0 - 1) : 0u, J1 = off(gl - 1);
    const uint32_t s = g < P ? (g ? off(g - 1) : 0u) : 0u;
    const uint32_t e = g < P ? off(g) : 0u;
    const uint32_t gid = g < P ? (rrect ? rrect[g].z : (uint32_t)g) : 0u;
    // the Gaussian's conic and opacity, loaded before the window loop (latency overlaps it)
    float4 q0 = make_float4(0.f, 0.f, 0.f, 0.f), q1 = q0;
    if (g < P && e > s) {
        q0 = rec[3 * (size_t)gid];
        q1 = rec[3 * (size_t)gid + 1];
    }
    float a[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) a[k] = 0.f;
    const uint8_t* wvb = reinterpret_cast<const uint8_t*>(wv);
#if GSR_GATHER_DATA_AHEAD
    // Each window's entries are loaded into registers during the previous window's sums (4 float4 +
    // 2 floats per thread), and its flags a window earlier still (double-buffered in LDS): after
    // the first window no window waits on a load round at all.
    static_assert(kGatherWin == 512, "two entries per thread");
    __shared__ uint32_t wvd[2][kGatherWin / 4];
    (void)wvb;
    auto nwin = [&](uint32_t W) -> uint32_t {
        return W < J1 ? (J1 - W < (uint32_t)kGatherWin ? J1 - W : (uint32_t)kGatherWin) : 0u;
    };
    float4 d8[4];
    float d1[2];
    auto load_data = [&](uint32_t Wx, uint32_t nx, const uint8_t* fb) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = threadIdx.x + 256u * k;
            d8[k] = i < 2 * nx && fb[i >> 1] ? p8[2 * (size_t)Wx + i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t i = threadIdx.x + 256u * k;
            d1[k] = i < nx && fb[i] ? p1[(size_t)Wx + i] : 0.f;
        }
    };
    uint32_t fa = 0u, fb2 = 0u;  // flags of the window after the next
    if (J0 < J1) {
        const uint32_t n0 = nwin(J0);
        uint8_t* f0 = reinterpret_cast<uint8_t*>(wvd[0]);
        if (threadIdx.x < n0) f0[threadIdx.x] = fl[(size_t)J0 + threadIdx.x];
        if (threadIdx.x + 256 < n0) f0[threadIdx.x + 256] = fl[(size_t)J0 + threadIdx.x + 256];
        __syncthreads();
        load_data(J0, n0, f0);
        const uint32_t n1 = nwin(J0 + kGatherWin);
        if (threadIdx.x < n1) fa = fl[(size_t)J0 + kGatherWin + threadIdx.x];
        if (threadIdx.x + 256 < n1) fb2 = fl[(size_t)J0 + kGatherWin + threadIdx.x + 256];
    }
    int buf = 0;
    for (uint32_t W = J0; W < J1; W += kGatherWin, buf ^= 1) {
        const uint32_t n = nwin(W);
        // this window's entries -> LDS; the next window's flags -> the other flag buffer
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = threadIdx.x + 256u * k;
            if (i < 2 * n) w8[i] = d8[k];
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t i = threadIdx.x + 256u * k;
            if (i < n) w1[i] = d1[k];
        }
        uint8_t* const fnx = reinterpret_cast<uint8_t*>(wvd[buf ^ 1]);
        const uint32_t n1 = nwin(W + kGatherWin);
        if (threadIdx.x < n1) fnx[threadIdx.x] = (uint8_t)fa;
        if (threadIdx.x + 256 < n1) fnx[threadIdx.x + 256] = (uint8_t)fb2;
        __syncthreads();
        // the next window's entries and the flags after it stay in flight during this window's sums
        if (n1) load_data(W + kGatherWin, n1, fnx);
        const uint32_t n2 = nwin(W + 2 * kGatherWin);
        fa = threadIdx.x < n2 ? fl[(size_t)W + 2 * kGatherWin + threadIdx.x] : 0u;
        fb2 = threadIdx.x + 256 < n2 ? fl[(size_t)W + 2 * kGatherWin + threadIdx.x + 256] : 0u;
        const uint32_t lo = s > W ? s : W, hi = e < W + n ? e : W + n;
        for (uint32_t j = lo; j < hi; ++j) {
            const float4 u = w8[2 * (j - W)], v = w8[2 * (j - W) + 1];
            a[0] += u.x; a[1] += u.y; a[2] += u.z; a[3] += u.w;
            a[4] += v.x; a[5] += v.y; a[6] += v.z; a[7] += v.w;
            a[8] += w1[j - W];
        }
        __syncthreads();
    }
#else
#if GSR_GATHER_FLAG_AHEAD
    // each window's flags are loaded during the previous window's entry loads (two per thread in
    // registers), so a window waits for one load round, not two
    static_assert(kGatherWin == 512, "two flags per thread");
    uint32_t fa = 0u, fb = 0u;
    {
        const uint32_t n0 = J1 - J0 < (uint32_t)kGatherWin ? J1 - J0 : (uint32_t)kGatherWin;
        if (threadIdx.x < n0) fa = fl[(size_t)J0 + threadIdx.x];
        if (threadIdx.x + 256 < n0) fb = fl[(size_t)J0 + threadIdx.x + 256];
    }
#endif
    for (uint32_t W = J0; W < J1; W += kGatherWin) {
        const uint32_t n = J1 - W < (uint32_t)kGatherWin ? J1 - W : (uint32_t)kGatherWin;
#if GSR_GATHER_FLAG_AHEAD
        if (threadIdx.x < n) reinterpret_cast<uint8_t*>(wv)[threadIdx.x] = (uint8_t)fa;
        if (threadIdx.x + 256 < n) reinterpret_cast<uint8_t*>(wv)[threadIdx.x + 256] = (uint8_t)fb;
        __syncthreads();
        {
            const uint32_t W2 = W + kGatherWin;
            const uint32_t n2 = W2 < J1 ? (J1 - W2 < (uint32_t)kGatherWin ? J1 - W2 : (uint32_t)kGatherWin) : 0u;
            fa = threadIdx.x < n2 ? fl[(size_t)W2 + threadIdx.x] : 0u;
            fb = threadIdx.x + 256 < n2 ? fl[(size_t)W2 + threadIdx.x + 256] : 0u;
        }
#else
        for (uint32_t i = threadIdx.x; i < n; i += 256) reinterpret_cast<uint8_t*>(wv)[i] = fl[(size_t)W + i];
        __syncthreads();
#endif
        for (uint32_t i = threadIdx.x; i < 2 * n; i += 256)
            w8[i] = wvb[i >> 1] ? p8[2 * (size_t)W + i] : make_float4(0.f, 0.f, 0.f, 0.f);
        for (uint32_t i = threadIdx.x; i < n; i += 256) w1[i] = wvb[i] ? p1[(size_t)W + i] : 0.f;
        __syncthreads();
        const uint32_t lo = s > W ? s : W, hi = e < W + n ? e : W + n;
        for (uint32_t j = lo; j < hi; ++j) {
            const float4 u = w8[2 * (j - W)], v = w8[2 * (j - W) + 1];
            a[0] += u.x; a[1] += u.y; a[2] += u.z; a[3] += u.w;
            a[4] += v.x; a[5] += v.y; a[6] += v.z; a[7] += v.w;
            a[8] += w1[j - W];
        }
        __syncthreads();
    }
#endif
    if (g >= P) return;
    // moments -> d mean2D (NDC), d conic, d opacity (sum G dL/dalpha = S0 / o), d colour
    const float A = -2.0f * kLn2 * q0.z, B = -kLn2 * q0.w, C = -2.0f * kLn2 * q1.x;
    const float Sx = a[0], Sy = a[1], S0 = a[5];
    float4* dst = reinterpret_cast<float4*>(grad2d + (size_t)kPart * gid);
    dst[0] = make_float4((-A * Sx - B * Sy) * hw, (-C * Sy - B * Sx) * hh, -0.5f * a[2], -a[3]);
    dst[1] = make_float4(-0.5f * a[4], S0 != 0.0f ? S0 / q1.y : 0.0f, a[6], a[7]);
    dst[2] = make_float4(a[8], 0.f, 0.f, 0.f);
}

// Per-Gaussian inputs of B2, loaded before the SH rows are staged so that their HBM
// latency overlaps the staging instead of following it.
struct BwdIn {
    bool visible;
    float g2[9];
    float p0, p1, p2;
    float c3[6];  // cov3D, or (rotation w, x, y, z, unused x2)
    float s[3];   // raw scales
    uint32_t cl;  // stored SH clamp bits (flags != nullptr)
};

template <bool SUM>
__device__ __forceinline__ BwdIn load_bwd_in(const GaussIn& in, int g, int o, const uint32_t* __restrict__ depth_key,
                                             const uint32_t* __restrict__ flags, const float* __restrict__ grad2d,
                                             const BandSum& bs) {
    BwdIn b;
    b.visible = depth_key[g] != 0xFFFFFFFFu;
    float4 v0, v1, v2;
    if (SUM) {  // the bands' returned rows, summed in band order
        v0 = make_float4(0.f, 0.f, 0.f, 0.f);
        v1 = v0;
        v2 = v0;
        if (bs.tiles[g] != 0u) {
            const uint4 rr = bs.rect[g];
            int b_lo, b_hi;
            band_span(bs.br, rr.x >> 16, rr.y >> 16, b_lo, b_hi);
            for (int k = b_lo; k <= b_hi; ++k) {
                const uint32_t slot = bs.slot_of[(size_t)k * in.P + g];
                if (slot >= (uint32_t)bs.pair_cap) continue;  // overflowed: never sent
                const float4* src = bs.back + ((size_t)k * bs.pair_cap + slot) * 3;
                const float4 u = src[0], v = src[1], w = src[2];
                v0.x += u.x; v0.y += u.y; v0.z += u.z; v0.w += u.w;
                v1.x += v.x; v1.y += v.y; v1.z += v.z; v1.w += v.w;
                v2.x += w.x;
            }
        }
    } else {
        const float4* src = reinterpret_cast<const float4*>(grad2d + (size_t)kPart * o);
        v0 = src[0];
        v1 = src[1];
        v2 = src[2];
    }
    b.g2[0] = v0.x; b.g2[1] = v0.y; b.g2[2] = v0.z; b.g2[3] = v0.w;
    b.g2[4] = v1.x; b.g2[5] = v1.y; b.g2[6] = v1.z; b.g2[7] = v1.w;
    b.g2[8] = v2.x;
    b.p0 = in.means3D[3 * g + 0];
    b.p1 = in.means3D[3 * g + 1];
    b.p2 = in.means3D[3 * g + 2];
    if (in.cov3D) {
#pragma unroll
        for (int k = 0; k < 6; ++k) b.c3[k] = in.cov3D[6 * g + k];
        b.s[0] = b.s[1] = b.s[2] = 0.f;
    } else {
        const float4 q = *reinterpret_cast<const float4*>(in.rots + 4 * g);
        b.c3[0] = q.x; b.c3[1] = q.y; b.c3[2] = q.z; b.c3[3] = q.w; b.c3[4] = b.c3[5] = 0.f;
        b.s[0] = in.scales[3 * g + 0];
        b.s[1] = in.scales[3 * g + 1];
        b.s[2] = in.scales[3 * g + 2];
    }
    b.cl = flags ? flags[g] : 0u;
    return b;
}

// One Gaussian's chain rule.  `lrest`: this thread's SH-rest row staged in LDS (read, then
// overwritten in place with the row's gradient), or nullptr when there is no SH-rest input.
__device__ __forceinline__ void preprocess_backward_one(const gsr_camera& cam, const GaussIn& in, int g, int o,
                                                        const BwdIn& bi, const uint32_t* __restrict__ flags,
                                                        const GradOut& out, float* lrest) {
    const bool visible = bi.visible;
    // ---- 2D gradients ----
    float g2[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) g2[k] = visible ? bi.g2[k] : 0.f;
    out.means2D[3 * o + 0] = g2[0];
    out.means2D[3 * o + 1] = g2[1];
    out.means2D[3 * o + 2] = 0.f;
    if (out.conic) {
        out.conic[3 * o + 0] = g2[2];
        out.conic[3 * o + 1] = g2[3];
        out.conic[3 * o + 2] = g2[4];
    }
    out.opac[o] = g2[5];

    const float* V = cam.viewmatrix;
    const float* Pm = cam.projmatrix;
    const float p0 = bi.p0, p1 = bi.p1, p2 = bi.p2;
    const float p[3] = {p0, p1, p2};
    float dm[3] = {0.f, 0.f, 0.f};
    const int D = in.D;
    const int nb = (D + 1) * (D + 1);

    if (!visible) {
        if (in.colors) {
#pragma unroll
            for (int k = 0; k < 3; ++k) out.colors[3 * o + k] = 0.f;
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) out.sh_dc[3 * o + k] = 0.f;
            if (lrest)
                for (int k = 0; k < 3 * in.M_rest; ++k) lrest[k] = 0.f;
        }
        out.means3D[3 * o + 0] = 0.f;
        out.means3D[3 * o + 1] = 0.f;
        out.means3D[3 * o + 2] = 0.f;
        if (in.cov3D) {
#pragma unroll
            for (int k = 0; k < 6; ++k) out.cov3D[6 * o + k] = 0.f;
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) out.scales[3 * o + k] = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) out.rots[4 * o + k] = 0.f;
        }
        return;
    }
    // ---- colour -> SH / view direction ----
    if (in.colors) {
        out.colors[3 * o + 0] = g2[6];
        out.colors[3 * o + 1] = g2[7];
        out.colors[3 * o + 2] = g2[8];
    } else {
        const float vx = p0 - cam.campos[0], vy = p1 - cam.campos[1], vz = p2 - cam.campos[2];
        const float len = sqrtf(vx * vx + vy * vy + vz * vz);
        const float x = vx / len, y = vy / len, z = vz / len;
        float basis[16], dbx[16], dby[16], dbz[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) basis[k] = dbx[k] = dby[k] = dbz[k] = 0.f;
        basis[0] = kC0;
        if (D >= 1) {
            basis[1] = -kC1 * y; basis[2] = kC1 * z; basis[3] = -kC1 * x;
            dby[1] = -kC1; dbz[2] = kC1; dbx[3] = -kC1;
        }
        if (D >= 2) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            basis[4] = kC2[0] * xy;
            basis[5] = kC2[1] * yz;
            basis[6] = kC2[2] * (2.0f * zz - xx - yy);
            basis[7] = kC2[3] * xz;
            basis[8] = kC2[4] * (xx - yy);
            dbx[4] = kC2[0] * y; dby[4] = kC2[0] * x;
            dby[5] = kC2[1] * z; dbz[5] = kC2[1] * y;
            dbx[6] = kC2[2] * -2.f * x; dby[6] = kC2[2] * -2.f * y; dbz[6] = kC2[2] * 4.f * z;
            dbx[7] = kC2[3] * z; dbz[7] = kC2[3] * x;
            dbx[8] = kC2[4] * 2.f * x; dby[8] = kC2[4] * -2.f * y;
            if (D >= 3) {
                basis[9] = kC3[0] * y * (3.0f * xx - yy);
                basis[10] = kC3[1] * xy * z;
                basis[11] = kC3[2] * y * (4.0f * zz - xx - yy);
                basis[12] = kC3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                basis[13] = kC3[4] * x * (4.0f * zz - xx - yy);
                basis[14] = kC3[5] * z * (xx - yy);
                basis[15] = kC3[6] * x * (xx - 3.0f * yy);
                dbx[9] = kC3[0] * 6.f * xy; dby[9] = kC3[0] * 3.f * (xx - yy);
                dbx[10] = kC3[1] * yz; dby[10] = kC3[1] * xz; dbz[10] = kC3[1] * xy;
                dbx[11] = kC3[2] * -2.f * xy; dby[11] = kC3[2] * (4.f * zz - xx - 3.f * yy); dbz[11] = kC3[2] * 8.f * yz;
                dbx[12] = kC3[3] * -6.f * xz; dby[12] = kC3[3] * -6.f * yz; dbz[12] = kC3[3] * (6.f * zz - 3.f * xx - 3.f * yy);
                dbx[13] = kC3[4] * (4.f * zz - 3.f * xx - yy); dby[13] = kC3[4] * -2.f * xy; dbz[13] = kC3[4] * 8.f * xz;
                dbx[14] = kC3[5] * 2.f * xz; dby[14] = kC3[5] * -2.f * yz; dbz[14] = kC3[5] * (xx - yy);
                dbx[15] = kC3[6] * 3.f * (xx - yy); dby[15] = kC3[6] * -6.f * xy;
            }
        }
        // Clamp bits of the forward's SH->RGB: stored by a full-image forward, else recomputed
        // with the forward's exact arithmetic (same basis expressions and summation order, both
        // files built -ffp-contract=off; gsr_preprocess.hip) -- a banded forward skips SH for
        // Gaussians outside its band, which B2 on this rank's slice may still need.
        uint32_t cl = 0;
        if (flags) {
            cl = bi.cl;
        } else {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            float r = basis[0] * in.sh_dc[3 * g + ch];
            if (lrest) {
#pragma unroll
                for (int k = 1; k < 16; ++k)
                    if (k < nb) r = r + basis[k] * lrest[3 * (k - 1) + ch];
            }
            r = r + 0.5f;
            cl |= (r < 0.0f ? 1u : 0u) << ch;
        }
        }
        const float dres[3] = {(cl & 1u) ? 0.f : g2[6], (cl & 2u) ? 0.f : g2[7], (cl & 4u) ? 0.f : g2[8]};
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) out.sh_dc[3 * o + ch] = basis[0] * dres[ch];
        float ddx = 0.f, ddy = 0.f, ddz = 0.f;
        if (lrest) {
            const float* rest = lrest;
            float* drest = lrest;
#pragma unroll
            for (int k = 1; k < 16; ++k) {
                if (k > in.M_rest) break;
                if (k < nb) {
                    const float c0 = rest[3 * (k - 1) + 0], c1 = rest[3 * (k - 1) + 1], c2 = rest[3 * (k - 1) + 2];
                    drest[3 * (k - 1) + 0] = basis[k] * dres[0];
                    drest[3 * (k - 1) + 1] = basis[k] * dres[1];
                    drest[3 * (k - 1) + 2] = basis[k] * dres[2];
                    const float sdot = c0 * dres[0] + c1 * dres[1] + c2 * dres[2];
                    ddx += dbx[k] * sdot;
                    ddy += dby[k] * sdot;
                    ddz += dbz[k] * sdot;
                } else {
                    drest[3 * (k - 1) + 0] = 0.f;
                    drest[3 * (k - 1) + 1] = 0.f;
                    drest[3 * (k - 1) + 2] = 0.f;
                }
            }
        }
        const float dd = x * ddx + y * ddy + z * ddz;
        dm[0] += (ddx - x * dd) / len;
        dm[1] += (ddy - y * dd) / len;
        dm[2] += (ddz - z * dd) / len;
    }
    // ---- mean2D (NDC) -> mean3D ----
    {
        const float hx = Pm[0] * p0 + Pm[4] * p1 + Pm[8] * p2 + Pm[12];
        const float hy = Pm[1] * p0 + Pm[5] * p1 + Pm[9] * p2 + Pm[13];
        const float hw = Pm[3] * p0 + Pm[7] * p1 + Pm[11] * p2 + Pm[15];
        const float mw = 1.0f / (hw + 0.0000001f);
        const float mw2 = mw * mw;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            dm[k] += (Pm[4 * k + 0] * mw - Pm[4 * k + 3] * hx * mw2) * g2[0] +
                     (Pm[4 * k + 1] * mw - Pm[4 * k + 3] * hy * mw2) * g2[1];
    }
    // ---- conic -> cov2D -> (cov3D, view-space mean) ----
    float c3[6], R[9], se[3] = {0.f, 0.f, 0.f};
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    if (in.cov3D) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3[k] = bi.c3[k];
    } else {
        q = make_float4(bi.c3[0], bi.c3[1], bi.c3[2], bi.c3[3]);
        const float r = q.x, x = q.y, y = q.z, z = q.w;
        R[0] = 1.f - 2.f * (y * y + z * z);
        R[1] = 2.f * (x * y - r * z);
        R[2] = 2.f * (x * z + r * y);
        R[3] = 2.f * (x * y + r * z);
        R[4] = 1.f - 2.f * (x * x + z * z);
        R[5] = 2.f * (y * z - r * x);
        R[6] = 2.f * (x * z - r * y);
        R[7] = 2.f * (y * z + r * x);
        R[8] = 1.f - 2.f * (x * x + y * y);
        se[0] = in.smod * bi.s[0];
        se[1] = in.smod * bi.s[1];
        se[2] = in.smod * bi.s[2];
        float L[9];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) L[3 * i + j] = R[3 * i + j] * se[j];
        c3[0] = L[0] * L[0] + L[1] * L[1] + L[2] * L[2];
        c3[1] = L[0] * L[3] + L[1] * L[4] + L[2] * L[5];
        c3[2] = L[0] * L[6] + L[1] * L[7] + L[2] * L[8];
        c3[3] = L[3] * L[3] + L[4] * L[4] + L[5] * L[5];
        c3[4] = L[3] * L[6] + L[4] * L[7] + L[5] * L[8];
        c3[5] = L[6] * L[6] + L[7] * L[7] + L[8] * L[8];
    }
    const float tx = V[0] * p0 + V[4] * p1 + V[8] * p2 + V[12];
    const float ty = V[1] * p0 + V[5] * p1 + V[9] * p2 + V[13];
    const float tz = V[2] * p0 + V[6] * p1 + V[10] * p2 + V[14];
    const float Wf = (float)cam.width, Hf = (float)cam.height;
    const float fx = Wf / (2.0f * cam.tanfovx), fy = Hf / (2.0f * cam.tanfovy);
    const float limx = 1.3f * cam.tanfovx, limy = 1.3f * cam.tanfovy;
    const float txtz = tx / tz, tytz = ty / tz;
    const float cx = fminf(limx, fmaxf(-limx, txtz)) * tz;
    const float cy = fminf(limy, fmaxf(-limy, tytz)) * tz;
    const float xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    const float ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    const float tz2 = tz * tz, tz3 = tz2 * tz;
    const float J00 = fx / tz, J02 = -(fx * cx) / tz2, J11 = fy / tz, J12 = -(fy * cy) / tz2;
    float T0[3], T1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        T0[k] = J00 * V[4 * k + 0] + J02 * V[4 * k + 2];
        T1[k] = J11 * V[4 * k + 1] + J12 * V[4 * k + 2];
    }
    const float S[9] = {c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]};
    float ST0[3], ST1[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        ST0[i] = S[3 * i + 0] * T0[0] + S[3 * i + 1] * T0[1] + S[3 * i + 2] * T0[2];
        ST1[i] = S[3 * i + 0] * T1[0] + S[3 * i + 1] * T1[1] + S[3 * i + 2] * T1[2];
    }
    const float a = (ST0[0] * T0[0] + ST0[1] * T0[1] + ST0[2] * T0[2]) + 0.3f;
    const float b = ST0[0] * T1[0] + ST0[1] * T1[1] + ST0[2] * T1[2];
    const float c = (ST1[0] * T1[0] + ST1[1] * T1[1] + ST1[2] * T1[2]) + 0.3f;
    const float det = a * c - b * b;
    const float dA = g2[2], dB = g2[3], dC = g2[4];
    const float inv2 = 1.0f / (det * det);
    const float dL_da = inv2 * (-c * c * dA + b * c * dB - b * b * dC);
    const float dL_db = inv2 * (2.f * b * c * dA - (a * c + b * b) * dB + 2.f * a * b * dC);
    const float dL_dc = inv2 * (-b * b * dA + a * b * dB - a * a * dC);
    float dS[6];
    dS[0] = T0[0] * T0[0] * dL_da + T0[0] * T1[0] * dL_db + T1[0] * T1[0] * dL_dc;
    dS[3] = T0[1] * T0[1] * dL_da + T0[1] * T1[1] * dL_db + T1[1] * T1[1] * dL_dc;
    dS[5] = T0[2] * T0[2] * dL_da + T0[2] * T1[2] * dL_db + T1[2] * T1[2] * dL_dc;
    dS[1] = 2.f * T0[0] * T0[1] * dL_da + (T0[0] * T1[1] + T0[1] * T1[0]) * dL_db + 2.f * T1[0] * T1[1] * dL_dc;
    dS[2] = 2.f * T0[0] * T0[2] * dL_da + (T0[0] * T1[2] + T0[2] * T1[0]) * dL_db + 2.f * T1[0] * T1[2] * dL_dc;
    dS[4] = 2.f * T0[1] * T0[2] * dL_da + (T0[1] * T1[2] + T0[2] * T1[1]) * dL_db + 2.f * T1[1] * T1[2] * dL_dc;
    float dJ00 = 0.f, dJ02 = 0.f, dJ11 = 0.f, dJ12 = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float dT0 = 2.f * ST0[i] * dL_da + ST1[i] * dL_db;
        const float dT1 = 2.f * ST1[i] * dL_dc + ST0[i] * dL_db;
        dJ00 += dT0 * V[4 * i + 0];
        dJ02 += dT0 * V[4 * i + 2];
        dJ11 += dT1 * V[4 * i + 1];
        dJ12 += dT1 * V[4 * i + 2];
    }
    const float dtx = xmul * (-fx / tz2) * dJ02;
    const float dty = ymul * (-fy / tz2) * dJ12;
    const float dtz = (-fx / tz2) * dJ00 + (-fy / tz2) * dJ11 + (2.f * fx * cx / tz3) * dJ02 +
                      (2.f * fy * cy / tz3) * dJ12;
#pragma unroll
    for (int k = 0; k < 3; ++k) dm[k] += V[4 * k + 0] * dtx + V[4 * k + 1] * dty + V[4 * k + 2] * dtz;
    out.means3D[3 * o + 0] = dm[0];
    out.means3D[3 * o + 1] = dm[1];
    out.means3D[3 * o + 2] = dm[2];
    (void)p;
    // ---- cov3D -> scale, rotation ----
    if (in.cov3D) {
#pragma unroll
        for (int k = 0; k < 6; ++k) out.cov3D[6 * o + k] = dS[k];
        return;
    }
    const float Gm[9] = {dS[0], 0.5f * dS[1], 0.5f * dS[2], 0.5f * dS[1], dS[3], 0.5f * dS[4],
                         0.5f * dS[2], 0.5f * dS[4], dS[5]};
    float L[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) L[3 * i + j] = R[3 * i + j] * se[j];
    float dR[9];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const float dl = 2.f * (Gm[3 * i + 0] * L[0 + j] + Gm[3 * i + 1] * L[3 + j] + Gm[3 * i + 2] * L[6 + j]);
            acc += dl * R[3 * i + j];
            dR[3 * i + j] = dl * se[j];
        }
        out.scales[3 * o + j] = in.smod * acc;
    }
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    out.rots[4 * o + 0] = 2.f * (-z * dR[1] + y * dR[2] + z * dR[3] - x * dR[5] - y * dR[6] + x * dR[7]);
    out.rots[4 * o + 1] = 2.f * (y * dR[1] + z * dR[2] + y * dR[3] - 2.f * x * dR[4] - r * dR[5] + z * dR[6] + r * dR[7] - 2.f * x * dR[8]);
    out.rots[4 * o + 2] = 2.f * (-2.f * y * dR[0] + x * dR[1] + r * dR[2] + x * dR[3] + z * dR[5] - r * dR[6] + z * dR[7] - 2.f * y * dR[8]);
    out.rots[4 * o + 3] = 2.f * (-2.f * z * dR[0] - r * dR[1] + x * dR[2] + r * dR[3] - 2.f * z * dR[4] + y * dR[5] + x * dR[6] + y * dR[7]);
}

#ifndef GSR_B2_VEC4
#define GSR_B2_VEC4 1
#endif

// Gaussians [g0, g0 + n): inputs indexed by g, grad2d and every output by o = g - g0.
// view v's leaf outputs: `out` for v = 0, slice v - 1 of `scratch`; its 2D gradients: rows v * P..
__device__ __forceinline__ GradOut view_out(const GradOut& out, const GradOut& scratch, int v, size_t P, int M3) {
    if (v == 0) return out;
    const size_t k = (size_t)(v - 1) * P;
    auto sl = [&](float* p, int width) { return p ? p + k * width : nullptr; };
    GradOut o;
    o.means2D = out.means2D ? out.means2D + (size_t)v * P * 3 : nullptr;
    o.conic = out.conic ? out.conic + (size_t)v * P * 3 : nullptr;
    o.opac = sl(scratch.opac, 1);
    o.colors = sl(scratch.colors, 3);
    o.means3D = sl(scratch.means3D, 3);
    o.sh_dc = sl(scratch.sh_dc, 3);
    o.sh_rest = sl(scratch.sh_rest, M3);
    o.scales = sl(scratch.scales, 3);
    o.rots = sl(scratch.rots, 4);
    o.cov3D = sl(scratch.cov3D, 6);
    return o;
}

// SUM: the 2D gradients are the shard's band returns (BandSum), summed here (g0 = 0).
template <int NV, bool SUM>
__global__ __launch_bounds__(256) void preprocess_backward_kernel(
    const CamArg<NV> cams, const GaussIn in, int g0, int n, const uint32_t* __restrict__ depth_key,
    const uint32_t* __restrict__ flags, const float* __restrict__ grad2d, GradOut out, const GradOut scratch,
    const BandSum bs) {
    extern __shared__ __attribute__((aligned(16))) float sh_lds[];
    const int o = blockIdx.x * 256 + threadIdx.x;
    const int M3 = in.M_rest * 3;
    const int view = NV > 1 ? (int)blockIdx.y : 0;
    const gsr_camera& cam = cams.c[NV > 1 ? view : 0];
    if (NV > 1) {  // views mode: this view's entries and outputs
        const size_t e0 = (size_t)view * in.P;
        depth_key += e0;
        if (flags) flags += e0;
        grad2d += e0 * kPart;
        out = view_out(out, scratch, view, (size_t)in.P, M3);
    }
    const bool stage = in.sh_rest != nullptr && !in.colors;  // block-uniform
    const int rows = n - blockIdx.x * 256 < 256 ? n - blockIdx.x * 256 : 256;
    const size_t obase = (size_t)blockIdx.x * 256 * M3, ibase = (size_t)g0 * M3 + obase;
    // 16-B staging when the rows start 16-B aligned (always for g0 = 0: a block's 256 rows are
    // 46080 B); 4-B otherwise
    const bool v4 = GSR_B2_VEC4 && ((reinterpret_cast<uintptr_t>(in.sh_rest + ibase) |
                                     reinterpret_cast<uintptr_t>(out.sh_rest + obase)) & 15u) == 0;
    // Aligned rows are staged by buffer-load-to-LDS DMA: the block's 256 * M3 floats are M3 pieces
    // of 1 KB (64 lanes x 16 B), piece q by wave q % 4, all issued before the per-Gaussian inputs
    // (loads return in order: one wait covers both); the piece offset is in voffset, which the
    // descriptor's range check covers (soffset is not checked), so the rows past n zero-fill.
    if (stage && v4) {
        const auto src = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in.sh_rest + ibase), 0,
                                                           rows * M3 * (int)sizeof(float), 0x00020000);
        const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
        auto* dst = (__attribute__((address_space(3))) char*)sh_lds;
#pragma unroll
        for (int j = 0; j < 12; ++j) {  // M3 <= 45 pieces: <= 12 per wave
            const int q = 4 * j + wu;
            if (q < M3) __builtin_amdgcn_raw_ptr_buffer_load_lds(src, dst + 1024 * q, 16, ln * 16 + 1024 * q, 0, 0, 0);
        }
    }
    BwdIn bi{};
    if (o < n) bi = load_bwd_in<SUM>(in, g0 + o, o, depth_key, flags, grad2d, bs);
    if (stage) {  // coalesced staging of the block's SH-rest rows (see preprocess_kernel)
        if (v4) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces have landed
        } else {
            const int nf = rows * M3;
            for (int i = threadIdx.x; i < nf; i += 256) sh_lds[i] = in.sh_rest[ibase + i];
        }
        __syncthreads();
    }
    if (o < n) preprocess_backward_one(cam, in, g0 + o, o, bi, flags, out, stage ? sh_lds + threadIdx.x * M3 : nullptr);
    if (stage) {  // coalesced write-back of the SH-rest gradient rows
        __syncthreads();
        const int nf = rows * M3;
        if (v4) {
            float4* dst = reinterpret_cast<float4*>(out.sh_rest + obase);
            for (int i = threadIdx.x; i < nf / 4; i += 256) dst[i] = reinterpret_cast<const float4*>(sh_lds)[i];
            for (int i = (nf & ~3) + threadIdx.x; i < nf; i += 256) out.sh_rest[obase + i] = sh_lds[i];
        } else {
            for (int i = threadIdx.x; i < nf; i += 256) out.sh_rest[obase + i] = sh_lds[i];
        }
    }
}

}  // namespace

int launch_gather_grad2d(const uint32_t* offsets, const float* partial, const float4* rec, int W, int H,
                         long long cap, int P, const uint4* rrect, float* grad2d, hipStream_t s, int split) {
    if (P <= 0) return 0;
    const PartLayout pl(cap * split);
    const char* base = reinterpret_cast<const char*>(partial);
    hipLaunchKernelGGL(gather_grad2d_kernel, dim3(div_up(P, 256)), dim3(256), 0, s, offsets,
                       reinterpret_cast<const float4*>(base + pl.p8), reinterpret_cast<const float*>(base + pl.p1),
                       reinterpret_cast<const uint8_t*>(base + pl.fl), rec, 0.5f * (float)W, 0.5f * (float)H, P,
                       (uint32_t)cap, rrect, grad2d, (uint32_t)split);
    return (int)hipGetLastError();
}

int launch_preprocess_backward(const gsr_camera& cam, const GaussIn& in, int g0, int g1,
                               const uint32_t* depth_key, const uint32_t* flags, const float* grad2d,
                               const GradOut& out, hipStream_t s) {
    const int n = g1 - g0;
    if (n <= 0) return 0;
    const size_t lds = (in.sh_rest && !in.colors) ? sizeof(float) * 256 * 3 * in.M_rest : 0;
    const CamArg<1> c1{{cam}};
    hipLaunchKernelGGL((preprocess_backward_kernel<1, false>), dim3(div_up(n, 256)), dim3(256), lds, s, c1, in, g0,
                       n, depth_key, flags, grad2d, out, GradOut{}, BandSum{});
    return (int)hipGetLastError();
}

int launch_preprocess_backward_banded(const gsr_camera& cam, const GaussIn& in, const uint32_t* depth_key,
                                      const uint32_t* flags, const BandSum& bs, const GradOut& out, hipStream_t s) {
    if (in.P <= 0) return 0;
    const size_t lds = (in.sh_rest && !in.colors) ? sizeof(float) * 256 * 3 * in.M_rest : 0;
    const CamArg<1> c1{{cam}};
    hipLaunchKernelGGL((preprocess_backward_kernel<1, true>), dim3(div_up(in.P, 256)), dim3(256), lds, s, c1, in, 0,
                       in.P, depth_key, flags, nullptr, out, GradOut{}, bs);
    return (int)hipGetLastError();
}

int launch_preprocess_backward_views(const gsr_camera* cams, int V, const GaussIn& in, const uint32_t* depth_key,
                                     const uint32_t* flags, const float* grad2d, const GradOut& out,
                                     const GradOut& scratch, hipStream_t s) {
    if (in.P <= 0 || V <= 0) return 0;
    if (V > kMaxViews) return -1;
    CamArg<kMaxViews> cv{};
    for (int v = 0; v < V; ++v) cv.c[v] = cams[v];
    const size_t lds = (in.sh_rest && !in.colors) ? sizeof(float) * 256 * 3 * in.M_rest : 0;
    hipLaunchKernelGGL((preprocess_backward_kernel<kMaxViews, false>), dim3(div_up(in.P, 256), V), dim3(256), lds, s,
                       cv, in, 0, in.P, depth_key, flags, grad2d, out, scratch, BandSum{});
    return (int)hipGetLastError();
}

// out[i] = ((out[i] + s_1[i]) + s_2[i]) + ... over the views' leaf-gradient slices, in view order
// (the same sum a caller forms from per-view backward calls).  blockIdx.y = output array.
struct SumArrays {
    float* dst[8];
    const float* src[8];
    long long n[8];
};
__global__ __launch_bounds__(256) void views_sum_kernel(const SumArrays a, int V) {
    const int k = blockIdx.y;
    float* d = a.dst[k];
    if (!d) return;
    const long long n = a.n[k];
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        float acc = d[i];
        for (int v = 0; v + 1 < V; ++v) acc = acc + a.src[k][(size_t)v * n + i];
        d[i] = acc;
    }
}

int launch_views_sum(const GaussIn& in, int V, const GradOut& out, const GradOut& scratch, hipStream_t s) {
    if (in.P <= 0 || V <= 1) return 0;
    SumArrays a{};
    const long long P = in.P;
    float* const dsts[8] = {out.opac, out.colors, out.means3D, out.sh_dc, out.sh_rest, out.scales, out.rots, out.cov3D};
    const float* const srcs[8] = {scratch.opac, scratch.colors, scratch.means3D, scratch.sh_dc, scratch.sh_rest,
                                  scratch.scales, scratch.rots, scratch.cov3D};
    const long long widths[8] = {1, 3, 3, 3, 3LL * in.M_rest, 3, 4, 6};
    long long nmax = 0;
    for (int k = 0; k < 8; ++k) {
        const bool on = dsts[k] && srcs[k] && widths[k] > 0;
        a.dst[k] = on ? dsts[k] : nullptr;
        a.src[k] = on ? srcs[k] : nullptr;
        a.n[k] = on ? P * widths[k] : 0;
        nmax = a.n[k] > nmax ? a.n[k] : nmax;
    }
    if (nmax == 0) return 0;
    const long long blocks = div_up(nmax, 256) < 4096 ? div_up(nmax, 256) : 4096;
    hipLaunchKernelGGL(views_sum_kernel, dim3((unsigned)blocks, 8), dim3(256), 0, s, a, V);
    return (int)hipGetLastError();
}

}  // namespace gsr

// gsr_preprocess.hip -- F1: per-Gaussian projection / EWA covariance / conic / radius /
// tile rect / SH->RGB on gfx950.
//
// Compiled with -ffp-contract=off (see __graft_entry__.build): every float that feeds a tile
// key (view z, projected xy, cov2D, radius) is produced by the same IEEE ops in the same
// order as the CPU oracle (oracle/gsr_oracle.c preprocess_one), so tile ids, depth bits and
// the sort order are bit-exact.  sqrtf / division are correctly rounded under
// hipcc's defaults (no fast-math).
//
// Reference anchors: quaternion layout (w,x,y,z) src/utils/general_utils.cpp:24-37;
// L = R diag(s) :91-97; Sigma = L L^T src/scene/gaussian_model.cpp:23-24; activated inputs
// gaussian_model.cpp:270-298; camera matrices src/scene/camera.cpp:66-71.
//
// Roofline: HBM-bound.  Algorithmic bytes per Gaussian: 44 B params + 12*M B SH (visible
// only) in; radius, depth key, tiles (12 B) + 48 B record + 16 B rect out.
// For a band (multi-GPU) only the band's candidates evaluate SH and write records.
#include <cstdlib>

#include "gsr_kernels.h"

namespace gsr {
namespace {

__constant__ float kSH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                                -1.0925484305920792f, 0.5462742152960396f};
__constant__ float kSH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                                0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                                -0.5900435899266435f};
constexpr float kSH_C0 = 0.28209479177387814f;
constexpr float kSH_C1 = 0.4886025119029199f;

__device__ inline int imin(int a, int b) { return a < b ? a : b; }
__device__ inline int imax(int a, int b) { return a > b ? a : b; }

// Geometry of one Gaussian (everything but its colour): radius, depth key, band-clipped
// tiles_touched and what the blend record needs.
struct Geo {
    float xs, ys, cA, cB, cC, a, c;
    int minx, miny, maxx, maxy;
    int32_t radius;
    uint32_t key, tiles;
};

// Per-Gaussian inputs, all loaded up front so their HBM latencies overlap (a load issued
// only after tz > 0.2 is known would add a second round trip per wave).
struct Params {
    float p0, p1, p2;
    float4 q;          // rotation (w, x, y, z), or cov3D[0..3]
    float s0, s1, s2;  // scales, or cov3D[4..5]
    float opac;
    float c0, c1, c2;  // sh_dc, or precomputed colours
};

__device__ __forceinline__ Params load_params(const GaussIn& in, int g) {
    Params P;
    P.p0 = in.means3D[3 * g + 0];
    P.p1 = in.means3D[3 * g + 1];
    P.p2 = in.means3D[3 * g + 2];
    if (in.cov3D) {
        P.q = make_float4(in.cov3D[6 * g + 0], in.cov3D[6 * g + 1], in.cov3D[6 * g + 2], in.cov3D[6 * g + 3]);
        P.s0 = in.cov3D[6 * g + 4];
        P.s1 = in.cov3D[6 * g + 5];
        P.s2 = 0.0f;
    } else {
        P.q = *reinterpret_cast<const float4*>(in.rots + 4 * g);
        P.s0 = in.scales[3 * g + 0];
        P.s1 = in.scales[3 * g + 1];
        P.s2 = in.scales[3 * g + 2];
    }
    P.opac = in.opac[g];
    const float* c = in.colors ? in.colors : in.sh_dc;
    P.c0 = c[3 * g + 0];
    P.c1 = c[3 * g + 1];
    P.c2 = c[3 * g + 2];
    return P;
}

__device__ __forceinline__ Geo preprocess_geom(const gsr_camera& cam, const GaussIn& in, const Params& I, int grid_x,
                                               int grid_y, int ty0, int ty1) {
    const float* V = cam.viewmatrix;
    const float* Pm = cam.projmatrix;
    const float p0 = I.p0, p1 = I.p1, p2 = I.p2;
    Geo G{};
    G.key = 0xFFFFFFFFu;

    const float tx = V[0] * p0 + V[4] * p1 + V[8] * p2 + V[12];
    const float ty = V[1] * p0 + V[5] * p1 + V[9] * p2 + V[13];
    const float tz = V[2] * p0 + V[6] * p1 + V[10] * p2 + V[14];
    if (tz > 0.2f) {
        const float hx = Pm[0] * p0 + Pm[4] * p1 + Pm[8] * p2 + Pm[12];
        const float hy = Pm[1] * p0 + Pm[5] * p1 + Pm[9] * p2 + Pm[13];
        const float hw = Pm[3] * p0 + Pm[7] * p1 + Pm[11] * p2 + Pm[15];
        const float pw = 1.0f / (hw + 0.0000001f);
        const float px = hx * pw, py = hy * pw;
        float c3[6];
        if (in.cov3D) {
            c3[0] = I.q.x;
            c3[1] = I.q.y;
            c3[2] = I.q.z;
            c3[3] = I.q.w;
            c3[4] = I.s0;
            c3[5] = I.s1;
        } else {
            const float r = I.q.x, x = I.q.y, y = I.q.z, z = I.q.w;
            float R[9];
            R[0] = 1.f - 2.f * (y * y + z * z);
            R[1] = 2.f * (x * y - r * z);
            R[2] = 2.f * (x * z + r * y);
            R[3] = 2.f * (x * y + r * z);
            R[4] = 1.f - 2.f * (x * x + z * z);
            R[5] = 2.f * (y * z - r * x);
            R[6] = 2.f * (x * z - r * y);
            R[7] = 2.f * (y * z + r * x);
            R[8] = 1.f - 2.f * (x * x + y * y);
            const float sx = in.smod * I.s0;
            const float sy = in.smod * I.s1;
            const float sz = in.smod * I.s2;
            float L[9];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                L[3 * i + 0] = R[3 * i + 0] * sx;
                L[3 * i + 1] = R[3 * i + 1] * sy;
                L[3 * i + 2] = R[3 * i + 2] * sz;
            }
#define SIG(i, j) (L[3 * (i) + 0] * L[3 * (j) + 0] + L[3 * (i) + 1] * L[3 * (j) + 1] + L[3 * (i) + 2] * L[3 * (j) + 2])
            c3[0] = SIG(0, 0);
            c3[1] = SIG(0, 1);
            c3[2] = SIG(0, 2);
            c3[3] = SIG(1, 1);
            c3[4] = SIG(1, 2);
            c3[5] = SIG(2, 2);
#undef SIG
        }
        const float Wf = (float)cam.width, Hf = (float)cam.height;
        const float fx = Wf / (2.0f * cam.tanfovx);
        const float fy = Hf / (2.0f * cam.tanfovy);
        const float limx = 1.3f * cam.tanfovx, limy = 1.3f * cam.tanfovy;
        const float txtz = tx / tz, tytz = ty / tz;
        const float cx = fminf(limx, fmaxf(-limx, txtz)) * tz;
        const float cy = fminf(limy, fmaxf(-limy, tytz)) * tz;
        const float tz2 = tz * tz;
        const float J00 = fx / tz, J02 = -(fx * cx) / tz2;
        const float J11 = fy / tz, J12 = -(fy * cy) / tz2;
        float T0[3], T1[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            T0[k] = J00 * V[4 * k + 0] + J02 * V[4 * k + 2];
            T1[k] = J11 * V[4 * k + 1] + J12 * V[4 * k + 2];
        }
        const float S[9] = {c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]};
        float U0[3], U1[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            U0[j] = T0[0] * S[0 + j] + T0[1] * S[3 + j] + T0[2] * S[6 + j];
            U1[j] = T1[0] * S[0 + j] + T1[1] * S[3 + j] + T1[2] * S[6 + j];
        }
        const float a = (U0[0] * T0[0] + U0[1] * T0[1] + U0[2] * T0[2]) + 0.3f;
        const float b = U0[0] * T1[0] + U0[1] * T1[1] + U0[2] * T1[2];
        const float c = (U1[0] * T1[0] + U1[1] * T1[1] + U1[2] * T1[2]) + 0.3f;
        const float det = a * c - b * b;
        if (det != 0.0f) {
            const float det_inv = 1.0f / det;
            const float cA = c * det_inv, cB = -b * det_inv, cC = a * det_inv;
            const float mid = 0.5f * (a + c);
            const float disc = fmaxf(0.1f, mid * mid - det);
            const float sq = sqrtf(disc);
            const float l1 = mid + sq, l2 = mid - sq;
            const int radius = (int)ceilf(3.0f * sqrtf(fmaxf(l1, l2)));
            const float xs = ((px + 1.0f) * Wf - 1.0f) * 0.5f;
            const float ys = ((py + 1.0f) * Hf - 1.0f) * 0.5f;
            const float rf = (float)radius;
            const int minx = imin(grid_x, imax(0, (int)((xs - rf) / (float)kTile)));
            const int miny = imin(grid_y, imax(0, (int)((ys - rf) / (float)kTile)));
            const int maxx = imin(grid_x, imax(0, (int)((xs + rf + (float)(kTile - 1)) / (float)kTile)));
            const int maxy = imin(grid_y, imax(0, (int)((ys + rf + (float)(kTile - 1)) / (float)kTile)));
            const int by0 = imax(miny, ty0), by1 = imin(maxy, ty1);
            const int band_rows = by1 > by0 ? by1 - by0 : 0;
            if ((maxx - minx) * (maxy - miny) != 0) {
                G.radius = radius;
                G.key = __float_as_uint(tz);
                G.tiles = (uint32_t)((maxx - minx) * band_rows);
            }
            G.xs = xs;
            G.ys = ys;
            G.cA = cA;
            G.cB = cB;
            G.cC = cC;
            G.a = a;
            G.c = c;
            G.minx = minx;
            G.miny = miny;
            G.maxx = maxx;
            G.maxy = maxy;
        }
    }
    return G;
}

// Real SH basis (degree <= 3) of the unit view direction of Gaussian g.
__device__ __forceinline__ void sh_basis(const gsr_camera& cam, const GaussIn& in, const Params& I,
                                         float (&basis)[16]) {
    const float dx = I.p0 - cam.campos[0], dy = I.p1 - cam.campos[1], dz = I.p2 - cam.campos[2];
    const float len = sqrtf(dx * dx + dy * dy + dz * dz);
    const float x = dx / len, y = dy / len, z = dz / len;
    const int D = in.D;
#pragma unroll
    for (int k = 0; k < 16; ++k) basis[k] = 0.0f;
    basis[0] = kSH_C0;
    if (D >= 1) {
        basis[1] = -kSH_C1 * y;
        basis[2] = kSH_C1 * z;
        basis[3] = -kSH_C1 * x;
    }
    if (D >= 2) {
        const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        basis[4] = kSH_C2[0] * xy;
        basis[5] = kSH_C2[1] * yz;
        basis[6] = kSH_C2[2] * (2.0f * zz - xx - yy);
        basis[7] = kSH_C2[3] * xz;
        basis[8] = kSH_C2[4] * (xx - yy);
        if (D >= 3) {
            basis[9] = kSH_C3[0] * y * (3.0f * xx - yy);
            basis[10] = kSH_C3[1] * xy * z;
            basis[11] = kSH_C3[2] * y * (4.0f * zz - xx - yy);
            basis[12] = kSH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
            basis[13] = kSH_C3[4] * x * (4.0f * zz - xx - yy);
            basis[14] = kSH_C3[5] * z * (xx - yy);
            basis[15] = kSH_C3[6] * x * (xx - 3.0f * yy);
        }
    }
}

// Blend record (SURVEY B.3 power with -0.5 and log2(e) folded in, so the blend evaluates exp2
// directly; log2(o) rides along so o * G is one exp2) + the half-extents of the alpha >= 1/255
// footprint: d^T Q d <= t, t = 2 ln(255 o)  =>  |dx| <= sqrt(t a), |dy| <= sqrt(t c), padded
// (x1.02 + 0.5 px) so the per-stripe cull never drops a contributing pixel.
__device__ __forceinline__ void write_record(size_t g, float opac, const Geo& G, const float (&rgb)[3],
                                             uint32_t clamped, const PreOut& out) {
    const float kL2E = 1.4426950408889634f;
    const float tthr = 2.0f * logf(255.0f * opac);
    const float ex = tthr > 0.0f ? sqrtf(tthr * G.a) * 1.02f + 0.5f : -1.0f;
    const float ey = tthr > 0.0f ? sqrtf(tthr * G.c) * 1.02f + 0.5f : -1.0f;
    float4* rec = out.rec + 3 * (size_t)g;
    rec[0] = make_float4(G.xs, G.ys, -0.5f * kL2E * G.cA, -kL2E * G.cB);
    rec[1] = make_float4(-0.5f * kL2E * G.cC, opac, rgb[0], rgb[1]);
    rec[2] = make_float4(rgb[2], ex, ey, log2f(opac));
    out.rect[g] = make_uint4((uint32_t)G.minx | ((uint32_t)G.miny << 16), (uint32_t)G.maxx | ((uint32_t)G.maxy << 16),
                             0u, 0u);
    if (out.flags) out.flags[g] = clamped;
}

// SH rows (M_rest x 3 floats per Gaussian, contiguous) reach the lanes in one of two ways:
//  kShDirect : each lane reads its own row from HBM (used only when there are no SH rows);
//  kShChunks : the block stages 5-coefficient column chunks (15 floats per row, 15 KB of LDS)
//              and accumulates the colour chunk by chunk in the same k order (bit-identical
//              to one pass), with 8 waves per SIMD.
// Measured at 1M/SH3: direct 0.53 ms -- each lane's 180-B row at a 180-B lane stride touches
// ~90 cache lines per load instruction; whole rows staged in LDS (46 KB, 3 waves per SIMD)
// 0.106 ms; chunks 0.082 ms.
//  kShWave   : wave w's 64 rows are one contiguous, 16-B aligned span; it stages them 16 rows at
//              a time with 16-B buffer loads (3 per lane at SH3) into a wave-private LDS window
//              (16 rows: 2.9 KB per wave at SH3) -- every cache line is read once, with a quarter
//              of the load instructions and no block barrier -- and the 16 lanes owning those
//              rows accumulate them (same k order: bit-identical).
//  kShGlds   : wave w's whole 64-row span goes to a wave-private LDS region at kernel start by
//              buffer-load-to-LDS DMA (16 B per lane, no VGPRs; the descriptor's range check
//              zero-fills past the block's rows), overlapping the geometry; each lane then reads
//              its own row (180-B stride: conflict-free) in the same k order.  One HBM round trip
//              per wave instead of one per window, at 12 KB of LDS per wave (3 waves per SIMD).
enum { kShDirect = 0, kShChunks = 2, kShWave = 3, kShGlds = 4 };
constexpr int kChunkK = 5;               // SH coefficients per staged chunk
constexpr int kChunkF = 3 * kChunkK;     // floats per row per chunk
constexpr int kSubRows = 16;             // kShWave: rows per staged window
#ifndef GSR_F1_SH_MODE
#define GSR_F1_SH_MODE kShGlds
#endif

// The block also adds its candidate count (Gaussians with tiles in the band) and instance
// count (sum of tiles_touched) into counters[slot] / counters[kCountSlots + slot], so the host
// can read K right after this kernel -- while the depth sort runs -- instead of after the scan.
//
// NV > 1 (gsr_forward_views): view v = blockIdx.y projects the same Gaussians with cams.c[v]; its
// outputs go to entry e = v * P + g and its tile rows are offset by v * grid_y -- the views are
// consecutive bands of tile rows of one tall image for every later stage.
template <int SH, int NV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void preprocess_kernel(const CamArg<NV> cams,
                                                         const GaussIn in,
                                                         int grid_x, int grid_y, int ty0, int ty1,
                                                         PreOut out) {
    extern __shared__ __attribute__((aligned(16))) float sh_lds[];
    __shared__ uint32_t wk[4], wc[4];
    const int view = NV > 1 ? (int)blockIdx.y : 0;
    const gsr_camera& cam = cams.c[NV > 1 ? view : 0];
    const int g = blockIdx.x * 256 + threadIdx.x;
    const size_t e = (size_t)view * in.P + g;  // output entry
    const int M3 = in.M_rest * 3;
    const int rows = in.P - blockIdx.x * 256 < 256 ? in.P - blockIdx.x * 256 : 256;
    const bool sh = in.sh_rest && !in.colors && in.D > 0;  // grid-uniform
    // kShChunks: lane (r0, col) moves column f0 + col of rows r0, r0 + 16, ...; chunk c + 1 is
    // loaded into registers while chunk c is consumed, and chunk 0 while the geometry runs.
    const int col = threadIdx.x & 15, r0 = threadIdx.x >> 4;
    const size_t base = (size_t)blockIdx.x * 256 * M3;
    const int nb = (in.D + 1) * (in.D + 1);
    // Buffer loads over the block's rows: the whole byte offset goes in the 32-bit lane offset
    // (a raw buffer's range check covers voffset + inst_offset, never soffset), so the
    // descriptor's range check zero-fills rows past the end of the array.
    float pre[16];
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in.sh_rest + base), 0,
                                                        rows * M3 * (int)sizeof(float), 0x00020000);
    auto load_chunk = [&](int c) {
        const int voff = (r0 * M3 + kChunkF * c + col) * (int)sizeof(float);
#pragma unroll
        for (int j = 0; j < 16; ++j)
            pre[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                   rsrc, voff + j * 16 * M3 * (int)sizeof(float), 0, 0));
    };
    // kShWave: this wave's rows [64 w, 64 w + 64) of the block, staged kSubRows at a time
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int sub_f4 = kSubRows * M3 / 4;          // 16-B words per window (16 M3 floats)
    constexpr int kWin = 4;                        // 16-B loads per lane per window (M3 <= 64)
    uint4 win[kWin];
    // the block's rows only (offsets stay 32-bit for any P; rows past the end read as zero)
    const auto wsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in.sh_rest + base), 0,
                                                        rows * M3 * (int)sizeof(float), 0x00020000);
    auto load_window = [&](int sub) {
        const int voff = ((wv * 64 + kSubRows * sub) * M3) * (int)sizeof(float);
#pragma unroll
        for (int q = 0; q < kWin; ++q) {
            const int i = q * 64 + ln;
            win[q] = make_uint4(0u, 0u, 0u, 0u);
            if (i < sub_f4) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(wsrc, voff + 16 * i, 0, 0);
                win[q] = make_uint4(v[0], v[1], v[2], v[3]);
            }
        }
    };
    // kShGlds: wave wv's LDS region (gq KB); the q-th DMA moves bytes [1024 q, 1024 q + 1024) of its
    // span, addressed by voffset alone so that pieces past the block's rows are range-checked
    // (zero-filled, never read).  Issued before the parameter loads: loads return in order, so
    // one wait covers both
    const int gq = (64 * M3 * 4 + 1023) / 1024;
    if (SH == kShGlds && sh) {
        const int wu = __builtin_amdgcn_readfirstlane(wv);
        auto* dst = (__attribute__((address_space(3))) char*)(sh_lds + wu * gq * 256);
        const int wbase = wu * 64 * M3 * 4;
#pragma unroll
        for (int q = 0; q < 12; ++q)
            if (q < gq)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(wsrc, dst + 1024 * q, 16, ln * 16 + wbase + 1024 * q, 0, 0, 0);
    }
    Params I{};
    if (g < in.P) I = load_params(in, g);
    if (SH == kShChunks && sh) load_chunk(0);
    if (SH == kShWave && sh) load_window(0);
    Geo G{};
    G.key = 0xFFFFFFFFu;
    if (g < in.P) {
        G = preprocess_geom(cam, in, I, grid_x, grid_y, ty0, ty1);
        if (NV > 1) {  // view v's band of tile rows in the tall image (the record stays in the
            G.miny += view * grid_y;  // view's own pixel coordinates: F6 / B1 take pixel y
            G.maxy += view * grid_y;  // relative to the view's band, so every value is bit-equal
        }                             // to a one-view render)
        out.radii[e] = G.radius;
        out.depth_key[e] = G.key;
        out.tiles[e] = G.tiles;
    }
    const bool need = G.tiles != 0;  // colour and record only for Gaussians this band blends
    float rgb[3] = {0.f, 0.f, 0.f}, basis[16];
    if (need) {
        rgb[0] = I.c0;
        rgb[1] = I.c1;
        rgb[2] = I.c2;
        if (!in.colors) {
            sh_basis(cam, in, I, basis);
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) rgb[ch] = basis[0] * rgb[ch];
        }
    }
    if (sh) {
        if (SH == kShGlds) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMAs have landed
            if (need) {
                const float* rest = sh_lds + wv * gq * 256 + ln * M3;
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    float r = rgb[ch];
#pragma unroll
                    for (int k = 1; k < 16; ++k)
                        if (k < nb) r = r + basis[k] * rest[3 * (k - 1) + ch];
                    rgb[ch] = r;
                }
            }
        } else if (SH == kShWave) {
            // wave-private window: wave wv's kSubRows x M3 floats
            float* const wnd = sh_lds + wv * kSubRows * M3;
            for (int sub = 0; sub < 64 / kSubRows; ++sub) {
                if (sub > 0) {  // the lanes of the previous window have read it
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
#pragma unroll
                for (int q = 0; q < kWin; ++q) {
                    const int i = q * 64 + ln;
                    if (i < sub_f4) *reinterpret_cast<uint4*>(wnd + 4 * i) = win[q];
                }
                if (sub + 1 < 64 / kSubRows) load_window(sub + 1);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (need && (ln >> 4) == sub) {
                    const float* rest = wnd + (ln & 15) * M3;
#pragma unroll
                    for (int ch = 0; ch < 3; ++ch) {
                        float r = rgb[ch];
#pragma unroll
                        for (int k = 1; k < 16; ++k)
                            if (k < nb) r = r + basis[k] * rest[3 * (k - 1) + ch];
                        rgb[ch] = r;
                    }
                }
            }
        } else if (SH == kShChunks) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {  // k = 1 + 5c .. 5 + 5c; SH degree <= 3 => k < 16
                const int k0 = 1 + kChunkK * c;
                if (k0 >= nb) break;  // grid-uniform
                if (c > 0) __syncthreads();  // the previous chunk has been consumed
                if (col < kChunkF)
#pragma unroll
                    for (int j = 0; j < 16; ++j) sh_lds[(r0 + 16 * j) * kChunkF + col] = pre[j];
                if (c < 2 && k0 + kChunkK < nb) load_chunk(c + 1);
                __syncthreads();
                if (need) {
                    const float* rest = sh_lds + threadIdx.x * kChunkF;
#pragma unroll
                    for (int kk = 0; kk < kChunkK; ++kk) {
                        const int k = k0 + kk;
                        if (k < nb)
#pragma unroll
                            for (int ch = 0; ch < 3; ++ch) rgb[ch] = rgb[ch] + basis[k] * rest[3 * kk + ch];
                    }
                }
            }
        } else if (need) {
            const float* rest = in.sh_rest + (size_t)g * M3;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                float r = rgb[ch];
#pragma unroll
                for (int k = 1; k < 16; ++k)
                    if (k < nb) r = r + basis[k] * rest[3 * (k - 1) + ch];
                rgb[ch] = r;
            }
        }
    }
    if (need) {
        uint32_t clamped = 0;
        if (!in.colors) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                const float r = rgb[ch] + 0.5f;
                clamped |= (r < 0.0f ? 1u : 0u) << ch;
                rgb[ch] = fmaxf(r, 0.0f);
            }
        }
        write_record(e, I.opac, G, rgb, clamped, out);
    }
    const uint32_t t = G.tiles;
    if (NV == 1 && out.rb_hist) {  // grid-uniform: the row-bucketed binning's per-block row counts
        __shared__ uint32_t rbc[kRbMaxRows];
        rbc[threadIdx.x] = 0u;
        __syncthreads();
        if (t) {
            const int by0 = G.miny > ty0 ? G.miny : ty0, by1 = G.maxy < ty1 ? G.maxy : ty1;
            for (int r = by0; r < by1; ++r) atomicAdd(&rbc[r - ty0], 1u);
        }
        __syncthreads();
        if ((int)threadIdx.x < ty1 - ty0) out.rb_hist[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = rbc[threadIdx.x];
    }
    if (out.counters) {
        uint32_t k = t, c = t ? 1u : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            k += __shfl_xor(k, o, 64);
            c += __shfl_xor(c, o, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            wk[threadIdx.x >> 6] = k;
            wc[threadIdx.x >> 6] = c;
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // spread over kCountSlots addresses: one hot word serialises
            const uint32_t K = wk[0] + wk[1] + wk[2] + wk[3], C = wc[0] + wc[1] + wc[2] + wc[3];
            if (NV == 1 && out.bsum) out.bsum[blockIdx.x] = K;  // the F2 scan's block partial
            const int slot = blockIdx.x & (kCountSlots - 1);
            if (K) atomicAdd(out.counters + kCountSlots + slot, K);
            if (C) atomicAdd(out.counters + slot, C);
        }
    }
}

}  // namespace

template <int NV>
static void launch_preprocess_nv(const CamArg<NV>& cams, int V, const GaussIn& in, int ty0, int ty1,
                                 const PreOut& out, hipStream_t s) {
    const int gx = div_up(cams.c[0].width, kTile), gy = div_up(cams.c[0].height, kTile);
    const bool sh = in.sh_rest && !in.colors && in.D > 0;
    const dim3 grid(div_up(in.P, 256), V), block(256);
    if (sh && GSR_F1_SH_MODE == kShGlds && in.M_rest * 3 <= 48 && (reinterpret_cast<uintptr_t>(in.sh_rest) & 15) == 0)
        hipLaunchKernelGGL((preprocess_kernel<kShGlds, NV>), grid, block,
                           4 * 1024 * ((64 * in.M_rest * 3 * 4 + 1023) / 1024), s, cams, in, gx, gy, ty0, ty1, out);
    else if (sh && GSR_F1_SH_MODE == kShWave && in.M_rest * 3 <= 64 && (reinterpret_cast<uintptr_t>(in.sh_rest) & 15) == 0)
        hipLaunchKernelGGL((preprocess_kernel<kShWave, NV>), grid, block, sizeof(float) * 4 * kSubRows * in.M_rest * 3,
                           s, cams, in, gx, gy, ty0, ty1, out);
    else if (sh)
        hipLaunchKernelGGL((preprocess_kernel<kShChunks, NV>), grid, block, sizeof(float) * 256 * kChunkF, s, cams, in,
                           gx, gy, ty0, ty1, out);
    else
        hipLaunchKernelGGL((preprocess_kernel<kShDirect, NV>), grid, block, 0, s, cams, in, gx, gy, ty0, ty1, out);
}

int launch_preprocess(const gsr_camera& cam, const GaussIn& in, int ty0, int ty1, const PreOut& out,
                      hipStream_t s) {
    if (in.P <= 0) return 0;
    CamArg<1> c1{{cam}};
    launch_preprocess_nv(c1, 1, in, ty0, ty1, out, s);
    return (int)hipGetLastError();
}

int launch_preprocess_views(const gsr_camera* cams, int V, const GaussIn& in, const PreOut& out, hipStream_t s) {
    if (in.P <= 0 || V <= 0) return 0;
    if (V > kMaxViews) return -1;
    CamArg<kMaxViews> cv{};
    for (int v = 0; v < V; ++v) cv.c[v] = cams[v];
    const int gy = div_up(cams[0].height, kTile);
    launch_preprocess_nv(cv, V, in, 0, gy, out, s);
    return (int)hipGetLastError();
}

}  // namespace gsr

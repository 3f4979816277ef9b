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

// The block's SH-rest rows (256 Gaussians x M_rest x 3 floats, contiguous in HBM) are staged
// through LDS with coalesced dword loads: read straight from HBM, each lane's 180-B row at a
// 180-B lane stride would touch ~90 cache lines per load instruction and thrash L1.
// One Gaussian; returns its band-clipped tiles_touched.
__device__ __forceinline__ uint32_t preprocess_one(const gsr_camera& cam, const GaussIn& in, int g, int grid_x,
                                                   int grid_y, int ty0, int ty1, const PreOut& out,
                                                   const float* sh_lds) {
    const int M3 = in.M_rest * 3;
    const float* V = cam.viewmatrix;
    const float* Pm = cam.projmatrix;
    const float p0 = in.means3D[3 * g + 0], p1 = in.means3D[3 * g + 1], p2 = in.means3D[3 * g + 2];
    int32_t radius_out = 0;
    uint32_t key_out = 0xFFFFFFFFu, tiles_out = 0;

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
#pragma unroll
            for (int k = 0; k < 6; ++k) c3[k] = in.cov3D[6 * g + k];
        } else {
            const float4 q = *reinterpret_cast<const float4*>(in.rots + 4 * g);
            const float r = q.x, x = q.y, y = q.z, z = q.w;
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
            const float sx = in.smod * in.scales[3 * g + 0];
            const float sy = in.smod * in.scales[3 * g + 1];
            const float sz = in.smod * in.scales[3 * g + 2];
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
                radius_out = radius;
                key_out = __float_as_uint(tz);
                tiles_out = (uint32_t)((maxx - minx) * band_rows);
            }
            // colour and blend record only for Gaussians this band blends (all visible ones
            // for a full image); B2 recomputes the clamp bits itself
            if (tiles_out != 0) {
                float rgb[3];
                uint32_t clamped = 0;
                if (in.colors) {
                    rgb[0] = in.colors[3 * g + 0];
                    rgb[1] = in.colors[3 * g + 1];
                    rgb[2] = in.colors[3 * g + 2];
                } else {
                    const float dx = p0 - cam.campos[0], dy = p1 - cam.campos[1], dz = p2 - cam.campos[2];
                    const float len = sqrtf(dx * dx + dy * dy + dz * dz);
                    const float x = dx / len, y = dy / len, z = dz / len;
                    float basis[16];
                    const int D = in.D;
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
                    const int nb = (D + 1) * (D + 1);
                    // LDS-staged row (full image) or this Gaussian's own row in HBM (band:
                    // only ~1/N of the rows are needed, so the block does not stage)
                    const float* rest = sh_lds ? sh_lds + threadIdx.x * M3 : in.sh_rest + (size_t)g * M3;
#pragma unroll
                    for (int ch = 0; ch < 3; ++ch) {
                        float r = basis[0] * in.sh_dc[3 * g + ch];
#pragma unroll
                        for (int k = 1; k < 16; ++k)
                            if (k < nb) r = r + basis[k] * rest[3 * (k - 1) + ch];
                        r = r + 0.5f;
                        clamped |= (r < 0.0f ? 1u : 0u) << ch;
                        rgb[ch] = fmaxf(r, 0.0f);
                    }
                }
                // Blend record (SURVEY B.3 power with -0.5 and log2(e) folded in, so the blend
                // evaluates exp2 directly; log2(o) rides along so o * G is one exp2) + the
                // half-extents of the alpha >= 1/255 footprint:
                // d^T Q d <= t, t = 2 ln(255 o)  =>  |dx| <= sqrt(t a), |dy| <= sqrt(t c),
                // padded (x1.02 + 0.5 px) so the per-stripe cull never drops a contributing pixel.
                const float opac = in.opac[g];
                const float kL2E = 1.4426950408889634f;
                const float tthr = 2.0f * logf(255.0f * opac);
                const float ex = tthr > 0.0f ? sqrtf(tthr * a) * 1.02f + 0.5f : -1.0f;
                const float ey = tthr > 0.0f ? sqrtf(tthr * c) * 1.02f + 0.5f : -1.0f;
                float4* rec = out.rec + 3 * (size_t)g;
                rec[0] = make_float4(xs, ys, -0.5f * kL2E * cA, -kL2E * cB);
                rec[1] = make_float4(-0.5f * kL2E * cC, opac, rgb[0], rgb[1]);
                rec[2] = make_float4(rgb[2], ex, ey, log2f(opac));
                out.rect[g] = make_uint4((uint32_t)minx | ((uint32_t)miny << 16),
                                         (uint32_t)maxx | ((uint32_t)maxy << 16), 0u, 0u);
                if (out.flags) out.flags[g] = clamped;
            }
        }
    }
    out.radii[g] = radius_out;
    out.depth_key[g] = key_out;
    out.tiles[g] = tiles_out;
    return tiles_out;
}

// The block's SH-rest rows are staged through LDS (see above).  The block also adds its
// candidate count (Gaussians with tiles in the band) and instance count (sum of
// tiles_touched) into counters[slot] / counters[kCountSlots + slot], so the host can read K
// right after this kernel -- while the depth sort runs -- instead of after the scan.
__global__ __launch_bounds__(256) void preprocess_kernel(const gsr_camera cam, const GaussIn in,
                                                         int grid_x, int grid_y, int ty0, int ty1,
                                                         PreOut out) {
    extern __shared__ __attribute__((aligned(16))) float sh_lds[];
    __shared__ uint32_t wk[4], wc[4];
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int M3 = in.M_rest * 3;
    const bool band = ty0 > 0 || ty1 < grid_y;
    const bool stage = in.sh_rest && !in.colors && in.D > 0 && !band;  // grid-uniform
    if (stage) {
        const size_t base = (size_t)blockIdx.x * 256 * M3;
        const int rows = in.P - blockIdx.x * 256 < 256 ? in.P - blockIdx.x * 256 : 256;
        const int cnt = rows * M3;
        for (int i = threadIdx.x; i < cnt; i += 256) sh_lds[i] = in.sh_rest[base + i];
        __syncthreads();
    }
    const uint32_t t = g < in.P ? preprocess_one(cam, in, g, grid_x, grid_y, ty0, ty1, out, stage ? sh_lds : nullptr)
                                : 0u;
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
            const int slot = blockIdx.x & (kCountSlots - 1);
            if (K) atomicAdd(out.counters + kCountSlots + slot, K);
            if (C) atomicAdd(out.counters + slot, C);
        }
    }
}

}  // namespace

int launch_preprocess(const gsr_camera& cam, const GaussIn& in, int ty0, int ty1, const PreOut& out,
                      hipStream_t s) {
    if (in.P <= 0) return 0;
    const int gx = div_up(cam.width, kTile), gy = div_up(cam.height, kTile);
    const bool band = ty0 > 0 || ty1 < gy;  // a band reads SH rows directly (see preprocess_kernel)
    const size_t lds = (in.sh_rest && !in.colors && in.D > 0 && !band) ? sizeof(float) * 256 * 3 * in.M_rest : 0;
    hipLaunchKernelGGL(preprocess_kernel, dim3(div_up(in.P, 256)), dim3(256), lds, s, cam, in, gx, gy,
                       ty0, ty1, out);
    return (int)hipGetLastError();
}

}  // namespace gsr

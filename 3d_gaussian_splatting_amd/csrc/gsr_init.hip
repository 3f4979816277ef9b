// gsr_init.hip -- Gaussian initialisation from a point cloud on gfx950.
//
// gsr_knn_mean_dist2: for every point, the mean of the squared distances to its 3 nearest
// other points -- the quantity upstream 3DGS's create_from_pcd takes from simple_knn's
// distCUDA2 and turns into the initial isotropic scale log(sqrt(max(d, 1e-7))).  The
// reference (seiya-kumada/3d_gaussian_splatting) has no point-cloud initialisation: its
// points3D / PLY branch is commented out (src/scene/dataset_readers.cpp:198-219).
//
// Exact, not approximate:
//   1. bounding box (ordered-integer atomics), 30-bit Morton code per point over it, and the
//      library's LSD radix sort of the codes -> the points in Morton order, spatially coherent;
//   2. boxes of kBox consecutive sorted points and their AABBs;
//   3. one wave per 64 consecutive sorted points visits every box nearest-first in Morton
//      order (its own box, then +-1, +-2, ...) and scans a box (wave-uniform loads, one point
//      per step) only when some lane's current third-best squared distance exceeds that lane's
//      distance to the box.  Both distances are evaluated without FMA contraction
//      (-ffp-contract=off), and f32 rounding is monotone, so the box distance never exceeds the
//      computed distance to any point inside: a skipped box cannot improve any lane.
// VALU-bound (N / kBox box tests per point); it runs once per scene, not per iteration.
#include <cfloat>

#include "gsr_kernels.h"
#include "../../include/gsr/gsr_train.h"

namespace gsr {
int set_error(int code, const char* msg);

namespace {

constexpr int kBox = 256;  // sorted points per box (= threads per box block)

__device__ __forceinline__ uint32_t f2ord(float f) {  // order-preserving float -> uint
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// bb[0..2] = ordered min (host-filled 0xFF..), bb[3..5] = ordered max (host-zeroed)
__global__ __launch_bounds__(256) void knn_bbox_kernel(const float* __restrict__ pts, int n, uint32_t* __restrict__ bb) {
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float v = pts[3 * (size_t)i + c];
            lo[c] = fminf(lo[c], v);
            hi[c] = fmaxf(hi[c], v);
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lo[c] = fminf(lo[c], __shfl_xor(lo[c], o, 64));
            hi[c] = fmaxf(hi[c], __shfl_xor(hi[c], o, 64));
        }
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            atomicMin(bb + c, f2ord(lo[c]));
            atomicMax(bb + 3 + c, f2ord(hi[c]));
        }
    }
}

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit
    v &= 0x3FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ __launch_bounds__(256) void knn_morton_kernel(const float* __restrict__ pts, int n,
                                                         const uint32_t* __restrict__ bb, uint32_t* __restrict__ code) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t c = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float lo = ord2f(bb[a]), ext = ord2f(bb[3 + a]) - lo;
        float q = ext > 0.0f ? (pts[3 * (size_t)i + a] - lo) / ext * 1023.0f : 0.0f;
        q = fminf(fmaxf(q, 0.0f), 1023.0f);
        c |= spread10((uint32_t)q) << a;
    }
    code[i] = c;
}

// sorted points (x, y, z, original index bits) and the AABB of each box of kBox of them
__global__ __launch_bounds__(kBox) void knn_boxes_kernel(const float* __restrict__ pts,
                                                         const uint32_t* __restrict__ order, int n,
                                                         float4* __restrict__ sp, float4* __restrict__ blo,
                                                         float4* __restrict__ bhi) {
    __shared__ float red[2][3][kBox / 64];
    const int i = blockIdx.x * kBox + threadIdx.x;
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    if (i < n) {
        const uint32_t g = order[i];
        const float x = pts[3 * (size_t)g], y = pts[3 * (size_t)g + 1], z = pts[3 * (size_t)g + 2];
        sp[i] = make_float4(x, y, z, __uint_as_float(g));
        lo[0] = hi[0] = x;
        lo[1] = hi[1] = y;
        lo[2] = hi[2] = z;
    }
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lo[c] = fminf(lo[c], __shfl_xor(lo[c], o, 64));
            hi[c] = fmaxf(hi[c], __shfl_xor(hi[c], o, 64));
        }
        if ((threadIdx.x & 63) == 0) {
            red[0][c][w] = lo[c];
            red[1][c][w] = hi[c];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float L[3], H[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            L[c] = red[0][c][0];
            H[c] = red[1][c][0];
            for (int k = 1; k < kBox / 64; ++k) {
                L[c] = fminf(L[c], red[0][c][k]);
                H[c] = fmaxf(H[c], red[1][c][k]);
            }
        }
        blo[blockIdx.x] = make_float4(L[0], L[1], L[2], 0.0f);
        bhi[blockIdx.x] = make_float4(H[0], H[1], H[2], 0.0f);
    }
}

__device__ __forceinline__ void insert3(float d, float& b0, float& b1, float& b2) {
    if (d < b2) {
        if (d < b1) {
            b2 = b1;
            if (d < b0) {
                b1 = b0;
                b0 = d;
            } else {
                b1 = d;
            }
        } else {
            b2 = d;
        }
    }
}

__global__ __launch_bounds__(256) void knn_kernel(const float4* __restrict__ sp, const float4* __restrict__ blo,
                                                  const float4* __restrict__ bhi, int n, int nbox,
                                                  float* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const bool valid = i < n;
    const float4 p = sp[valid ? i : n - 1];
    const int own = (i & ~63) / kBox;  // the wave's box (wave-uniform)
    float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
    for (int off = 0; off < nbox; ++off) {
        if (own - off < 0 && own + off >= nbox) break;
        for (int side = 0; side < 2; ++side) {
            if (off == 0 && side == 1) break;
            const int q = side ? own - off : own + off;
            if (q < 0 || q >= nbox) continue;
            const float4 lo = blo[q], hi = bhi[q];
            const float dx = fmaxf(fmaxf(lo.x - p.x, p.x - hi.x), 0.0f);
            const float dy = fmaxf(fmaxf(lo.y - p.y, p.y - hi.y), 0.0f);
            const float dz = fmaxf(fmaxf(lo.z - p.z, p.z - hi.z), 0.0f);
            const float db = dx * dx + dy * dy + dz * dz;
            if (!__any(valid && db < b2)) continue;
            const int j1 = (q + 1) * kBox < n ? (q + 1) * kBox : n;
            for (int j = q * kBox; j < j1; ++j) {
                const float4 o = sp[j];  // wave-uniform address
                const float ex = o.x - p.x, ey = o.y - p.y, ez = o.z - p.z;
                const float d = ex * ex + ey * ey + ez * ez;
                if (j != i) insert3(d, b0, b1, b2);
            }
        }
    }
    // fewer than 3 other points: the missing neighbours stay at FLT_MAX, as in the upstream
    // kernel (a huge mean, or +inf when two are missing)
    if (valid) out[__float_as_uint(p.w)] = (b0 + b1 + b2) / 3.0f;
}

struct KnnLayout {
    size_t bb, code, k0, v0, v1, hist, sp, blo, bhi, total;
    explicit KnnLayout(int n) {
        const size_t m = (size_t)(n > 0 ? n : 1), nbox = (m + kBox - 1) / kBox;
        size_t o = 0;
        auto take = [&](size_t bytes) { size_t r = o; o += align_up(bytes); return r; };
        bb = take(6 * 4);
        code = take(4 * m);  // Morton codes; also the sort's second key buffer
        k0 = take(4 * m);
        v0 = take(4 * m);
        v1 = take(4 * m);
        hist = take(4 * sort_scratch_words((long long)m));
        sp = take(16 * m);
        blo = take(16 * nbox);
        bhi = take(16 * nbox);
        total = o;
    }
};

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_knn_scratch_bytes(int32_t N) { return KnnLayout(N).total; }

int gsr_knn_mean_dist2(const float* points, int32_t N, float* dist2, void* scratch, void* stream) {
    if (N < 0) return set_error(-1, "knn: negative N");
    if (N == 0) return 0;
    if (!points || !dist2 || !scratch) return set_error(-1, "knn: null pointer");
    hipStream_t s = (hipStream_t)stream;
    const KnnLayout L(N);
    char* base = static_cast<char*>(scratch);
    uint32_t* bb = reinterpret_cast<uint32_t*>(base + L.bb);
    uint32_t* code = reinterpret_cast<uint32_t*>(base + L.code);
    uint32_t* k0 = reinterpret_cast<uint32_t*>(base + L.k0);
    uint32_t* v0 = reinterpret_cast<uint32_t*>(base + L.v0);
    uint32_t* v1 = reinterpret_cast<uint32_t*>(base + L.v1);
    float4* sp = reinterpret_cast<float4*>(base + L.sp);
    float4* blo = reinterpret_cast<float4*>(base + L.blo);
    float4* bhi = reinterpret_cast<float4*>(base + L.bhi);
    if (hipError_t e = hipMemsetAsync(bb, 0xFF, 3 * sizeof(uint32_t), s)) return (int)e;
    if (hipError_t e = hipMemsetAsync(bb + 3, 0, 3 * sizeof(uint32_t), s)) return (int)e;
    const int nb = (N + 255) / 256;
    hipLaunchKernelGGL(knn_bbox_kernel, dim3(nb < 1024 ? nb : 1024), dim3(256), 0, s, points, N, bb);
    hipLaunchKernelGGL(knn_morton_kernel, dim3(nb), dim3(256), 0, s, points, N, bb, code);
    // 30-bit codes, identity values: 4 passes ping-pong (k0, v0) -> (code, v1)
    int which = -1;
    if (int e = radix_sort(code, nullptr, k0, v0, code, v1, N, nullptr, 30,
                           reinterpret_cast<uint32_t*>(base + L.hist), &which, s))
        return e;
    const uint32_t* order = which == 0 ? v0 : v1;
    const int nbox = (N + kBox - 1) / kBox;
    hipLaunchKernelGGL(knn_boxes_kernel, dim3(nbox), dim3(kBox), 0, s, points, order, N, sp, blo, bhi);
    hipLaunchKernelGGL(knn_kernel, dim3(nb), dim3(256), 0, s, sp, blo, bhi, N, nbox, dist2);
    return (int)hipGetLastError();
}

}  // extern "C"

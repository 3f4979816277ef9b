// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of this
// repository's kernels (MI355X_MICROARCH.md: "FETCH_SIZE reports 1/2 of the bytes of a wide
// coalesced streaming read ... other access widths are uncalibrated: calibrate on a known byte
// count in your own access pattern").  Each kernel moves a known number of bytes from/to a
// 2 GiB buffer (far beyond the 256 MiB Infinity Cache, so nothing is served on-die):
//   stream16   coalesced 16-B-per-lane reads               (F1 / B2 / gather streams)
//   stream4    coalesced 4-B-per-lane reads                 (scan, sort key streams)
//   gather16   one random 16-B record per lane              (F6 / B1 record gathers)
//   gather48   three consecutive 16-B loads of a random 48-B record per lane (the blend record)
//   gather4    one random 4-B word per lane                 (per-tile depth-key gathers)
//   write16    coalesced 16-B-per-lane stores
//   write4s    scattered 4-B stores, 9 of a 36-B entry per lane group (B1 partials pattern)
// Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes); the
// known bytes per kernel are printed so scripts/pmc_summary.py --calib can form the ratios.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr size_t kBytes = size_t(2) << 30;     // 2 GiB buffer
constexpr size_t kMoved = size_t(512) << 20;   // bytes each kernel moves

__device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void stream16(const float4* __restrict__ a, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i].x;
    if (s == 12345.f) out[0] = s;
}
__global__ void stream4(const float* __restrict__ a, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
    if (s == 12345.f) out[0] = s;
}
__global__ void gather16(const float4* __restrict__ a, size_t n_rec, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = a[hash32((uint32_t)i) % n_rec];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;
}
__global__ void gather48(const float4* __restrict__ a, size_t n_rec, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4* r = a + 3 * (size_t)(hash32((uint32_t)i) % n_rec);
        const float4 v0 = r[0], v1 = r[1], v2 = r[2];
        s += v0.x + v1.y + v2.z + v0.w + v1.x + v2.w;
    }
    if (s == 12345.f) out[0] = s;
}
__global__ void gather4(const float* __restrict__ a, size_t n_word, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        s += a[hash32((uint32_t)i) % n_word];
    if (s == 12345.f) out[0] = s;
}
__global__ void write16(float4* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        a[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
// a group of 9 lanes writes one 36-B entry (8 floats + 1 float in a second array), entries at
// random positions: the B1 partial stores
__global__ void write4s(float* __restrict__ p8, float* __restrict__ p1, size_t n_ent, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const size_t e = hash32((uint32_t)(i / 9)) % n_ent;
        const int c = (int)(i % 9);
        if (c < 8) p8[8 * e + c] = 1.f;
        else p1[e] = 1.f;
    }
}

int main() {
    float *buf = nullptr, *out = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, kBytes);
    const int grid = 256 * 16;
    hipLaunchKernelGGL(stream16, dim3(grid), dim3(256), 0, 0, (const float4*)buf, kMoved / 16, out);
    hipLaunchKernelGGL(stream4, dim3(grid), dim3(256), 0, 0, buf, kMoved / 4, out);
    hipLaunchKernelGGL(gather16, dim3(grid), dim3(256), 0, 0, (const float4*)buf, kBytes / 16, kMoved / 16, out);
    hipLaunchKernelGGL(gather48, dim3(grid), dim3(256), 0, 0, (const float4*)buf, kBytes / 48, kMoved / 48, out);
    hipLaunchKernelGGL(gather4, dim3(grid), dim3(256), 0, 0, buf, kBytes / 4, kMoved / 4, out);
    hipLaunchKernelGGL(write16, dim3(grid), dim3(256), 0, 0, (float4*)buf, kMoved / 16);
    hipLaunchKernelGGL(write4s, dim3(grid), dim3(256), 0, 0, buf, buf + (kBytes / 4) * 8 / 9,
                       (kBytes / 4) / 9 - 1, kMoved / 4);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"moved_bytes\": %zu, \"kernels\": [\"stream16\", \"stream4\", \"gather16\", \"gather48\", "
           "\"gather4\", \"write16\", \"write4s\"]}\n", kMoved);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}

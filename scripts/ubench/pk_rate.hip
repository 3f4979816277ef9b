// Microbenchmark: issue rate of v_fma_f32 vs v_pk_fma_f32 (wave64, 8 waves/SIMD).
// Prints ns per wave-instruction per SIMD for each form.  Used to decide whether the blend
// kernels gain from packing two pixels per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void scalar_fma(float* out, float s) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < kIters; ++i) {
        a0 = fmaf(a0, s, 1.0f); a1 = fmaf(a1, s, 1.0f); a2 = fmaf(a2, s, 1.0f); a3 = fmaf(a3, s, 1.0f);
        a4 = fmaf(a4, s, 1.0f); a5 = fmaf(a5, s, 1.0f); a6 = fmaf(a6, s, 1.0f); a7 = fmaf(a7, s, 1.0f);
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ __launch_bounds__(256) void packed_fma(float* out, float s) {
    f2 a0 = {(float)threadIdx.x, 1.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const f2 ss = {s, s}, one = {1.f, 1.f};
    for (int i = 0; i < kIters; ++i) {
        a0 = __builtin_elementwise_fma(a0, ss, one); a1 = __builtin_elementwise_fma(a1, ss, one);
        a2 = __builtin_elementwise_fma(a2, ss, one); a3 = __builtin_elementwise_fma(a3, ss, one);
        a4 = __builtin_elementwise_fma(a4, ss, one); a5 = __builtin_elementwise_fma(a5, ss, one);
        a6 = __builtin_elementwise_fma(a6, ss, one); a7 = __builtin_elementwise_fma(a7, ss, one);
    }
    f2 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}

__global__ __launch_bounds__(256) void scalar_exp(float* out, float s) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1e-3f, a2 = a0 + 2e-3f, a3 = a0 + 3e-3f;
    for (int i = 0; i < kIters; ++i) {
        a0 = __builtin_amdgcn_exp2f(a0) * s; a1 = __builtin_amdgcn_exp2f(a1) * s;
        a2 = __builtin_amdgcn_exp2f(a2) * s; a3 = __builtin_amdgcn_exp2f(a3) * s;
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 8 blocks x 4 waves per CU = 8 waves / SIMD
    float* out;
    hipMalloc(&out, sizeof(float) * blocks * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, const char* name, double insts_per_iter) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0.999f);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0.999f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double waves_per_simd = blocks * 4.0 / (cus * 4.0);
        const double insts = waves_per_simd * kIters * insts_per_iter * 5;
        printf("%-12s %.3f ms  %.3f ns per wave-instruction per SIMD\n", name, ms, ms * 1e6 / insts);
    };
    run(scalar_fma, "v_fma_f32", 8);
    run(packed_fma, "v_pk_fma_f32", 8);
    run(scalar_exp, "v_exp+v_mul", 8);
    hipFree(out);
    return 0;
}

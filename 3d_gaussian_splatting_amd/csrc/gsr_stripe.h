// gsr_stripe.h -- the per-(record, tile) stripe mask shared by F3 (gsr_sort.hip), which stores it
// in the low 4 bits of each list entry's sort value (value = gid << 4 | mask, kValShift), and the
// blend kernels (gsr_blend.hip), which read it back instead of recomputing it.  Compiled with FP
// contraction off inside the function whatever the including file's flags, so every file rounds
// it the same way.
#ifndef GSR_STRIPE_H
#define GSR_STRIPE_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

constexpr int kPPL = 4;       // pixels per lane = 16x4 stripes per 16x16 tile
constexpr int kValShift = 4;  // list values: gid << kValShift | stripe mask
constexpr uint32_t kValMask = (1u << kValShift) - 1u;

// Which of the tile's four 16x4 pixel stripes (slot p = rows 4p..4p+3) can hold a pixel
// with alpha >= 1/255.  Two conservative tests, both on the record the loading lane holds:
//  1. the padded footprint box (ext_x, ext_y) must overlap the stripe;
//  2. the footprint ellipse itself must reach the stripe's pixel-centre rectangle: with the
//     PD form Q(d) = -(a' dx^2 + b' dx dy + c' dy^2) (the exponent without log2 o), a pixel
//     passes alpha >= 1/255 iff Q <= log2(255 o), so the stripe is needed iff the minimum of Q
//     over the rectangle (0 if the mean is inside, else the minimum over its four edges,
//     each a clamped 1-D quadratic) is within that bound -- padded by 2 % + 0.05 for float
//     rounding.  Records whose form is not negative definite keep the box test only.
// Exact culling: a skipped stripe has no pixel that the per-pixel test would accept, so no
// output bit changes; the ellipse test removes ~22 % of the box test's stripe evaluations
// and ~17 % of the visited records at 1M/1080p (scripts/cull_stats.py).
// min over v in [v0, v1] of a u^2 + b u v + c v^2 (c > 0), given k = -b / (2c): the minimiser
// k u clamped to the edge.  k comes from a hardware reciprocal (1 ulp), not an IEEE division
// (~11 instructions each, 16 per record): a minimiser off by a few ulp raises q by c d^2, far
// inside the 2 % + 0.05 pad, and any point of the edge bounds the minimum from above only by
// that amount, so the test stays conservative.
__device__ __forceinline__ float edge_min_q(float a, float b, float c, float k, float u, float v0, float v1) {
#pragma clang fp contract(off)
    const float vs = fminf(fmaxf(k * u, v0), v1);
    return fmaf(fmaf(c, vs, b * u), vs, a * u * u);
}

__device__ inline uint32_t stripe_mask(const float4 r0, const float4 r1, const float4 r2, float bx0, float by0) {
#pragma clang fp contract(off)
    const float ex = r2.y, ey = r2.z;
    if (!(ex >= 0.0f) || r0.x + ex < bx0 || r0.x - ex > bx0 + 15.0f) return 0u;
    const float ylo = r0.y - ey, yhi = r0.y + ey;
    // PD form coefficients (A dx^2 + B dx dy + C dy^2) and the log2-domain bound
    const float A = -r0.z, B = -r0.w, C = -r1.x;
    const bool pd = A > 0.0f && C > 0.0f && 4.0f * A * C - B * B > 0.0f;
    const float bound = fmaf(fmaxf(r2.w + 7.99435343f, 0.0f), 1.02f, 0.05f);  // log2(255 o)
    const float x0 = bx0 - r0.x, x1 = bx0 + 15.0f - r0.x;  // rect in mean-relative coords
    const float kc = -B * __builtin_amdgcn_rcpf(2.0f * C), ka = -B * __builtin_amdgcn_rcpf(2.0f * A);
    uint32_t m = 0;
#pragma unroll
    for (int p = 0; p < kPPL; ++p) {
        const float s0 = by0 + 4.0f * p;
        bool hit = yhi >= s0 && ylo <= s0 + 3.0f;
        if (hit && pd) {
            const float y0 = s0 - r0.y, y1 = s0 + 3.0f - r0.y;
            const bool inside = x0 <= 0.0f && x1 >= 0.0f && y0 <= 0.0f && y1 >= 0.0f;
            const float q = fminf(fminf(edge_min_q(A, B, C, kc, x0, y0, y1), edge_min_q(A, B, C, kc, x1, y0, y1)),
                                  fminf(edge_min_q(C, B, A, ka, y0, x0, x1), edge_min_q(C, B, A, ka, y1, x0, x1)));
            hit = inside || q <= bound;
        }
        m |= hit ? (1u << p) : 0u;
    }
    return m;
}


}  // namespace gsr
#endif  // GSR_STRIPE_H

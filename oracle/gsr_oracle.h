/*
 * gsr_oracle.h -- CPU restatement of the differentiable 3DGS rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (3d_gaussian_splatting_amd/,
 * include/, libgsr_hip.so) includes, links or loads this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker.
 *
 * What it restates (see oracle/gsr_oracle.c for per-function citations):
 *   - reference math the rasterizer consumes, restated from the reference's own
 *     KAT-tested functions: build_rotation (src/utils/general_utils.cpp:12-40),
 *     build_scaling_rotation (:88-99), strip_lowerdiag (:49-62),
 *     build_covariance_from_scaling_rotation (src/scene/gaussian_model.cpp:18-28);
 *   - the rasterizer itself (preprocess, binning, blend, blend-backward,
 *     preprocess-backward).  The reference has NO rasterizer: the
 *     insertion point is src/utils/train_utils.cpp:137-144.  Its algorithm is the
 *     published 3DGS / EWA splatting algorithm restated in SURVEY.md Appendix B.
 *
 * Parity status: rasterizer outputs are "parity unpinned" against the reference
 * (it has no rasterizer and no golden vectors for one).  The inputs the rasterizer
 * consumes are pinned by the reference KATs (tests/test_reference_kats.py); the
 * rasterizer outputs are cross-checked against an independent dense torch-autograd
 * restatement (tests/golden/gen_golden.py -> committed fixtures) and central finite
 * differences.  See DESIGN.md "Oracle".
 */
#ifndef GSR_ORACLE_H
#define GSR_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gsro_camera {
    int width, height;
    float tanfovx, tanfovy;
    float viewmatrix[16]; /* column-major: t.r = sum_k m[4k+r] p_k + m[12+r] */
    float projmatrix[16]; /* full projection, same layout */
    float campos[3];
} gsro_camera;

typedef struct gsro_state gsro_state;

/* ---- reference math restatements (KAT-pinned) ---- */
/* build_rotation: q (w,x,y,z), normalised first, exactly general_utils.cpp:14-37 */
void gsro_build_rotation(const float* q, float* R /* 3x3 row-major */);
/* cov6 = strip_symmetric(L L^T), L = R(q) diag(mod*s): gaussian_model.cpp:18-28 */
void gsro_covariance(const float* s, float mod, const float* q, float* cov6);

/* ---- rasterizer ---- */
/* Forward.  All pointers are host memory.  sh_rest holds M_rest coefficients
 * (x3 channels) per Gaussian; D is the active SH degree ((D+1)^2-1 <= M_rest).
 * colors_precomp / cov3D_precomp are nullable and replace SH / (scale,rot).
 * Only tile rows [tile_y0, tile_y1) are binned and blended (band); pass 0 and
 * a large value for the whole image.  Returns num_rendered (>=0) or <0 on error. */
int gsro_forward(const gsro_camera* cam, int P, int D, int M_rest, const float* bg,
                 const float* means3D, const float* sh_dc, const float* sh_rest,
                 const float* colors_precomp, const float* opacities,
                 const float* scales, float scale_mod, const float* rotations,
                 const float* cov3D_precomp, int tile_y0, int tile_y1,
                 float* out_color /* 3*H*W */, int* radii /* P */,
                 gsro_state** state_out);

/* Backward for the state produced by gsro_forward.  Output arrays are fully
 * written (zeros for culled Gaussians).  Nullable outputs are skipped. */
int gsro_backward(gsro_state* st, const float* dL_dpix /* 3*H*W */,
                  float* dL_dmeans2D /* P*3 */, float* dL_dconic /* P*3: A,B,C */,
                  float* dL_dopacity /* P */, float* dL_dcolors /* P*3 */,
                  float* dL_dmeans3D /* P*3 */, float* dL_dsh_dc /* P*3 */,
                  float* dL_dsh_rest /* P*M_rest*3 */, float* dL_dscales /* P*3 */,
                  float* dL_drotations /* P*4 */, float* dL_dcov3D /* P*6 */);

void gsro_free(gsro_state* st);

/* ---- state accessors (tests) ---- */
int gsro_num_rendered(const gsro_state* st);
/* sorted instance list: tile id, depth bits and Gaussian id per entry */
void gsro_get_sorted(const gsro_state* st, uint32_t* tile, uint32_t* depth_bits, uint32_t* gid);
/* per-tile [start,end) ranges into the sorted list, num_tiles*2 */
void gsro_get_ranges(const gsro_state* st, uint32_t* ranges);
/* per-pixel final transmittance and last contributor */
void gsro_get_pixel_state(const gsro_state* st, float* final_T, uint32_t* n_contrib);
/* per-Gaussian preprocess: xy (P*2), depth (P), conic+opacity (P*4), rgb (P*3),
 * tiles_touched (P, band-clipped) */
void gsro_get_preprocess(const gsro_state* st, float* xy, float* depth, float* conic_o,
                         float* rgb, uint32_t* tiles_touched);
/* count of (pixel, list entry) evaluations the forward made (VALU-bound proxy) */
uint64_t gsro_forward_pairs(const gsro_state* st);
/* blend kernels' stripe-culling work statistics (F6 wave visits, B1 stripe evaluations, those
 * with a contributing pixel, B1 visited entries): lower bounds, see gsr_oracle.c */
void gsro_blend_work(const gsro_state* st, uint64_t out[4]);
/* per pixel: list entries examined by the forward before termination */
void gsro_get_examined(const gsro_state* st, uint32_t* examined);

#ifdef __cplusplus
}
#endif
#endif

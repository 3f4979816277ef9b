/*
 * gsr_train.h -- C ABI of the training-step kernels around the rasterizer (SURVEY.md §8f
 * rows 1-2): photometric loss, fused Adam over the six parameter groups, densification
 * statistics and the prune compaction.  Same conventions as gsr.h: caller-owned DEVICE
 * memory (f32, contiguous, channel-major images), one hipStream_t, 0 = ok / < 0 = error with
 * the message in gsr_last_error of gsr.h, no persistent allocations.
 *
 * What each entry point replaces in the reference (seiya-kumada/3d_gaussian_splatting):
 *
 *   gsr_activate           <- GaussianModel::get_scaling / get_rotation / get_opacity
 *                             (src/scene/gaussian_model.cpp:270-280,295-298; activations
 *                             exp / normalize / sigmoid bound at :54-58)
 *   gsr_loss_forward       <- the loss the training loop at src/utils/train_utils.cpp:128-145
 *   gsr_loss_backward         would compute: (1 - lambda_dssim) L1 + lambda_dssim (1 - SSIM),
 *                             lambda_dssim from OptimizationParams (src/arguments/params.h:62).
 *                             The reference has no loss code (its loop is a stub); the
 *                             definition is the upstream 3DGS one (11x11 Gaussian window,
 *                             sigma 1.5, zero padding, C1 = 0.01^2, C2 = 0.03^2, mean).
 *   gsr_adam_step          <- the six torch::optim::Adam instances of GaussianModel::setup
 *                             (src/scene/gaussian_model.cpp:323-345: default AdamOptions,
 *                             betas 0.9 / 0.999, eps 1e-8, no weight decay) stepped once each,
 *                             with the activation backward (exp / sigmoid / normalize) of
 *                             the getters fused in front of the moment update.
 *   gsr_densify_stats      <- max_radii2D_ / xyz_gradient_accum_ / denom_ updates
 *                             (src/scene/gaussian_model.h:18-20; setup :318-319)
 *   gsr_compact_index      <- the boolean-mask selection of prune_points / densify_and_clone
 *   gsr_gather_rows           (upstream densification; the reference declares only the stats
 *                             tensors): index list from a mask, then one multi-tensor row
 *                             gather for parameters, Adam moments and statistics.
 */
#ifndef GSR_GSR_TRAIN_H
#define GSR_GSR_TRAIN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* exp / normalize / sigmoid of the raw leaves (GaussianModel getters).  Any output may be
 * NULL (skipped).  rot_raw / rot rows of 4 (w first), 16-B aligned. */
int gsr_activate(const float* scale_raw, const float* rot_raw, const float* opac_raw, int32_t P,
                 float* scales, float* rots, float* opacs, void* stream);

/* Loss over C x H x W images: stats[0] = loss, stats[1] = mean |img - gt|, stats[2] = mean SSIM
 * (device floats).  `maps` is caller scratch of gsr_loss_scratch_bytes(C, H, W) bytes holding
 * the per-pixel SSIM derivative maps for gsr_loss_backward.  Deterministic (fixed-order sums). */
size_t gsr_loss_scratch_bytes(int32_t C, int32_t H, int32_t W);
int gsr_loss_forward(const float* img, const float* gt, int32_t C, int32_t H, int32_t W,
                     float lambda_dssim, void* maps, float* stats, void* stream);
/* dL/dimg (C x H x W) for dL/dloss = 1, from the maps the forward left in `maps`. */
int gsr_loss_backward(const float* img, const float* gt, int32_t C, int32_t H, int32_t W,
                      float lambda_dssim, const void* maps, float* dL_dimg, void* stream);

/* Activation applied by the getter in front of a parameter group (its gradient arrives with
 * respect to the activated value; gsr_adam_step converts it to the raw leaf first). */
#define GSR_ACT_NONE 0       /* xyz, features_dc, features_rest */
#define GSR_ACT_EXP 1        /* scaling */
#define GSR_ACT_SIGMOID 2    /* opacity */
#define GSR_ACT_NORMALIZE4 3 /* rotation: rows of 4, x / max(|x|, 1e-12) */

typedef struct gsr_adam_group {
    float* param;            /* raw leaf, n floats (updated in place) */
    const float* grad;       /* gradient w.r.t. the ACTIVATED value (n floats) */
    float* exp_avg;          /* Adam state, n floats */
    float* exp_avg_sq;       /* Adam state, n floats */
    int64_t n;
    int32_t act;             /* GSR_ACT_* */
    int32_t step;            /* this group's step count AFTER increment (>= 1) */
    float lr;
} gsr_adam_group;
#define GSR_ADAM_MAX_GROUPS 8
/* One Adam step (libtorch torch::optim::Adam semantics, amsgrad off, weight_decay 0) of up
 * to GSR_ADAM_MAX_GROUPS groups in ONE launch; `groups` is a HOST array. */
int gsr_adam_step(const gsr_adam_group* groups, int32_t ngroups, float beta1, float beta2, float eps,
                  void* stream);
/* The same step behind a device-side guard: it is skipped ON THE DEVICE when
 * *guard_k > guard_cap (guard_k NULL: never skipped).  guard_k is the forward's instance count K
 * (gsr_view(GSR_VIEW_COUNTS) word 0, the scan's counter: the true K, not clamped) and guard_cap
 * the max_rendered bound that render ran under.  A render above its bound was truncated; a
 * training loop that renders without a per-iteration host read of K passes them so that the
 * truncated iteration's update is dropped instead of applied (the groups' step counts the host
 * already advanced are not rolled back). */
int gsr_adam_step_guarded(const gsr_adam_group* groups, int32_t ngroups, float beta1, float beta2, float eps,
                          const uint32_t* guard_k, uint32_t guard_cap, void* stream);

/* Densification statistics for the visible Gaussians (radii > 0):
 *   max_radii2D = max(max_radii2D, radii); grad_accum += |dL/dmeans2D[:, :2]|; denom += 1.
 * dmeans2D: P x 3 (the rasterizer's dL_dmeans2D, the reference's viewspace_points grad). */
int gsr_densify_stats(const int32_t* radii, const float* dmeans2D, int32_t P, float* max_radii2D,
                      float* grad_accum, float* denom, void* stream);
/* ... skipped on the device when *guard_k > guard_cap (as gsr_adam_step_guarded). */
int gsr_densify_stats_guarded(const int32_t* radii, const float* dmeans2D, int32_t P, float* max_radii2D,
                              float* grad_accum, float* denom, const uint32_t* guard_k, uint32_t guard_cap,
                              void* stream);

/* Stream compaction: idx_out[0 .. count) = the i with mask[i] != 0, ascending; *count_out
 * (device int32).  scratch: gsr_compact_scratch_bytes(n). */
size_t gsr_compact_scratch_bytes(int32_t n);
int gsr_compact_index(const uint8_t* mask, int32_t n, int32_t* idx_out, int32_t* count_out, void* scratch,
                      void* stream);

typedef struct gsr_row_copy {
    const float* src;        /* rows of `width` floats */
    float* dst;              /* n_out rows of `width` floats (must not alias src) */
    int32_t width;
} gsr_row_copy;
#define GSR_GATHER_MAX 24
/* dst[i] = src[idx[i]] (row copies) for every entry of `copies` (HOST array) in one launch. */
int gsr_gather_rows(const gsr_row_copy* copies, int32_t ncopies, const int32_t* idx, int32_t n_out,
                    void* stream);

/* Point-cloud initialisation (upstream create_from_pcd, whose distCUDA2 this
 * replaces -- the reference's point-cloud branch is commented out,
 * src/scene/dataset_readers.cpp:198-219): dist2[i] = mean of the squared distances from point i
 * to its 3 nearest OTHER points (exact; with fewer than 3 other points the missing ones count as
 * FLT_MAX, as in upstream's kernel, so the mean is FLT_MAX / 3 or overflows to +inf).
 * points: N x 3 f32 device; scratch: gsr_knn_scratch_bytes(N) bytes. */
size_t gsr_knn_scratch_bytes(int32_t N);
int gsr_knn_mean_dist2(const float* points, int32_t N, float* dist2, void* scratch, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_GSR_TRAIN_H */

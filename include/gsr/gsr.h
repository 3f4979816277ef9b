/*
 * gsr.h -- C ABI of the MI355X-native differentiable 3D Gaussian splat rasterizer.
 *
 * This is the ONLY interface host code uses to reach the HIP kernels (libgsr_hip.so).
 * Plain C: no torch types, no C++ types, no exceptions across the boundary.
 *
 * What it replaces in the reference (seiya-kumada/3d_gaussian_splatting):
 * the reference has no rasterizer.  The render -> loss -> backward
 * call belongs at src/utils/train_utils.cpp:137-144 (the commented camera pick in the
 * training loop); the inputs it consumes are the GaussianModel getters
 * (src/scene/gaussian_model.h:85-90, activations gaussian_model.cpp:270-298), the Camera
 * matrices (src/scene/camera.cpp:66-71), PipelineParams (src/arguments/params.h:93-106)
 * and the background tensor (src/utils/train_utils.cpp:115-117).  The libtorch layer
 * (3d_gaussian_splatting_amd/csrc/torch/gsr_torch.cpp) maps those to the structs below.
 *
 *   gsr_forward            <- render() forward         (F1..F6)
 *   gsr_backward           <- loss.backward() into it  (B1+B2, a17-a18)
 *   gsr_backward_blend     <- B1 + per-Gaussian sum only (multi-GPU: all-reduce between)
 *   gsr_backward_preprocess<- B2 only, from per-Gaussian 2D gradients
 *   gsr_backward_preprocess_range <- B2 on one Gaussian slice (multi-GPU, after reduce-scatter)
 *
 * Conventions
 *   - Every pointer in gsr_gaussians / gsr_grads / outputs is caller-owned DEVICE memory
 *     (f32, contiguous, row-major as torch lays out the (N,...) tensors).
 *   - Camera matrices are host values, f32, column-major: t.r = sum_k m[4k+r] p_k + m[12+r]
 *     (= the reference's row-vector-convention 4x4 tensors flattened row-major).
 *   - Scratch: the library allocates nothing persistent.  Forward asks the caller for three
 *     buffers through gsr_alloc_fn (geometry: per Gaussian, binning: per tile instance,
 *     image: per pixel); the caller keeps them alive and passes them back to backward.
 *   - Streams: all work is ordered on `stream` (a hipStream_t; NULL = default stream).
 *     One device->host read per forward (num_rendered) synchronises that stream; a banded
 *     forward (tile_y0/y1 narrower than the image) adds a second (its candidate count).
 *   - Errors: 0 = ok, < 0 = error; message in gsr_last_error() (thread-local).
 *   - Re-entrant; no global state besides the thread-local error string and the optional,
 *     off-by-default stage profiler (gsr_profile_*).
 */
#ifndef GSR_GSR_H
#define GSR_GSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ABI_VERSION 1
#define GSR_TILE 16 /* screen tiles are GSR_TILE x GSR_TILE pixels */
#define GSR_GRAD2D_STRIDE 12 /* floats per Gaussian in a grad2d buffer (9 used) */

/* flags */
#define GSR_FLAG_DEBUG 1u /* synchronise + check after every stage */
#define GSR_FLAG_BAND_ONLY 2u /* band forward/backward_blend for multi-GPU: leave pixels outside
                                 the band and grad2d rows of Gaussians outside the band's
                                 ranking unwritten (only those rows are exchanged) */

typedef struct gsr_camera {
    int32_t width, height;
    float tanfovx, tanfovy;  /* tan(FoV/2) */
    float viewmatrix[16];    /* world_view_transform, column-major (see above) */
    float projmatrix[16];    /* full_proj_transform, column-major */
    float campos[3];         /* camera centre, world space */
} gsr_camera;

typedef struct gsr_gaussians {
    int32_t P;               /* number of Gaussians */
    int32_t sh_degree;       /* active SH degree D (0..3) */
    int32_t sh_rest_coeffs;  /* coefficients per Gaussian stored in sh_rest (>= (D+1)^2-1) */
    float scale_modifier;
    const float* means3D;    /* P x 3 */
    const float* sh_dc;      /* P x 1 x 3            (NULL iff colors_precomp) */
    const float* sh_rest;    /* P x sh_rest_coeffs x 3 (NULL if D == 0 or colors_precomp) */
    const float* colors_precomp; /* P x 3 or NULL (PipelineParams::convert_SHs_python_) */
    const float* opacities;  /* P (activated: sigmoid) */
    const float* scales;     /* P x 3 (activated: exp)   (NULL iff cov3D_precomp) */
    const float* rotations;  /* P x 4 (normalised, w first) (NULL iff cov3D_precomp) */
    const float* cov3D_precomp; /* P x 6 [xx,xy,xz,yy,yz,zz] or NULL
                                   (PipelineParams::compute_cov3D_python_) */
} gsr_gaussians;

typedef struct gsr_raster_settings {
    float bg[3];             /* background colour */
    int32_t tile_y0;         /* band of tile rows to bin/blend: [tile_y0, tile_y1); */
    int32_t tile_y1;         /* 0 and INT32_MAX = whole image (multi-GPU sharding)   */
    uint32_t flags;          /* GSR_FLAG_* */
} gsr_raster_settings;

typedef struct gsr_grads {
    float* dL_dmeans2D;      /* P x 3 (NDC x,y; z = 0)               required */
    float* dL_dconic;        /* P x 3 (A,B,C of the inverse cov2D)   nullable */
    float* dL_dopacity;      /* P                                    required */
    float* dL_dcolors;       /* P x 3   required iff colors_precomp */
    float* dL_dmeans3D;      /* P x 3                                required */
    float* dL_dsh_dc;        /* P x 1 x 3   required iff !colors_precomp */
    float* dL_dsh_rest;      /* P x sh_rest_coeffs x 3  (required iff sh_rest != NULL) */
    float* dL_dscales;       /* P x 3   required iff !cov3D_precomp */
    float* dL_drotations;    /* P x 4   required iff !cov3D_precomp */
    float* dL_dcov3D;        /* P x 6   required iff cov3D_precomp */
} gsr_grads;

/* Allocation callback: return device memory of at least `bytes` (16-B aligned) that stays
 * valid until the matching backward; NULL on failure. */
typedef void* (*gsr_alloc_fn)(void* ctx, size_t bytes);

typedef struct gsr_buffers {
    void* geom;              /* returned by the geometry allocation */
    void* binning;           /* returned by the binning allocation (may be NULL if K == 0) */
    void* image;             /* returned by the image allocation */
    int32_t num_rendered;    /* K = number of (Gaussian, tile) instances */
    int32_t num_ranked;      /* Gaussians in the depth ranking: P for a full image; for a band,
                                only those with tiles in the band (pass back unchanged) */
} gsr_buffers;

int gsr_abi_version(void);
const char* gsr_last_error(void);

/* Forward: out_color (3 x H x W, channel-major) and radii (P, int32; 0 = culled).
 * Pixels outside the tile band are set to the background (left unwritten under
 * GSR_FLAG_BAND_ONLY).  Fills *bufs. */
int gsr_forward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                float* out_color, int32_t* radii, gsr_alloc_fn alloc_geom,
                gsr_alloc_fn alloc_binning, gsr_alloc_fn alloc_image, void* alloc_ctx,
                gsr_buffers* bufs, void* stream);

/* Batched forward over V views of the same Gaussians (the reference's loop
 * renders one camera per iteration, src/utils/train_utils.cpp:128-145).  Per view the work of
 * gsr_forward, but the V first phases (preprocess + scan) are enqueued back to back and ONE
 * device->host read returns all V instance counts, so the host waits once per batch instead of
 * once per view and the GPU is not left idle between views.  cams[v], out_colors[v]
 * (3 x H_v x W_v), radii[v] (P), bufs[v]: as for gsr_forward; each view's backward is
 * gsr_backward with bufs[v].  Full-image views only (rs->tile_y0/y1 must cover every view);
 * one extra 8*V-byte allocation through alloc_image holds the counts.  0 < V <= GSR_MAX_BATCH. */
#define GSR_MAX_BATCH 64
int gsr_forward_batch(int32_t V, const gsr_camera* cams, const gsr_gaussians* gs,
                      const gsr_raster_settings* rs, float* const* out_colors, int32_t* const* radii,
                      gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_binning, gsr_alloc_fn alloc_image,
                      void* alloc_ctx, gsr_buffers* bufs, void* stream);

/* Full backward (B1 + gather + B2).  dL_dout_color: 3 x H x W.  scratch: asked for twice
 * through alloc_scratch (gsr_scratch_bytes(K) for per-instance partial gradients, then
 * 48 * P bytes for the per-Gaussian screen-space gradient), valid for the duration of the call. */
int gsr_backward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                 const gsr_buffers* bufs, const float* dL_dout_color, gsr_alloc_fn alloc_scratch,
                 void* alloc_ctx, const gsr_grads* grads, void* stream);

/* B1 only: per-Gaussian 2D gradients into grad2d (P x GSR_GRAD2D_STRIDE floats:
 * mean2D.x, mean2D.y, conic A, B, C, opacity, r, g, b, 0, 0, 0). Summable across
 * tile bands (all-reduce) before gsr_backward_preprocess.  A band writes zeros for the
 * Gaussians outside its ranking (GSR_VIEW_GID_BY_RANK), or nothing under GSR_FLAG_BAND_ONLY. */
int gsr_backward_blend(const gsr_camera* cam, const gsr_gaussians* gs,
                       const gsr_raster_settings* rs, const gsr_buffers* bufs,
                       const float* dL_dout_color, gsr_alloc_fn alloc_scratch, void* alloc_ctx,
                       float* grad2d, void* stream);

/* B2 only: leaf gradients from grad2d (P x GSR_GRAD2D_STRIDE). */
int gsr_backward_preprocess(const gsr_camera* cam, const gsr_gaussians* gs,
                            const gsr_raster_settings* rs, const gsr_buffers* bufs,
                            const float* grad2d, const gsr_grads* grads, void* stream);

/* B2 on the Gaussian slice [g0, g1) only (multi-GPU: each rank owns a slice after a
 * reduce-scatter of grad2d).  grad2d holds the slice's (g1 - g0) rows, and every output in
 * `grads` is the slice's own array (row g - g0); the inputs in `gs` stay full-size. */
int gsr_backward_preprocess_range(const gsr_camera* cam, const gsr_gaussians* gs,
                                  const gsr_raster_settings* rs, const gsr_buffers* bufs,
                                  int32_t g0, int32_t g1, const float* grad2d,
                                  const gsr_grads* grads, void* stream);

/* Introspection for tests / the benchmark (all device pointers into the caller's buffers,
 * or NULL when not applicable).  `what`: see gsr_view_* below. */
#define GSR_VIEW_RADII_SORTED_GID 1 /* uint32[K]: Gaussian id of sorted instance i       */
#define GSR_VIEW_SORTED_TILE 2      /* uint32[K]: tile id of sorted instance i             */
#define GSR_VIEW_RANGES 3           /* uint32[2*tiles]: [start,end) per tile               */
#define GSR_VIEW_FINAL_T 4          /* float[H*W]                                          */
#define GSR_VIEW_N_CONTRIB 5        /* retired (always NULL): the blend no longer keeps a   
                                       per-pixel contributor count; B1 re-derives the      
                                       termination point from T                             */
#define GSR_VIEW_DEPTH_KEY 6        /* uint32[P]: depth bits, 0xFFFFFFFF when culled       */
#define GSR_VIEW_TILES_TOUCHED 7    /* uint32[P]                                           */
#define GSR_VIEW_GID_BY_RANK 9      /* uint32[num_ranked]: the ranked Gaussian ids -- ascending
                                       (shipped binning; depth order under GSR_BIN_VARIANT=0);
                                       a band's candidates: exactly the Gaussians it can touch */
#define GSR_VIEW_RECORDS 8          /* float4[3*P]: {x,y,a',b'},{c',o,r,g},{b,ext_x,ext_y,log2 o};
                                       a',b',c' = -log2(e) * (A/2, B, C/2) of the conic */
const void* gsr_view(const gsr_camera* cam, int32_t P, const gsr_buffers* bufs, int what);

/* Optional stage profiler (off by default; process-wide, mutex-protected).  When enabled,
 * every stage in `stage_mask` (bit i = stage i below) is bracketed by two hipEvents on the
 * call's stream; gsr_profile_read synchronises those events and returns the accumulated
 * milliseconds and launch counts per stage (arrays of GSR_NUM_STAGES), then resets. */
#define GSR_STAGE_PREPROCESS 0     /* F1 */
#define GSR_STAGE_DEPTH_SORT 1     /* depth order: per-tile depth sort (shipped) or the global
                                      depth-key LSD sort of the P Gaussians; band compaction */
#define GSR_STAGE_SCAN 2           /* F2 scan of tiles_touched (rank order) */
#define GSR_STAGE_DUPLICATE 3      /* F3 */
#define GSR_STAGE_TILE_SORT 4      /* F4 tile-key LSD sort of the K instances */
#define GSR_STAGE_FINALIZE 5       /* F5 sorted gid + tile ranges */
#define GSR_STAGE_BLEND_FWD 6      /* F6 */
#define GSR_STAGE_BLEND_BWD 7      /* B1 */
#define GSR_STAGE_PREPROCESS_BWD 8 /* B2 */
#define GSR_STAGE_GATHER 9         /* per-Gaussian grad2d sum of the B1 partials */
#define GSR_STAGE_MISC 10          /* memsets, background fill, num_rendered read */
#define GSR_NUM_STAGES 11
int gsr_profile_enable(uint32_t stage_mask);
int gsr_profile_read(double* ms, uint32_t* counts);
const char* gsr_stage_name(int stage);

/* Byte sizes the allocation callbacks will be asked for (for pre-sizing pools). */
size_t gsr_geom_bytes(int32_t P);
size_t gsr_binning_bytes(int32_t K);
size_t gsr_image_bytes(int32_t width, int32_t height);
size_t gsr_scratch_bytes(int32_t K);

#ifdef __cplusplus
}
#endif
#endif /* GSR_GSR_H */

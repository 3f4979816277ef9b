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
 *   gsr_backward_blend     <- B1 + per-Gaussian sum only (2D gradients)
 *   gsr_backward_preprocess<- B2 only, from per-Gaussian 2D gradients
 *   gsr_shard_* / gsr_band_* <- the multi-GPU split of the same path: F1/B2 on a
 *                             Gaussian shard, F2..F6/B1 on a band of tile rows, with two
 *                             all-to-all exchanges in between (done by the caller over RCCL)
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
 *   - Host waits: with rs->max_rendered == 0 the forward reads K (num_rendered) back once to
 *     size the binning exactly (the read overlaps the scan); with rs->max_rendered > 0 the
 *     binning is sized for that many instances and nothing is read back: K stays on the
 *     device (gsr_read_num_rendered), and K > max_rendered is an overflow the caller detects
 *     there (instances past the bound are dropped, every kernel stays inside its buffers).
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

#define GSR_ABI_VERSION 4
#define GSR_TILE 16 /* screen tiles are GSR_TILE x GSR_TILE pixels */
#define GSR_GRAD2D_STRIDE 12 /* floats per Gaussian in a grad2d buffer (9 used) */

/* flags */
#define GSR_FLAG_DEBUG 1u /* synchronise + check after every stage */
/* gsr_shard_forward: row_hist holds 3 x grid_y u32 -- the instances per tile row, then the
 * visible Gaussians whose tile rect starts in row y, then those whose rect ends (last row) in y:
 * the splats any band cut [r0, r1) receives are sum_{y<r1} starts - sum_{y<r0} ends, so a
 * multi-GPU step re-plans its cuts and capacities from a step's own statistics (no probe). */
#define GSR_FLAG_ROW_SPANS 2u
#define GSR_ERR_OVERFLOW (-4) /* gsr_read_num_rendered: K exceeded the binning's capacity */

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
    int32_t max_rendered;    /* 0: binning sized from K (one host read per forward);
                                > 0: binning for this many instances, no host read */
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
    void* binning;           /* returned by the binning allocation */
    void* image;             /* returned by the image allocation */
    int32_t num_rendered;    /* K = number of (Gaussian, tile) instances; -1 while it is only on
                                the device (max_rendered > 0; see gsr_read_num_rendered) */
    int32_t capacity;        /* instances the binning (and the backward's scratch) hold */
    int32_t n_local;         /* Gaussians (or received splat slots, gsr_band_forward) indexed */
    uint32_t layout;         /* set by the forward: GSR_LAYOUT_TAG | GSR_LAYOUT_* bits, which arrays of
                                the binning hold the sorted list.  Pass the forward's gsr_buffers to the
                                backward / gsr_view unchanged: a word without the tag (e.g. a struct
                                rebuilt with this field zeroed) or with bits that disagree with the
                                buffers' sizes is refused (< 0, gsr_last_error), never read blindly */
} gsr_buffers;
#define GSR_LAYOUT_TAG 0x47530000u      /* 'G' 'S' in the upper half: written by a forward (ABI 4) */
#define GSR_LAYOUT_TAG_MASK 0xFFFF0000u
#define GSR_LAYOUT_ROW_BUCKETED 1u      /* row-bucketed binning (tile keys not stored in the step) */
#define GSR_LAYOUT_PRESORT 2u           /* global depth pre-sort (rank-order payload) */
#define GSR_ERR_LAYOUT (-13)            /* gsr_buffers.layout missing or inconsistent */

int gsr_abi_version(void);
const char* gsr_last_error(void);

/* Forward: out_color (3 x H x W, channel-major) and radii (P, int32; 0 = culled).
 * Pixels outside the tile band are set to the background.  Fills *bufs. */
int gsr_forward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                float* out_color, int32_t* radii, gsr_alloc_fn alloc_geom,
                gsr_alloc_fn alloc_binning, gsr_alloc_fn alloc_image, void* alloc_ctx,
                gsr_buffers* bufs, void* stream);

/* K of a forward, read back synchronously (waits for the forward on `stream`): sets
 * bufs->num_rendered and returns 0, or GSR_ERR_OVERFLOW when K > bufs->capacity (the
 * forward's outputs are then incomplete: re-run it with a larger max_rendered). */
int gsr_read_num_rendered(const gsr_camera* cam, const gsr_buffers* bufs, int32_t* num_rendered,
                          void* stream);

/* Batched forward over V views of the same Gaussians (the reference's loop
 * renders one camera per iteration, src/utils/train_utils.cpp:128-145).  Per view the work of
 * gsr_forward; with rs->max_rendered == 0 the V preprocess passes are enqueued back to back and
 * ONE device->host read returns all V instance counts, so the host waits once per batch
 * instead of once per view.  cams[v], out_colors[v] (3 x H_v x W_v), radii[v] (P), bufs[v]: as
 * for gsr_forward; each view's backward is gsr_backward with bufs[v].  Full-image views only;
 * one extra 8*V-byte allocation through alloc_image holds the counts.  0 < V <= GSR_MAX_BATCH. */
#define GSR_MAX_BATCH 64
int gsr_forward_batch(int32_t V, const gsr_camera* cams, const gsr_gaussians* gs,
                      const gsr_raster_settings* rs, float* const* out_colors, int32_t* const* radii,
                      gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_binning, gsr_alloc_fn alloc_image,
                      void* alloc_ctx, gsr_buffers* bufs, void* stream);

/* Views mode: V same-size cameras rendered as ONE pass -- one launch per
 * stage for all views.  The views are stacked as bands of ceil(H/16) tile rows of one tall
 * binning, so F1, the scan, F3, the tile sort, F6 and (in gsr_backward_views) B1, the gather
 * and B2 each run once over V*P (view, Gaussian) entries.  The result is bit-identical to V
 * gsr_forward / gsr_backward calls: a tile belongs to one view and keeps the canonical
 * (depth, Gaussian) order.
 *   cams: V cameras, all of one width and height (full image, no tile band in rs)
 *   out_color: V x 3 x H x W;  radii: V x P;  bufs: ONE gsr_buffers for the whole pass
 *   (geometry for V*P entries, image and binning for the tall V*ceil(H/16)*16 x W image).
 * The backward reads dL_dout_color as V x 3 x H x W and writes dL_dmeans2D / dL_dconic as
 * V x P x 3 (per view, as the reference's viewspace points are); every leaf gradient is the
 * sum over the views, added in view order -- (((g_0 + g_1) + g_2) + ...) -- as a caller
 * summing per-view backward results would.  alloc_scratch is asked for three blocks: the
 * partial gradients, 48 * V * P bytes of grad2d, and (V > 1) the V-1 per-view leaf gradient
 * slices.  1 <= V <= GSR_MAX_VIEWS.  Under a binning bound (rs->max_rendered > 0) the pass's K
 * is read with gsr_read_num_rendered given the tall camera: cams[0] with height
 * V * ceil(H / 16) * 16 (the layout of the pass's image buffer). */
#define GSR_MAX_VIEWS 8
int gsr_forward_views(int32_t V, const gsr_camera* cams, const gsr_gaussians* gs,
                      const gsr_raster_settings* rs, float* out_color, int32_t* radii,
                      gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_binning, gsr_alloc_fn alloc_image,
                      void* alloc_ctx, gsr_buffers* bufs, void* stream);
int gsr_backward_views(int32_t V, const gsr_camera* cams, const gsr_gaussians* gs,
                       const gsr_raster_settings* rs, const gsr_buffers* bufs, const float* dL_dout_color,
                       gsr_alloc_fn alloc_scratch, void* alloc_ctx, const gsr_grads* grads, void* stream);

/* Full backward (B1 + gather + B2).  dL_dout_color: 3 x H x W.  scratch: asked for twice
 * through alloc_scratch (gsr_scratch_bytes(capacity) for per-instance partial gradients, then
 * 48 * P bytes for the per-Gaussian screen-space gradient), valid for the duration of the call. */
int gsr_backward(const gsr_camera* cam, const gsr_gaussians* gs, const gsr_raster_settings* rs,
                 const gsr_buffers* bufs, const float* dL_dout_color, gsr_alloc_fn alloc_scratch,
                 void* alloc_ctx, const gsr_grads* grads, void* stream);

/* B1 only: per-Gaussian 2D gradients into grad2d (P x GSR_GRAD2D_STRIDE floats:
 * mean2D.x, mean2D.y, conic A, B, C, opacity, r, g, b, 0, 0, 0).  Summable across tile bands
 * before gsr_backward_preprocess (zeros for Gaussians outside the band). */
int gsr_backward_blend(const gsr_camera* cam, const gsr_gaussians* gs,
                       const gsr_raster_settings* rs, const gsr_buffers* bufs,
                       const float* dL_dout_color, gsr_alloc_fn alloc_scratch, void* alloc_ctx,
                       float* grad2d, void* stream);

/* B2 only: leaf gradients from grad2d (P x GSR_GRAD2D_STRIDE). */
int gsr_backward_preprocess(const gsr_camera* cam, const gsr_gaussians* gs,
                            const gsr_raster_settings* rs, const gsr_buffers* bufs,
                            const float* grad2d, const gsr_grads* grads, void* stream);

/* ---- Multi-GPU: Gaussian shards x tile-row bands (the scaling version) ----
 * Rank r of N owns the Gaussian shard [g0_r, g1_r) (contiguous, in rank order) and the band
 * of tile rows [band_rows[r], band_rows[r+1]).  One step:
 *   1. gsr_shard_forward   F1 on the shard, then every projected Gaussian ("splat", 64 B) is
 *                          packed into the send block of each band its tile rect overlaps
 *   2. caller              all-to-all of the send blocks (block b -> rank b)
 *   3. gsr_band_forward    F2..F6 on the band over the splats received from every shard
 *   4. caller              all-gather of the band images
 *   5. gsr_band_backward   B1 + per-splat 2D gradient, written in the received slot layout
 *   6. caller              all-to-all back (block s -> rank s)
 *   7. gsr_shard_backward  per Gaussian, the sum of its bands' 2D gradients in band order,
 *                          then B2 on the shard
 * Exchange block layout (nblocks blocks of gsr_exchange_block_bytes(pair_cap) each): a 64-B
 * header whose first u32 is the number of splats the sender packed for that pair (it may
 * exceed pair_cap: an overflow -- the splats past pair_cap are not sent), then pair_cap
 * 64-B splats.  The gradient blocks going back are pair_cap x 48 B (no header).  Splats
 * reach the band in (source rank, shard index) order = ascending global Gaussian id, so the
 * canonical order and every rendered pixel are those of the single-GPU forward. */
#define GSR_SPLAT_BYTES 64
#define GSR_SPLAT_GRAD_BYTES 48
size_t gsr_exchange_block_bytes(int32_t pair_cap);
size_t gsr_shard_state_bytes(int32_t P, int32_t nbands, int32_t pair_cap);

/* radii: P (shard rows).  shard_state: gsr_shard_state_bytes, kept until gsr_shard_backward.
 * send: nbands exchange blocks.  row_hist (nullable, device, zeroed by the caller): += the
 * instances per tile row of this shard (grid_y u32) -- band balancing for the next step; with
 * rs->flags & GSR_FLAG_ROW_SPANS also the rect start / end rows (3 x grid_y u32, see above). */
int gsr_shard_forward(const gsr_camera* cam, const gsr_gaussians* shard, const gsr_raster_settings* rs,
                      int32_t nbands, const int32_t* band_rows, int32_t pair_cap, void* send,
                      int32_t* radii, void* shard_state, uint32_t* row_hist, void* stream);

/* recv: nsrc exchange blocks.  rs->tile_y0/y1 = this rank's band; rs->max_rendered > 0 is the
 * band's instance capacity (no host read).  Writes out_color's band pixels only. */
int gsr_band_forward(const gsr_camera* cam, const gsr_raster_settings* rs, int32_t nsrc, int32_t pair_cap,
                     const void* recv, float* out_color, gsr_alloc_fn alloc_geom, gsr_alloc_fn alloc_binning,
                     gsr_alloc_fn alloc_image, void* alloc_ctx, gsr_buffers* bufs, void* stream);

/* grad_send: nsrc x pair_cap x GSR_SPLAT_GRAD_BYTES (the received slot layout; zeros for empty
 * slots).  dL_dout_color: full image, only the band's pixels are read. */
int gsr_band_backward(const gsr_camera* cam, const gsr_raster_settings* rs, int32_t nsrc, int32_t pair_cap,
                      const gsr_buffers* bufs, const float* dL_dout_color, gsr_alloc_fn alloc_scratch,
                      void* alloc_ctx, void* grad_send, void* stream);

/* grad_recv: nbands x pair_cap x GSR_SPLAT_GRAD_BYTES (what gsr_band_backward wrote for this
 * shard, one block per band).  band_rows: the forward's.  grads: the shard's rows.  B2 sums
 * each Gaussian's returned rows in band order as it loads them (one launch; shard_state is
 * only read). */
int gsr_shard_backward(const gsr_camera* cam, const gsr_gaussians* shard, const gsr_raster_settings* rs,
                       int32_t nbands, const int32_t* band_rows, int32_t pair_cap, void* shard_state,
                       const void* grad_recv, const gsr_grads* grads, void* stream);

/* The step's glue around the exchanges, one launch each (what a caller would otherwise do with
 * ~20 small copies, reductions and clears per step):
 *   gsr_band_publish   this rank's row of the image all-gather: the band's pixel rows of
 *                      out_color (3 x H x W; tile rows rs->tile_y0..tile_y1) into row[0, 3*tall*W)
 *                      laid out 3 x tall x W, then at row + status_off (u32 words) the nbands
 *                      send-block header counts and the band's K (bufs: the band forward's)
 *   gsr_gather_finish  from `gathered` (world rows of row_floats floats, as the all-gather left
 *                      them): every rank's band pixels into image (3 x H x W); into *guard (device
 *                      int32) the number of ranks whose header counts exceed pair_cap or whose K
 *                      exceeds capacity -- the agreed overflow word, the same on every rank; and
 *                      nzero floats at `zero` cleared (e.g. the next step's row statistics, which
 *                      gsr_shard_forward accumulates into).  0 <= status_off, world <= 16 ranks. */
int gsr_band_publish(const gsr_camera* cam, const gsr_raster_settings* rs, int32_t tall, const float* out_color,
                     int32_t nbands, const void* send, int32_t pair_cap, const gsr_buffers* bufs, float* row,
                     int64_t status_off, void* stream);
int gsr_gather_finish(const gsr_camera* cam, int32_t world, const int32_t* band_rows, int32_t tall,
                      const float* gathered, int64_t row_floats, int64_t status_off, int32_t pair_cap,
                      int32_t capacity, float* image, int32_t* guard, float* zero, int64_t nzero, void* stream);

/* Introspection for tests / the benchmark (all device pointers into the caller's buffers,
 * or NULL when not applicable).  `what`: see gsr_view_* below. */
#define GSR_VIEW_SORTED_GID 1       /* uint32[K]: Gaussian id of sorted instance i       */
#define GSR_VIEW_SORTED_TILE 2      /* uint32[K]: tile id of sorted instance i (row-bucketed binning:
                                       filled from the ranges by this call between two device-wide
                                       synchronisations, so it follows the forward on whatever stream
                                       ran it, blocking or not; NULL while a stream is being captured) */
#define GSR_VIEW_RANGES 3           /* uint32[2*tiles]: [start,end) per tile               */
#define GSR_VIEW_FINAL_T 4          /* float[H*W]                                          */
#define GSR_VIEW_N_CONTRIB 5        /* retired (always NULL): the blend no longer keeps a   
                                       per-pixel contributor count; B1 re-derives the      
                                       termination point from T                             */
#define GSR_VIEW_DEPTH_KEY 6        /* uint32[P]: depth bits, 0xFFFFFFFF when culled       */
#define GSR_VIEW_TILES_TOUCHED 7    /* uint32[P]                                           */
#define GSR_VIEW_COUNTS 9           /* uint32[1]: K, written by the scan (device)          */
#define GSR_VIEW_TERM 10            /* uint32[tiles*GSR_TERM_STRIDE]: per tile the F6
                                       termination index, then the B1 chunk 1..31 start
                                       records (UINT32_MAX: no such chunk)                 */
#define GSR_TERM_STRIDE 32          /* words per tile of GSR_VIEW_TERM                     */
#define GSR_VIEW_CK_LIVE 11         /* uint8[slots*4]: per B1 checkpoint slot and 16x4
                                       pixel stripe, 1 where F6 wrote that stripe's
                                       checkpoint (0: it had finished).  Tile t's chunk
                                       c >= 1 (opened per GSR_VIEW_TERM) uses slot
                                       t*31 + c-1 when gsr_ck_pool_slots(cap, W, H) ==
                                       31*tiles, else floor(start_t / 48) + t + c-1, start_t
                                       = the tile's first index in the sorted list          */
#define GSR_VIEW_RECORDS 8          /* float4[3*P]: {x,y,a',b'},{c',o,r,g},{b,ext_x,ext_y,log2 o};
                                       a',b',c' = -log2(e) * (A/2, B, C/2) of the conic */
/* NULL (and gsr_last_error set) for buffers whose layout word is not a forward's. */
const void* gsr_view(const gsr_camera* cam, int32_t P, const gsr_buffers* bufs, int what);

/* Optional stage profiler (off by default; process-wide, mutex-protected).  When enabled,
 * every stage in `stage_mask` (bit i = stage i below) is bracketed by two hipEvents on the
 * call's stream; gsr_profile_read synchronises those events and returns the accumulated
 * milliseconds and launch counts per stage (arrays of GSR_NUM_STAGES), then resets. */
#define GSR_STAGE_PREPROCESS 0     /* F1 */
#define GSR_STAGE_DEPTH_SORT 1     /* per-tile depth order */
#define GSR_STAGE_SCAN 2           /* F2 scan of tiles_touched (gid order) */
#define GSR_STAGE_DUPLICATE 3      /* F3 (with the F2 scan when the two run as one kernel) */
#define GSR_STAGE_TILE_SORT 4      /* F4 tile-key LSD sort of the K instances */
#define GSR_STAGE_FINALIZE 5       /* F5 sorted gid + tile ranges */
#define GSR_STAGE_BLEND_FWD 6      /* F6 */
#define GSR_STAGE_BLEND_BWD 7      /* B1 */
#define GSR_STAGE_PREPROCESS_BWD 8 /* B2 */
#define GSR_STAGE_GATHER 9         /* per-Gaussian grad2d sum of the B1 partials */
#define GSR_STAGE_MISC 10          /* memsets, background fill, num_rendered read */
#define GSR_STAGE_EXCHANGE 11      /* multi-GPU splat pack / unpack / gradient sum */
#define GSR_NUM_STAGES 12
int gsr_profile_enable(uint32_t stage_mask);
int gsr_profile_read(double* ms, uint32_t* counts);
const char* gsr_stage_name(int stage);

/* Byte sizes the allocation callbacks will be asked for (for pre-sizing pools).  The binning
 * buffer holds the instance arrays for `capacity` instances and the B1 checkpoint slots (ABI >= 3:
 * min(31 per tile, capacity / 48 + tiles + 1) slots of 4 KB -- a chunk opens only after 192
 * visited (record, stripe) pairs, so a tile of n instances opens at most n / 48 -- instead of a
 * fixed 31 per tile in the image buffer). */
size_t gsr_geom_bytes(int32_t P);
size_t gsr_binning_bytes(int32_t capacity, int32_t width, int32_t height);
size_t gsr_ck_pool_slots(int32_t capacity, int32_t width, int32_t height);
size_t gsr_image_bytes(int32_t width, int32_t height);
size_t gsr_scratch_bytes(int32_t capacity);

#ifdef __cplusplus
}
#endif
#endif /* GSR_GSR_H */

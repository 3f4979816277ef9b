// gsr_kernels.h -- host-side launchers of the CDNA4 kernels (one per pipeline stage).
// Every launcher enqueues on `stream` and returns hipGetLastError() as an int.
#pragma once
#include <hip/hip_runtime.h>

#include "gsr_internal.h"

namespace gsr {

struct GaussIn {
    int P, D, M_rest;
    float smod;
    const float *means3D, *sh_dc, *sh_rest, *colors, *opac, *scales, *rots, *cov3D;
};

struct PreOut {
    int32_t* radii;
    uint32_t* depth_key;
    uint32_t* tiles;
    float4* rec;   // blend records: {x, y, a', b'}, {c', o, r, g}, {b, ext_x, ext_y, log2 o}
    uint4* rect;   // (minx | miny << 16, maxx | maxy << 16, inst_start (set by F3), 0)
    uint32_t* flags;     // nullable: SH clamp bits per Gaussian (B2 recomputes them when absent)
    uint32_t* counters;  // nullable, zeroed: [slot] += Gaussians with tiles in the band,
                         // [kCountSlots + slot] += K (slot = block % kCountSlots)
    uint32_t* rb_hist = nullptr;  // nullable (one view only): per 256-Gaussian block b, its pairs per
                                  // band row r at [r * blocks + b] (row-bucketed binning, pass A)
    uint32_t* bsum = nullptr;     // with rb_hist: per block b, its Gaussians' tiles_touched sum (the
                                  // F2 scan's block partials: launch_scan_blocks scans them)
};

// F1: projection, EWA cov2D, conic, radius, tile rect (clipped to the tile rows [ty0, ty1)),
// SH->RGB (bit-exact vs the oracle).  A Gaussian shard is `in` with every pointer advanced to
// its first Gaussian and P = its length (outputs are indexed by the shard-local index).
int launch_preprocess(const gsr_camera& cam, const GaussIn& in, int ty0, int ty1, const PreOut& out,
                      hipStream_t s);
// Cameras by value in the kernel arguments: one, or up to kMaxViews (views mode, grid.y = view).
template <int NV>
struct CamArg {
    gsr_camera c[NV];
};
// Views mode (gsr_forward_views): V <= kMaxViews views of the same size, one launch (grid.y =
// view); view v's outputs at entries v * P + g, its tiles / pixel rows offset into a tall image.
int launch_preprocess_views(const gsr_camera* cams, int V, const GaussIn& in, const PreOut& out, hipStream_t s);

// LSD radix sort of (u32 key, u32 value) by key bits [0, nbits); vals_in == nullptr means the
// identity permutation.  Ping-pongs between (k0,v0) and (k1,v1); returns in *which (0/1) where
// the sorted data ended.  Launched for `cap` items; n_dev (nullable) holds the live count
// (clamped to cap).  hist: sort_scratch_words(cap) u32.
int radix_sort(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* k0, uint32_t* v0,
               uint32_t* k1, uint32_t* v1, long long cap, const uint32_t* n_dev, int nbits, uint32_t* hist,
               int* which, hipStream_t s);

// F2: inclusive scan of tiles[0..n) (gid order) -> offsets and the total K -> *total_out
// (device), as three kernels for n > kFusedScanMax (nothing to do below: the fused kernel of
// launch_duplicate scans).  scan_partials_buf: sort_blocks(n) + 16 u32.
int launch_scan(const uint32_t* tiles, int n, uint32_t* offsets, uint32_t* scan_partials_buf, uint32_t* total_out,
                hipStream_t s, bool fused_ok = true);
// F3: inst_start (rect[g].z) and the emitted (tile key, gid) pairs in gid order, rect row-major,
// band rows from ty0 -- at most `cap` of them.  For n <= kFusedScanMax one look-back kernel
// also does F2 (offsets, *total_out); lookback: 16 + ceil(n / 256) u32.
int launch_duplicate(const uint32_t* tiles, uint4* rect, int n, int grid_x, int ty0, uint32_t* offsets,
                     uint32_t* lookback, uint32_t* tkey, uint32_t* tgid, long long cap, uint32_t* total_out,
                     hipStream_t s, bool scanned = false);  // scanned: the three-kernel scan already ran

// F2 from F1's block sums (PreOut.bsum, one per 256 Gaussians): the sums scanned in place
// (exclusive) and K into *total_out -- one launch; the per-Gaussian offsets then come from
// rb_rows_place, or from launch_block_offsets when the radix binning runs instead.
int launch_scan_blocks(uint32_t* bsum, int n, uint32_t* total_out, hipStream_t s);
int launch_block_offsets(const uint32_t* tiles, int n, const uint32_t* bsum, uint32_t* offsets, hipStream_t s);
// Row-bucketed binning (gsr_internal.h use_rb_binning): from the inclusive F2 scan `offsets`, F3
// (inst_start into rect.z), the stable tile sort of the instances and F5 -- the (tile key, gid)
// arrays tkey / tgid in (tile, gid) order and `ranges` (cleared beforehand) -- in two counting
// passes over (Gaussian, tile row) pairs.  histA: GeomLayout.rb_hist; histB: BinLayout.rb_hist;
// rb_status: ImgLayout.rb_status (cleared); pgid / pxr: cap u32 each of scratch.
int launch_rb_binning(const uint32_t* tiles, uint4* rect, uint32_t* offsets, int n, int gx, int ty0, int ty1,
                      uint32_t* histA, uint32_t* histB, uint32_t* rb_status, uint32_t* pgid, uint32_t* pxr,
                      uint32_t* tkey, uint32_t* tgid, uint2* ranges, long long cap, hipStream_t s,
                      bool rows_counted = false,     // rows_counted: F1 wrote histA (PreOut.rb_hist)
                      const uint32_t* bsum = nullptr,  // with it: F1's scanned block sums -- the
                                                         // placement writes `offsets` itself
                      uint32_t* K_dev = nullptr,       // set to UINT32_MAX if the look-back times out
                      const uint32_t* depth_key = nullptr,  // with ppair and tpair: the pairs go to ppair as
                      uint2* ppair = nullptr,               // (gid, depth key) (pgid unused; pxr any cap u32)
                      uint2* tpair = nullptr);              // and the instances to tpair as (gid, key), not tgid

// Per-tile depth order: every tile's slice of `gid` (tile-sorted, gid order within a tile) is
// sorted in place by (depth_key[gid], gid) -- the canonical (tile, depth, gid) order -- with a
// stable LDS radix sort of the depth keys.  Slices longer than the first kernel's LDS form are
// queued in `ovf` (count at *ovf_count, zeroed) for 8192-entry blocks, longer ones again in
// ovf2 for a global-memory form using scratch_hi / scratch_lo (K u32 each, free after the tile
// sort).  K: the binning's capacity (it sizes the LDS form from the mean slice).
// Presort mode (gsr_internal.h use_presort): the P depth keys sorted (stable, gid values), then
// each rank's (tiles, rect, gid) gathered into rank order with its 256-rank block's tiles_touched
// sum in bsum (div_up(n, 256) words), which are then scanned in place (exclusive) with the total
// K into *total_out.
int launch_depth_presort(const uint32_t* depth_key, const uint32_t* tiles, const uint4* rect, int n, uint32_t* dk0,
                         uint32_t* dv0, uint32_t* dk1, uint32_t* dv1, uint32_t* hist, uint32_t* rtiles, uint4* rrect,
                         uint32_t* bsum, uint32_t* total_out, hipStream_t s);
// F3 in rank order: each 256-rank block scans its rtiles from its offset bexcl[block] (writing
// `offsets`, the inclusive scan the gather reads) and writes inst_start into rect[gid].z.
int launch_duplicate_ranked(const uint32_t* rtiles, const uint4* rrect, uint4* rect, int n, int grid_x, int ty0,
                            const uint32_t* bexcl, uint32_t* offsets, uint32_t* tkey, uint32_t* tgid, long long cap,
                            hipStream_t s);
// Mean slices of up to ~1365 entries use the register form instead (one wave per slice of <= 1024
// entries, a 2048-entry wave for the queued longer ones where the mean is near 1024; the rest
// through the 1024-thread LDS form of tile_depth_sort_big).
int launch_tile_depth_sort(const uint2* ranges, int tile0, int ntiles, long long K, const uint32_t* depth_key,
                           uint32_t* gid, uint32_t* ovf, uint32_t* ovf_count, uint32_t* ovf2, uint32_t* ovf2_count,
                           uint32_t* done, uint32_t* scratch_hi, uint32_t* scratch_lo, hipStream_t s,
                           bool unordered = false, const uint2* src = nullptr);
// src (optional): the slices as placed (gid, depth key) pairs (the row-bucketed placement's tpair):
// the sort reads them coalesced, instead of gathering depth_key[gid], and writes the ordered gids
// to `gid` (the forms that sort in place get their slices' gids copied there first).
// unordered: the tiles' entries are in arbitrary order (row-bucketed binning), not gid order --
// the register form needs nothing else; the LDS forms then also sort by gid (LSD, gid passes first).
// True when the register form takes the mean slice (the row-bucketed binning is used only then).
bool tile_wave_sort_eligible(long long K, int ntiles);

// F5: ranges[tile] = [start, end) of the sorted tile keys (K = min(*K_dev, cap))
int launch_tile_keys_from_ranges(const uint2* ranges, int tiles, long long cap, uint32_t* tkey, hipStream_t s);
int launch_finalize(const uint32_t* sorted_tile, long long cap, const uint32_t* K_dev, uint2* ranges, hipStream_t s);

// F6: per-tile front-to-back blend -> colour, final T, colour sum without background, the
// tile's termination index term[], the B1 chunk checkpoints (ck: the binning buffer's
// ck_pool_slots(cap, tiles of the image) slots, chunk slot ck_slot_of(...), gsr_internal.h)
int launch_blend_forward(const gsr_camera& cam, const float bg[3], int ty0, int ty1,
                         const uint2* ranges, const uint32_t* sorted_gid, const float4* rec,
                         float* out_color, float* final_T, float* accum, uint32_t* term, float4* ck, long long cap,
                         hipStream_t s, int vgy = 0, int vh = 0, uint8_t* mk = nullptr);

// F6 writes term[t] (see kMaxChunks) and the B1 chunk checkpoints `ck` (ImgLayout.ck).
// B1: per-tile front-to-back gradients -> per-instance partial entry j (PartLayout(cap)), where
// the emission index j = inst_start[g] + row-major index of the tile in g's band-clipped rect.
// B1 writes the entries of the records that changed a pixel and sets their flag byte
// (PartLayout.fl); launch_clear_flags zeroes the flags (K bytes) and must precede it.  The
// gather reads only flagged entries, so the 36-B entries are never cleared.
int launch_clear_flags(float* partial, long long cap, hipStream_t s);
int launch_blend_backward(const gsr_camera& cam, const float bg[3], int ty0, int ty1,
                          const uint2* ranges, const uint32_t* sorted_gid, const uint4* rect,
                          const float4* rec, const float* final_T,
                          const float* accum, const float* dL_dpix, float* partial, long long cap,
                          const uint32_t* term, const float4* ck, hipStream_t s, int vgy = 0, int vh = 0,
                          const uint8_t* mk = nullptr, int split = 1);
// B1 parts per (tile, chunk) for a launch over tile rows [ty0, ty1) (views mode: vgy rows per
// view): 1 on full images, GSR_B1_BAND_SPLIT on band launches; the partial block then holds
// cap * split entries (entry j * split + part) and the gather sums them (launch_gather_grad2d)
int b1_split(int W, int H, int ty0, int ty1, int vgy);
// (vgy, vh: views mode -- bands of vgy tile rows per view, vh valid pixel rows each; 0 = one image)

// record layout constants shared by preprocess and the blend kernels
constexpr float kLn2 = 0.6931471805599453f;  // conic A = -2 ln2 a', B = -ln2 b', C = -2 ln2 c' 

// sum partials per Gaussian (emission order) -> grad2d (kPart floats per Gaussian; zeros for
// culled Gaussians).  offsets: the inclusive tile scan in gid order; partial: PartLayout(cap).
// rrect: the rank-order payload in presort mode (offsets then in rank order), else nullptr
int launch_gather_grad2d(const uint32_t* offsets, const float* partial, const float4* rec, int W, int H,
                         long long cap, int P, const uint4* rrect, float* grad2d, hipStream_t s, int split = 1);

struct GradOut {
    float *means2D, *conic, *opac, *colors, *means3D, *sh_dc, *sh_rest, *scales, *rots, *cov3D;
};

// B2: chain rule to the leaves for Gaussians [g0, g1) from their 2D gradients (grad2d, kPart
// floats each).  Inputs are indexed by g; grad2d and all outputs by g - g0.
int launch_preprocess_backward(const gsr_camera& cam, const GaussIn& in, int g0, int g1,
                               const uint32_t* depth_key, const uint32_t* flags, const float* grad2d,
                               const GradOut& out, hipStream_t s);
// Views mode: B2 of V views in one launch (grid.y = view) from the per-(view, Gaussian) entries
// v * P + g of depth_key / flags / grad2d; view v's 2D gradients (means2D, conic) go to rows
// v * P.. of out's, its leaf gradients to `out` (v = 0) or to slice v - 1 of `scratch` (P rows per
// slice), which launch_views_sum then adds to `out` in view order.
int launch_preprocess_backward_views(const gsr_camera* cams, int V, const GaussIn& in, const uint32_t* depth_key,
                                     const uint32_t* flags, const float* grad2d, const GradOut& out,
                                     const GradOut& scratch, hipStream_t s);
int launch_views_sum(const GaussIn& in, int V, const GradOut& out, const GradOut& scratch, hipStream_t s);

// ---- multi-GPU exchange (gsr_shard.hip) ----
// Shard side: pack every visible Gaussian of [0, P) into the send block of each band its rect
// overlaps (order-preserving; headers = true counts; slots past pair_cap dropped), remember the
// slots (slot_of[b * P + g]); row_hist (nullable) += per-tile-row instance counts.
// partials: (sort_blocks(P) + 1) * nbands u32.
int launch_pack_splats(const uint32_t* tiles, const uint4* rect, const uint32_t* depth_key, const float4* rec, int P,
                       const BandRows& br, uint32_t* partials, char* send, int pair_cap, uint32_t* slot_of,
                       uint32_t* row_hist, int grid_y, bool spans, hipStream_t s, uint32_t* rowpart = nullptr);
// Band side: nsrc received blocks -> local arrays of nsrc * pair_cap entries (empty slots: no tiles)
// rb_hist / bsum (nullable, together): the row-bucketed binning's pass-A row counts and the F2 scan's
// block partials per 256 slots, as F1 writes them for a single-GPU forward (PreOut.rb_hist / bsum)
int launch_unpack_splats(const char* recv, int nsrc, int pair_cap, int ty0, int ty1, float4* rec, uint32_t* depth_key,
                         uint32_t* tiles, uint4* rect, hipStream_t s, uint32_t* rb_hist = nullptr,
                         uint32_t* bsum = nullptr);

// The step's glue around the exchanges (gsr.h gsr_band_publish / gsr_gather_finish)
int launch_band_publish(const float* color, int W, int H, int py0, int py1, int tall, float* mine,
                        long long status_off, const char* send, size_t block_bytes, int nbands, const uint32_t* K_dev,
                        hipStream_t s);
int launch_gather_finish(const float* gathered, long long row_floats, long long status_off, int world,
                         const BandRows& br, int W, int H, int tall, float* image, uint32_t pair_cap,
                         uint32_t capacity, int32_t* guard, float* zero, int nzero, hipStream_t s);

// the bands [b_lo, b_hi] a rect's tile rows [miny, maxy) overlap (b_lo > b_hi: none)
__device__ __forceinline__ void band_span(const BandRows& br, uint32_t miny, uint32_t maxy, int& b_lo, int& b_hi) {
    b_lo = br.n;
    b_hi = -1;
    for (int b = 0; b < br.n; ++b) {
        if ((int)miny < br.row[b + 1] && (int)maxy > br.row[b]) {
            b_lo = b < b_lo ? b : b_lo;
            b_hi = b;
        }
    }
}

// The shard's returned 2D gradients as B2 reads them when the band sum is fused into it: g's
// row is the sum, in band order, of back[b][slot_of[b][g]] over the bands g was sent to .
struct BandSum {
    const uint32_t* tiles;
    const uint4* rect;
    const uint32_t* slot_of;
    const float4* back;
    int pair_cap;
    BandRows br;
};
int launch_preprocess_backward_banded(const gsr_camera& cam, const GaussIn& in, const uint32_t* depth_key,
                                      const uint32_t* flags, const BandSum& bs, const GradOut& out, hipStream_t s);

}  // namespace gsr

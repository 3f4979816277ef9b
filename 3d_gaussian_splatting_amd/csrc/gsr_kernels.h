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
};

// F1: projection, EWA cov2D, conic, radius, tile rect, SH->RGB (bit-exact vs the oracle)
int launch_preprocess(const gsr_camera& cam, const GaussIn& in, int ty0, int ty1, const PreOut& out,
                      hipStream_t s);
// A band's F1 leaves the record colours zero when they come from SH (only ~1/N of the rows
// are needed); launch_colour fills them for the band's compacted candidates `cand`.
bool colour_pass_needed(const gsr_camera& cam, const GaussIn& in, int ty0, int ty1);
int launch_colour(const gsr_camera& cam, const GaussIn& in, const uint32_t* cand, int n, float4* rec,
                  hipStream_t s);

// LSD radix sort of (u32 key, u32 value) by key bits [0, nbits); vals_in == nullptr means the
// identity permutation.  Ping-pongs between (k0,v0) and (k1,v1); returns in *which (0/1) where
// the sorted data ended.  hist: 256*(blocks+1)+256 u32.
// v2_in (nullable): a second value array carried along, ping-ponging between v2_0 / v2_1
// (reduce-then-scan passes only).
// depth_sort: selects the per-pass scheme (onesweep look-back for the P-key depth sort,
// reduce-then-scan for the K-key tile sort; gsr_sort.hip use_onesweep).
int radix_sort(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* k0, uint32_t* v0,
               uint32_t* k1, uint32_t* v1, long long n, int nbits, uint32_t* hist, int* which,
               hipStream_t s, bool depth_sort, const uint32_t* v2_in = nullptr, uint32_t* v2_0 = nullptr,
               uint32_t* v2_1 = nullptr);

// inclusive scan out[r] = sum_{q<=r} in[idx ? idx[q] : q]; partials: blocks+16 u32;
// iota_out (nullable): also writes iota_out[r] = r (the identity ranking)
int inclusive_scan_gather(const uint32_t* in, const uint32_t* idx, uint32_t* out, int n,
                          uint32_t* partials, hipStream_t s, uint32_t* iota_out = nullptr);

// Per-tile depth order: every tile's slice of `gid` (tile-sorted, gid order within a tile) is
// sorted in place by (depth_key[gid], gid) -- the canonical (tile, depth, gid) order.  Tiles
// of up to 1.5x the mean slice (pow2, 1024..8192) sort in LDS; larger ones are queued in `ovf`
// (count at *ovf_count, zeroed) and sorted by a second launch (LDS up to 8192, global
// scratch lo/hi beyond; the radix form queues those once more in ovf2 / *ovf2_count).  scratch_hi / scratch_lo: K u32 each, free after the tile sort.
// gid_ordered: each slice is in ascending gid order (stable tile sort of gid-order emissions),
// so a stable sort of the depth keys alone suffices (LDS radix form).  sdepth (nullable): the
// depth key of every sorted instance (carried through the tile sort); without it the keys are
// gathered per instance from depth_key[gid].
int launch_tile_depth_sort(const uint2* ranges, int tile0, int ntiles, long long K, const uint32_t* depth_key,
                           uint32_t* gid, uint32_t* ovf, uint32_t* ovf_count, uint32_t* ovf2, uint32_t* ovf2_count,
                           uint32_t* scratch_hi, uint32_t* scratch_lo, hipStream_t s, bool gid_ordered,
                           const uint32_t* sdepth = nullptr);

// Band candidates: the Gaussians with tiles[g] != 0, in gid order -> (depth key, gid) pairs
// and their count (device u32).  partials: sort_blocks(n) + 16 u32.
int compact_candidates(const uint32_t* tiles, const uint32_t* depth_key, int n, uint32_t* partials,
                       uint32_t* keys_out, uint32_t* gids_out, uint32_t* count_out, hipStream_t s);

// F3: emit (tile key, owner gid) for every (Gaussian, tile in band) in depth-rank order
// tcount (nullable): per-tile instance counts, += 1 per emitted instance (count binning);
// inst_depth (nullable): the owner's depth key per emitted instance (read from depth_key)
int launch_duplicate(const uint32_t* gid_by_rank, const uint32_t* offsets, const uint32_t* tiles,
                     uint4* rect, int P, int grid_x, int ty0, int ty1, uint32_t* tkey, uint32_t* inst_gid,
                     hipStream_t s, uint32_t* tcount = nullptr, const uint32_t* depth_key = nullptr,
                     uint32_t* inst_depth = nullptr);

// F2 + F3 fused (decoupled look-back scan): offsets (inclusive), inst_start, emitted
// (tile key, gid) pairs.  scratch: 16 + ceil(n / 256) u32 (zeroed here).
int launch_scan_duplicate(const uint32_t* gid_by_rank, const uint32_t* tiles, uint4* rect, int n,
                          int grid_x, int ty0, uint32_t* offsets, uint32_t* tkey, uint32_t* inst_gid,
                          uint32_t* scratch, hipStream_t s, uint32_t* tcount = nullptr,
                          const uint32_t* depth_key = nullptr, uint32_t* inst_depth = nullptr);

// Count binning: tcount[t] (t in [tile0, tile0 + ntiles)) holds the per-tile instance counts
// F3 added; one block scans them into `ranges` (turning each count into its tile's cursor),
// then every emitted instance (tkey[i], gid[i]) claims the next slot of its tile with a
// returning atomic -> stile / sgid grouped by tile (order inside a tile arbitrary until
// launch_tile_depth_sort).
int launch_tile_bins(const uint32_t* tkey, const uint32_t* gid, long long K, int tile0, int ntiles,
                     uint32_t* tcount, uint2* ranges, uint32_t* stile, uint32_t* sgid, hipStream_t s);

// F5: ranges[tile] = [start, end) of the sorted tile keys
int launch_finalize(const uint32_t* sorted_tile, long long K, uint2* ranges, hipStream_t s);

// F6: per-tile front-to-back blend -> colour, final T, colour sum without background; with
// ck != nullptr also the B1 chunk checkpoints (ImgLayout.ck, chunked_tiles)
int launch_blend_forward(const gsr_camera& cam, const float bg[3], int ty0, int ty1,
                         const uint2* ranges, const uint32_t* sorted_gid, const float4* rec,
                         float* out_color, float* final_T, float* accum, float4* ck, hipStream_t s);

// B1: per-tile front-to-back gradients -> per-instance partial entry j (PartLayout), where the
// emission index j = inst_start[g] + row-major index of the tile in g's band-clipped rect.
// `partial` is the base of a PartLayout(K) block.
// Zeroes the partial block launch_blend_backward fills (must precede it on the stream).
int launch_clear_partial(float* partial, long long K, hipStream_t s);
int launch_blend_backward(const gsr_camera& cam, const float bg[3], int ty0, int ty1,
                          const uint2* ranges, const uint32_t* sorted_gid, const uint4* rect,
                          const float4* rec, const float* final_T,
                          const float* accum, const float* dL_dpix, float* partial, long long K,
                          const float4* ck, hipStream_t s);

// record layout constants shared by preprocess and the blend kernels
constexpr float kLn2 = 0.6931471805599453f;  // conic A = -2 ln2 a', B = -ln2 b', C = -2 ln2 c' 

// sum partials per Gaussian (emission order) -> grad2d (kPart floats per Gaussian; zeros for
// culled Gaussians).  gid_by_rank / offsets: depth-sort permutation and inclusive tile scan.
int launch_gather_grad2d(const uint32_t* gid_by_rank, const uint32_t* offsets, const float* partial,
                         const float4* rec, int W, int H, long long K, int P, float* grad2d, hipStream_t s);

struct GradOut {
    float *means2D, *conic, *opac, *colors, *means3D, *sh_dc, *sh_rest, *scales, *rots, *cov3D;
};

// gather + B2 in one kernel for a full image whose ranking is the identity (gid order): the
// per-Gaussian 2D gradient never leaves registers.  Same results as launch_gather_grad2d
// followed by launch_preprocess_backward over [0, P).
int launch_gather_backward(const gsr_camera& cam, const GaussIn& in, const uint32_t* depth_key, const uint32_t* flags,
                           const uint32_t* offsets, const float* partial, const float4* rec, long long K,
                           const GradOut& out, hipStream_t s);

// B2: chain rule to the leaves for Gaussians [g0, g1) from their 2D gradients (grad2d, kPart
// floats each).  Inputs are indexed by g; grad2d and all outputs by g - g0.
int launch_preprocess_backward(const gsr_camera& cam, const GaussIn& in, int g0, int g1,
                               const uint32_t* depth_key, const uint32_t* flags, const float* grad2d,
                               const GradOut& out, hipStream_t s);

}  // namespace gsr

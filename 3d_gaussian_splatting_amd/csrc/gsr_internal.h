// gsr_internal.h -- buffer layouts and launch helpers shared by the C-ABI (gsr_api.cpp)
// and the kernels.  HBM layout (DESIGN.md "Data layout"):
//
//   geometry (per Gaussian, P):   depth_key u32 | tiles u32 | flags u32 | rec float4[3]
//                                 | rect uint4 (rect + inst_start) | offsets u32 | scan scratch
//   binning  (per instance, cap): tile key/val ping-pong 4 x u32 (values = Gaussian id)
//                                 | radix histogram
//   image    (per pixel / tile):  ranges uint2[tiles] | counters | sort queues | term
//                                 | final_T f32 | accum 3 x f32 | B1 chunk checkpoints
//   scratch  (backward, per cap): partial moments float4[2] | partial float  (indexed by emission j)
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/gsr/gsr.h"

namespace gsr {

constexpr int kTile = GSR_TILE;
constexpr int kSortBlock = 256;             // threads per radix-sort / scan block
constexpr int kSortItems = 16;              // items per thread
constexpr int kSortTile = kSortBlock * kSortItems;  // 4096 items per block
constexpr int kRecFloats = 12;              // 3 x float4 per Gaussian record
constexpr int kPart = GSR_GRAD2D_STRIDE;    // floats per partial / grad2d entry
constexpr int kCountSlots = 64;             // preprocess count partials (host sums them)
constexpr int kFusedScanMax = 1 << 19;      // Gaussian counts up to this scan + duplicate in one kernel

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }
inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }
inline int sort_blocks(long long n) { return n > 0 ? div_up(n, kSortTile) : 0; }
// multi-GPU splat packing: 256 threads x 1 round = 256 Gaussians per block (a 1/8 shard of 1M
// launches ~490 blocks).  Measured at 1M / 1080p, N = 8 (slowest rank, scripts/band_ab.sh):
// 1 round 0.386-0.388 ms, 2 rounds 0.398-0.404, 4 rounds 0.409-0.439, and a one-launch pack with
// a decoupled look-back 0.403-0.406 (slower still on whole-image shards: its look-back chain)
constexpr int kPackItems = 1;
constexpr int kPackTile = kSortBlock * kPackItems;
inline int pack_blocks(long long n) { return n > 0 ? div_up(n, kPackTile) : 0; }
// reduce-then-scan radix-sort scratch (u32 words): 256 digit columns of (blocks + 1) counts
// plus 256 digit totals
// LSD radix passes (tile keys, Morton codes): kRadixItems rounds of 64 per wave (4096 keys
// per block; 2048 measured slower: 0.137 vs 0.120 ms for the 1M / 1080p tile sort)
constexpr int kRadixItems = 16;
constexpr int kRadixTile = kSortBlock * kRadixItems;
// Sorts of fewer than kRadixSmallN keys (multi-GPU band launches, ~1M keys at 1M / 1080p, N = 8)
// use 1024-key blocks (kRadixItemsSmall rounds per wave), so that they still launch several
// blocks per CU.
#ifndef GSR_RADIX_SMALL_N
#define GSR_RADIX_SMALL_N (1 << 21)
#endif
constexpr long long kRadixSmallN = GSR_RADIX_SMALL_N;
constexpr int kRadixItemsSmall = 4;
inline int radix_tile_for(long long n) { return n < kRadixSmallN ? kSortBlock * kRadixItemsSmall : kRadixTile; }
inline int radix_blocks(long long n) { return n > 0 ? div_up(n, radix_tile_for(n)) : 0; }
inline size_t sort_scratch_words(long long n) { return 256 * ((size_t)radix_blocks(n) + 1) + 256; }

// lengths and emission index bases are u32: n instances must stay below 2^32, and the blend's
// per-tile index arithmetic below 2^31
// Global depth pre-sort: at and above kPresortMin Gaussians (or splat slots) the binning sorts
// the Gaussians by their 32-bit depth key once (stable LSD, gid as value) and emits the
// instances in that (depth, gid) rank order, so the stable tile-key sort that follows leaves
// every tile's slice already in canonical (tile, depth, gid) order and the per-tile depth sort
// goes away.  Each rank's binning payload (tiles, rect, gid) is gathered once into rank order
// (rtiles / rrect) so the scan, F3 and the gather stream it coalesced.  Below the threshold the
// fused look-back scan + duplicate and the per-tile sort are kept (small scenes).
// Measured at 1M / 1080p: presort 0.114 (sort + payload + block scan) + F3 0.028 + gather 0.097
// (its records / grad2d rows are random by gid in rank order) = 0.239 ms, against 0.211 for the
// per-tile order (0.102 + scan 0.018 + 0.021 + 0.070): it pays only where the per-tile sort's
// cost grows faster (5M: 0.49 ms), hence the 2^21 threshold.
// Round 5: with the row-bucketed binning below it, the pre-sort pays only where tiles are deep:
// it is taken when, besides, there are more than kPresortPerTile Gaussians per tile of the
// image (a proxy for the mean slice, which is not known before the scan).  Measured (iters/s,
// pre-sort vs row-bucketed): 5M / 1080p (613 per tile) 344 vs 367; 3M / 1280x832 (721) 577 vs
// 577; 6M / 1280x832 (1442) 329 vs 281.
#ifndef GSR_PRESORT_MIN
#define GSR_PRESORT_MIN ((1 << 21) + 1)
#endif
#ifndef GSR_PRESORT_PER_TILE
#define GSR_PRESORT_PER_TILE 700
#endif
constexpr long long kPresortMin = GSR_PRESORT_MIN;
constexpr long long kPresortPerTile = GSR_PRESORT_PER_TILE;
constexpr int kMaxViews = 8;  // gsr_forward_views: views per call (= GSR_MAX_VIEWS)
// Row-bucketed binning (gsr_sort.hip): images of at most kRbMaxRows x kRbMaxCols tiles outside
// presort mode; chunks of kRbChunkPairs (Gaussian, row) pairs in its second pass.
#ifndef GSR_RB_BIN
#define GSR_RB_BIN 1
#endif
// GSR_RB_TILE_KEYS 1: the row-bucketed placement writes every instance's tile key in the step
// (0: the GSR_VIEW_SORTED_TILE accessor fills them from the ranges when asked)
#ifndef GSR_RB_TILE_KEYS
#define GSR_RB_TILE_KEYS 0
#endif
// GSR_RB_SORT_KEYS 1: the row-bucketed placement writes every instance's depth key beside its gid
// (into the tile-key array kA, free in that mode), so the per-tile sort that follows reads its keys
// coalesced instead of through a dependent depth_key[gid] gather per entry (round 6)
#ifndef GSR_RB_SORT_KEYS
#define GSR_RB_SORT_KEYS 1
#endif
// GSR_RB_DEEP 0: only where the per-tile sort takes its register form (mean slices <= ~1365)
#ifndef GSR_RB_DEEP
#define GSR_RB_DEEP 1
#endif
constexpr int kRbMaxRows = 256, kRbMaxCols = 256, kRbChunkPairs = 1024;
// the binning's row scan splits a row into at most this many column partitions (gsr_sort.hip)
#ifndef GSR_RB_SCAN_SPLIT
#define GSR_RB_SCAN_SPLIT 16
#endif
constexpr int kRbScanSplit = GSR_RB_SCAN_SPLIT;
constexpr long long kRbMaxCap = 1LL << 30;  // the look-back's 30-bit counts (rb_tiles_scan)
// gsr_buffers.layout (set by the forward, checked by every later use of the buffers): the tag
// and the binning in use (gsr.h GSR_LAYOUT_*)
constexpr uint32_t kBufRowBucketed = GSR_LAYOUT_ROW_BUCKETED;
constexpr uint32_t kBufPresort = GSR_LAYOUT_PRESORT;
// the pre-sort's buffers (GeomLayout: sized from n alone) / the pre-sort itself for an image of
// gx x gy tiles
inline bool presort_possible(long long n) { return n >= kPresortMin; }
inline bool use_presort(long long n, int gx, int gy) {
    return presort_possible(n) && n > kPresortPerTile * (long long)gx * gy;
}
inline bool use_rb_binning(long long n, int gx, int gy) {
    return GSR_RB_BIN && !use_presort(n, gx, gy) && gx <= kRbMaxCols && gy <= kRbMaxRows;
}

struct GeomLayout {
    size_t depth_key, tiles, flags, rec, rect, offsets, partials, lookback, rb_hist, total;
    size_t dk0 = 0, dv0 = 0, dk1 = 0, dv1 = 0, dhist = 0, rtiles = 0, rrect = 0;  // presort only
    GeomLayout(long long P) {
        size_t o = 0, n = (size_t)(P > 0 ? P : 1);
        auto take = [&](size_t bytes) { size_t r = o; o += align_up(bytes); return r; };
        depth_key = take(4 * n);
        tiles = take(4 * n);
        flags = take(4 * n);  // SH clamp bits (B2 reads them instead of recomputing the colour)
        rec = take(16 * 3 * n);
        rect = take(16 * n);  // uint4: minx|miny<<16, maxx|maxy<<16, inst_start, 0
        offsets = take(4 * n);
        partials = take(4 * ((size_t)sort_blocks(n) + 16));  // three-kernel scan
        lookback = take(4 * (16 + (n + 255) / 256));        // fused scan + duplicate; presort: block sums
        rb_hist = take(4 * (256 * ((n + 255) / 256) + 256));  // row-bucketed binning: [row][block] + row totals
        if (presort_possible(P)) {
            dk0 = take(4 * n);
            dv0 = take(4 * n);
            dk1 = take(4 * n);
            dv1 = take(4 * n);
            dhist = take(4 * sort_scratch_words(n));
            rtiles = take(4 * n);   // tiles_touched in rank order
            rrect = take(16 * n);   // uint4 (rect lo, rect hi, gid, 0) in rank order
        }
        total = o;
    }
};

// Chunked B1: F6 checkpoints every pixel's (T, colour sum) at up to kMaxChunks - 1 points of each
// tile's list, so B1 sweeps the chunks of one tile in parallel blocks (a shorter tail; essential
// for multi-GPU bands, which hold 1/N of the tiles).  The points are chosen by B1's own cost:
// F6 counts the (record, stripe) pairs B1 will visit -- a record's stripe mask against the
// stripes still live -- and starts a new chunk at the first 64-record boundary where the
// current chunk holds kChunkWork of them.  Chunks are therefore balanced in work whatever the
// list length, no checkpoint is written past the tile's termination (every pixel finished),
// and the per-tile chunk table (term[]) tells B1 where each chunk starts.
#ifndef GSR_MAX_CHUNKS
#define GSR_MAX_CHUNKS 32
#endif
constexpr int kMaxChunks = GSR_MAX_CHUNKS;
// B1 batch window: mask bytes per lane (gsr_blend.hip)
#ifndef GSR_B1_WIN
#define GSR_B1_WIN 4
#endif  // = GSR_TERM_STRIDE (gsr.h) in the shipped build

// Checkpoint slots.  A checkpoint is 4 KB (float4 (T, C) per pixel of a tile).  A chunk opens
// only after kChunkWork visited (record, stripe) pairs and a record has at most 4 stripes, so a
// tile of n records opens at most floor(n / kCkDiv) chunks (kCkDiv = kChunkWork / 4 = 48).  Tile
// t's chunk c >= 1 therefore takes slot  floor(start_t / kCkDiv) + t + (c - 1)  (start_t: the
// tile's first index in the sorted list): the tiles' slot ranges never overlap, no counter or
// atomic is needed, and the slots in use are bounded by K / kCkDiv + tiles -- instead of a
// fixed 31 per tile (1.0 GB at 1080p, 4.1 GB at 4K, whether or not a chunk opens).  When that
// bound is larger than the fixed array anyway (deep lists: > 31 * 48 instances per tile on
// average, e.g. 5M / 1080p), the fixed layout t * 31 + (c - 1) is used.
// B1 chunk size in (record, stripe) pairs (measured in gsr_blend.hip), and for band launches
#ifndef GSR_CHUNK_WORK
#define GSR_CHUNK_WORK 192
#endif
#ifndef GSR_BAND_CHUNK_WORK
#define GSR_BAND_CHUNK_WORK GSR_CHUNK_WORK
#endif
constexpr int kChunkWork = GSR_CHUNK_WORK;
constexpr int kBandChunkWork = GSR_BAND_CHUNK_WORK;
constexpr int kCkDiv = (kChunkWork < kBandChunkWork ? kChunkWork : kBandChunkWork) / 4;  // records per possible open
__host__ __device__ inline bool ck_fixed_layout(long long cap, long long tiles) {
    return cap / kCkDiv + tiles + 1 >= tiles * (kMaxChunks - 1);
}
inline size_t ck_pool_slots(long long cap, long long tiles) {
    const long long t = tiles > 0 ? tiles : 1, c = cap > 0 ? cap : 0;
    return (size_t)(ck_fixed_layout(c, t) ? t * (kMaxChunks - 1) : c / kCkDiv + t + 1);
}
__host__ __device__ inline size_t ck_slot_of(bool fixed, uint32_t start, int tile, int chunk) {
    return fixed ? (size_t)tile * (kMaxChunks - 1) + (chunk - 1) : (size_t)(start / kCkDiv) + tile + (chunk - 1);
}

// Binning for up to `cap` instances (the exact K, or a caller-given bound) of an image of
// `tiles` tiles.  The tile-key sort ping-pongs (kA, vA) <-> (kB, vB); F3 emits into (kA, vA).
// Then the checkpoint slots: ck_slots x 256 float4, and one live byte per (slot, 16x4 stripe).
struct BinLayout {
    size_t kA, vA, kB, vB, hist, rb_hist, ck, ckm, mk = 0, total, ck_slots;
    BinLayout(long long cap, long long tiles) {
        size_t o = 0, n = (size_t)(cap > 0 ? cap : 1);
        auto take = [&](size_t bytes) { size_t r = o; o += align_up(bytes); return r; };
        kA = take(4 * n);
        vA = take(4 * n);
        kB = take(4 * n);
        vB = take(4 * n);
        hist = take(4 * sort_scratch_words(n));
        // row-bucketed binning: [column][chunk] counts of every row's chunks of kRbChunkPairs pairs
        rb_hist = take(4 * (size_t)kRbMaxCols * (n / kRbChunkPairs + 1 + kRbMaxRows));
        ck_slots = ck_pool_slots(cap, tiles);
        ck = take(ck_slots * 256 * 16);
        ckm = take(ck_slots * 4);
        // F6's stripe mask of every list entry it loads (one byte each), from which B1 picks the
        // entries it has to visit before loading any record (+ B1's 256-entry window past the end)
        mk = take(n + 64 * GSR_B1_WIN);  // B1 reads whole windows of 64 * GSR_B1_WIN bytes
        total = o;
    }
};

struct ImgLayout {
    size_t ranges, counters, rb_status, done, ovf, ovf2, term, final_T, accum, total;
    static size_t tile_count(int W, int H) {
        const size_t t = (size_t)div_up(W, kTile) * div_up(H, kTile);
        return t ? t : 1;
    }
    ImgLayout(int W, int H) {
        size_t o = 0;
        auto take = [&](size_t bytes) { size_t r = o; o += align_up(bytes); return r; };
        const size_t tiles = tile_count(W, H);
        size_t pix = (size_t)W * H;
        ranges = take(8 * tiles);
        counters = take(4 * (2 * kCountSlots + 16));  // ranges, counters, rb_status and done are
        rb_status = take(4 * (16 + kRbMaxRows * kRbScanSplit));  // contiguous: one memset clears them
        done = take(4 * tiles);  // (rb_status: the row-bucketed binning's ticket + look-back words;
                                 // done: chunks sorted per queued tile)
        ovf = take(4 * tiles);   // tiles the per-tile depth sort hands to its larger
        ovf2 = take(4 * tiles);  // forms (queues: the 8192-entry form, then the 16384-entry / chunked one)
        term = take(4 * tiles * kMaxChunks);  // F6: per tile [termination index, chunk 1..kMaxChunks-1 starts]
        final_T = take(4 * (pix ? pix : 1));
        accum = take(12 * (pix ? pix : 1));  // colour sum without background, 3 x H x W
        total = o;
    }
};

// B1 output, one entry per (tile, instance) at emission index j: 8 floats (two float4:
// d mean2D x/y, d conic A/B/C, d opacity, d colour r/g) and a ninth float (d colour b) in a
// separate array, so the entry is 36 B and every store/load stays 16-B aligned.
// `fl`: one byte per entry, 1 where B1 wrote the entry (a record that changed a pixel).  Only
// the flags are zeroed before B1 (K bytes instead of the 36-B entries), and the gather reads
// the entries whose flag is set.
struct PartLayout {
    size_t p8, p1, fl, total;
    explicit PartLayout(long long K) {
        const size_t n = (size_t)(K > 0 ? K : 1);
        p8 = 0;
        p1 = align_up(32 * n);
        fl = p1 + align_up(4 * n);
        total = fl + align_up(n);
    }
};

// ---- multi-GPU exchange (gsr_shard.hip) ----
constexpr int kMaxBands = 16;       // tile-row bands (ranks) of one exchange
constexpr int kMaxHistRows = 4096;  // tile rows the per-row instance histogram covers
constexpr int kSplatBytes = GSR_SPLAT_BYTES;
constexpr int kSplatGradBytes = GSR_SPLAT_GRAD_BYTES;
static_assert(kSplatGradBytes == 4 * kPart, "a returned splat gradient is one grad2d row");
inline size_t exchange_block_bytes(long long pair_cap) { return (size_t)kSplatBytes * (1 + (size_t)pair_cap); }

// tile-row bounds of the bands: band b = rows [row[b], row[b + 1])
struct BandRows {
    int n;
    int row[kMaxBands + 1];
};

// State a shard keeps from gsr_shard_forward to gsr_shard_backward: its geometry (F1), the slot
// each splat took in each band's send block and the pack's per-block counts (B2 sums the
// returned 2D gradients itself: launch_preprocess_backward_banded).
struct ShardLayout {
    size_t slot_of, partials, total;
    GeomLayout geo;
    ShardLayout(long long P, int nbands) : geo(P) {
        size_t o = geo.total;
        const size_t n = (size_t)(P > 0 ? P : 1);
        auto take = [&](size_t bytes) { size_t r = o; o += align_up(bytes); return r; };
        slot_of = take(4 * n * (size_t)nbands);
        partials = take(4 * ((size_t)pack_blocks(n) + 1) * (size_t)nbands);
        total = o;
    }
};

// counters[] slots past the preprocess partials (2 x kCountSlots)
constexpr int kTotalSlot = 2 * kCountSlots;          // K = sum of tiles_touched, written by the scan
constexpr int kOvfCountSlot = 2 * kCountSlots + 8;   // tiles queued for the large per-tile depth sort
constexpr int kOvf2CountSlot = 2 * kCountSlots + 9;  // ... then for its 16384-entry / chunked form

// number of 8-bit LSD passes to sort tile ids of a grid with `tiles` tiles
inline int tile_bits(int tiles) {
    int b = 1;
    while ((1ll << b) < tiles) ++b;
    return b;
}
inline int tile_passes(int tiles) { return (tile_bits(tiles) + 7) / 8; }

template <class T>
inline T* at(void* base, size_t off) { return reinterpret_cast<T*>(static_cast<char*>(base) + off); }
template <class T>
inline const T* at(const void* base, size_t off) {
    return reinterpret_cast<const T*>(static_cast<const char*>(base) + off);
}

}  // namespace gsr

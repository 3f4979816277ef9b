// gsr_internal.h -- buffer layouts and launch helpers shared by the C-ABI (gsr_api.cpp)
// and the kernels.  HBM layout (DESIGN.md "Data layout"):
//
//   geometry (per Gaussian, P):   depth_key u32 | tiles u32 | rec float4[3]
//                                 | rect uint4 (rect + inst_start) | cand_tmp u32 | offsets u32
//                                 | sort ping-pong 4 x u32
//                                 | radix histogram (256 x blocks) | scan partials
//   binning  (per instance, K):   tile key/val ping-pong 4 x u32 (values = Gaussian id)
//                                 | inst_gid u32 (emission order) | depth key ping-pong 2 x u32
//                                 | radix histogram
//   image    (per pixel):         ranges uint2[tiles] | counters | final_T f32 | accum 3 x f32
//   scratch  (backward, per K):   partial moments float4[2] | partial float  (indexed by emission j)
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/gsr/gsr.h"

namespace gsr {

constexpr int kTile = GSR_TILE;
constexpr int kSortBlock = 256;             // threads per radix-sort / scan block
constexpr int kSortItems = 16;              // items per thread
constexpr int kSortTile = kSortBlock * kSortItems;  // 4096 items per block
constexpr int kRecFloats = 12;              // 3 x float4 per Gaussian record
constexpr int kPart = GSR_GRAD2D_STRIDE;    // floats per partial / grad2d entry
constexpr int kCountSlots = 64;             // preprocess count partials (host sums them)

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }
inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }
inline int sort_blocks(long long n) { return n > 0 ? div_up(n, kSortTile) : 0; }
// radix-sort scratch (u32 words): reduce-then-scan needs 256 x (blocks + 1) + 256; onesweep
// needs 4 x 256 digit totals + 16 tickets + 4 passes x tiles x 256 look-back words, with
// tiles of 1024 keys (the small-n form) in the worst case.
constexpr long long kOnesweepSmall = 1 << 19;  // key counts up to this use 1024-key tiles
inline size_t sort_scratch_words(long long n) {
    const size_t nb = (size_t)sort_blocks(n) + 1;
    const size_t nbs = (size_t)(n > 0 ? (n + 1023) / 1024 : 0) + 1;
    const size_t a = 256 * nb + 256, b = 4 * 256 + 16 + 4 * (nbs > nb ? nbs : nb) * 256;
    return a > b ? a : b;
}

struct GeomLayout {
    size_t depth_key, tiles, flags, rec, rect, cand_tmp, offsets, sA_k, sA_v, sB_k, sB_v, hist,
        partials, total;
    GeomLayout(int P) {
        size_t o = 0, n = (size_t)(P > 0 ? P : 1);
        auto take = [&](size_t bytes) { size_t r = o; o += align_up(bytes); return r; };
        depth_key = take(4 * n);
        tiles = take(4 * n);
        flags = take(4 * n);  // SH clamp bits (full-image forwards; bands let B2 recompute)
        rec = take(16 * 3 * n);
        rect = take(16 * n);  // uint4: minx|miny<<16, maxx|maxy<<16, inst_start, 0
        cand_tmp = take(4 * n);  // band compaction: candidate gids before the depth sort
        offsets = take(4 * n);
        sA_k = take(4 * n);
        sA_v = take(4 * n);
        sB_k = take(4 * n);
        sB_v = take(4 * n);
        hist = take(4 * sort_scratch_words(n));
        partials = take(4 * ((size_t)sort_blocks(n) + 16));
        total = o;
    }
};

struct BinLayout {
    size_t kA, vA, kB, vB, inst_gid, dA, dB, hist, total;
    BinLayout(long long K) {
        size_t o = 0, n = (size_t)(K > 0 ? K : 1);
        auto take = [&](size_t bytes) { size_t r = o; o += align_up(bytes); return r; };
        kA = take(4 * n);
        vA = take(4 * n);
        kB = take(4 * n);
        vB = take(4 * n);
        inst_gid = take(4 * n);
        dA = take(4 * n);  // per-instance depth keys carried through the tile sort (ping-pong)
        dB = take(4 * n);
        hist = take(4 * sort_scratch_words(n));
        total = o;
    }
};

// Chunked B1: F6 checkpoints every pixel's (T, colour sum) at kMaxChunks - 1 points of each
// tile's list, so B1 sweeps the chunks of one tile in parallel blocks.  Essential for the
// multi-GPU bands (1/N of the tiles: B1 0.27 -> 0.13 ms at N = 8) and still -7 % B1 on a full
// 1080p image (shorter tail), for 16 B per pixel per checkpoint of extra F6 writes.
constexpr int kMaxChunks = 8;
constexpr int kChunkTiles = 1 << 30;  // launches with fewer tiles than this are chunked
inline int chunked_tiles(int W, int ty0, int ty1) {
    const char* e = std::getenv("GSR_CHUNK");  // A/B switch: 0 never, 2 always (bench/ablation only)
    const int mode = e ? std::atoi(e) : 1;
    const int nwg = (ty1 - ty0) * div_up(W, kTile);
    if (mode == 0 || nwg <= 0) return 0;
    return mode == 2 || nwg < kChunkTiles ? nwg : 0;
}

struct ImgLayout {
    size_t ranges, counters, tcount, ovf, ovf2, final_T, accum, ck, total;
    ImgLayout(int W, int H, int ck_tiles = 0) {
        size_t o = 0;
        auto take = [&](size_t bytes) { size_t r = o; o += align_up(bytes); return r; };
        size_t tiles = (size_t)div_up(W, kTile) * div_up(H, kTile);
        size_t pix = (size_t)W * H;
        ranges = take(8 * (tiles ? tiles : 1));
        counters = take(4 * (2 * kCountSlots + 16));  // ranges, counters and tcount are
        tcount = take(4 * (tiles ? tiles : 1));       // contiguous: one memset clears all three
        // (tcount: per-tile instance counts from F3, then the count binning's scatter cursors)
        ovf = take(4 * (tiles ? tiles : 1));   // tiles the per-tile depth sort hands to its larger
        ovf2 = take(4 * (tiles ? tiles : 1));  // forms (two queues: LDS, then global memory)
        final_T = take(4 * (pix ? pix : 1));
        accum = take(12 * (pix ? pix : 1));  // colour sum without background, 3 x H x W
        ck = take((size_t)ck_tiles * (kMaxChunks - 1) * 256 * 16);  // float4 (T, C) checkpoints
        total = o;
    }
};

// B1 output, one entry per (tile, instance) at emission index j: 8 floats (two float4:
// d mean2D x/y, d conic A/B/C, d opacity, d colour r/g) and a ninth float (d colour b) in a
// separate array, so the entry is 36 B and every store/load stays 16-B aligned.
struct PartLayout {
    size_t p8, p1, total;
    explicit PartLayout(long long K) {
        const size_t n = (size_t)(K > 0 ? K : 1);
        p8 = 0;
        p1 = align_up(32 * n);
        total = p1 + align_up(4 * n);
    }
};

// counters[] slots past the preprocess partials (2 x kCountSlots)
constexpr int kCandCountSlot = 2 * kCountSlots;      // band candidate count (compaction)
constexpr int kOvfCountSlot = 2 * kCountSlots + 8;   // tiles queued for the large per-tile depth sort
constexpr int kOvf2CountSlot = 2 * kCountSlots + 9;  // ... and for its global-memory form

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

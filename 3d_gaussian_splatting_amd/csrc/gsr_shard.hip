// gsr_shard.hip -- the multi-GPU split of the path (the scaling version): pack the
// projected Gaussians ("splats") of a Gaussian shard into per-band send blocks, unpack the
// blocks a band owner receives into its local geometry arrays.  (The 2D gradients the bands
// send back are summed per Gaussian, in band order, by B2 itself: gsr_preprocess_bwd.hip.)
//
// Splat (64 B, GSR_SPLAT_BYTES): the F1 blend record (3 float4) and {depth key, rect lo,
// rect hi, 0}.  A band owner needs nothing else: its binning (F2..F5), blend (F6) and blend
// backward (B1 + gather) read only these.  Splats of one (source, band) pair are packed in
// shard order by an order-preserving compaction (wave64 ballot prefix per band), and sources
// are laid out in rank order, so a band's local index order is ascending global Gaussian id:
// the canonical (tile, depth, gid) order -- and every pixel -- equal the single-GPU forward's.
//
// All integer / copy work: HBM-bound, no MFMA.
#include "gsr_kernels.h"

namespace gsr {
namespace {

constexpr int kB = kSortBlock;   // 256 threads
constexpr int kI = kPackItems;   // rounds of 64 per wave: kPackTile Gaussians per block
constexpr int kWaves = kB / 64;

__device__ inline uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return (lane == 0) ? 0ull : (~0ull >> (64 - lane));
}

// Per block: splats per band (partials[b * nblk + blk]); optionally the per-tile-row instance
// histogram (LDS, then one global add per row).  SPANS: also the per-row counts of the visible
// Gaussians whose rect starts / ends in that row (row_hist[gy + y]: first tile row y;
// row_hist[2 gy + y]: last tile row y) -- from which the splats any band cut would receive
// follow exactly: #(miny < r1) - #(maxy <= r0) (the live re-plan of the multi-GPU step).
// With rowpart (at most 256 histogram rows), each block stores its rows there ([row][block],
// the F1 row-count region, unused by a shard) and pack_scan_kernel sums them: one global atomic
// per row instead of one per (block, row) -- thousands of blocks adding to the same ~200
// addresses serialise at the L2 (~20 us at 625k Gaussians per shard).
template <bool SPANS>
__global__ __launch_bounds__(kB) void pack_count_kernel(const uint32_t* __restrict__ tiles,
                                                        const uint4* __restrict__ rect, int P, BandRows br,
                                                        uint32_t* __restrict__ partials, int nblk,
                                                        uint32_t* __restrict__ row_hist, int grid_y,
                                                        uint32_t* __restrict__ rowpart) {
    __shared__ uint32_t cnt[kWaves][kMaxBands];
    __shared__ uint32_t hist[(SPANS ? 3 : 1) * kMaxHistRows];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool do_hist = row_hist != nullptr;
    const int hrows = (SPANS ? 3 : 1) * grid_y;
    if (do_hist)
        for (int y = threadIdx.x; y < hrows; y += kB) hist[y] = 0u;
    __syncthreads();
    uint32_t c[kMaxBands];
#pragma unroll
    for (int b = 0; b < kMaxBands; ++b) c[b] = 0u;
    const int base = blockIdx.x * kPackTile + w * (kI * 64);
    for (int r = 0; r < kI; ++r) {
        const int g = base + r * 64 + lane;
        int b_lo = kMaxBands, b_hi = -1;
        if (g < P && tiles[g] != 0u) {
            const uint4 rr = rect[g];
            const uint32_t miny = rr.x >> 16, maxy = rr.y >> 16;
            band_span(br, miny, maxy, b_lo, b_hi);
            if (do_hist) {
                const uint32_t wd = (rr.y & 0xFFFF) - (rr.x & 0xFFFF);
                for (uint32_t y = miny; y < maxy; ++y) atomicAdd(&hist[y], wd);
                if constexpr (SPANS) {
                    atomicAdd(&hist[grid_y + miny], 1u);
                    atomicAdd(&hist[2 * grid_y + maxy - 1], 1u);
                }
            }
        }
#pragma unroll
        for (int b = 0; b < kMaxBands; ++b)
            if (b < br.n) c[b] += (uint32_t)__popcll(__ballot(b >= b_lo && b <= b_hi));
    }
    if (lane == 0)
        for (int b = 0; b < br.n; ++b) cnt[w][b] = c[b];
    __syncthreads();
    if (threadIdx.x < br.n) {
        uint32_t t = 0;
        for (int k = 0; k < kWaves; ++k) t += cnt[k][threadIdx.x];
        partials[threadIdx.x * nblk + blockIdx.x] = t;
    }
    if (do_hist && rowpart)
        for (int y = threadIdx.x; y < hrows; y += kB) rowpart[(size_t)y * nblk + blockIdx.x] = hist[y];
    else if (do_hist)
        for (int y = threadIdx.x; y < hrows; y += kB)
            if (hist[y]) atomicAdd(row_hist + y, hist[y]);
}

// Block b: exclusive scan of band b's per-block counts in place; the band's total into its send
// block's header (the true count, which may exceed pair_cap).
// Blocks past the bands: histogram row (blockIdx.x - nbands) summed over the count blocks
// (rowpart), added to row_hist.
__global__ __launch_bounds__(1024) void pack_scan_kernel(uint32_t* __restrict__ partials, int nblk,
                                                         char* __restrict__ send, size_t block_bytes, int nbands,
                                                         const uint32_t* __restrict__ rowpart,
                                                         uint32_t* __restrict__ row_hist) {
    __shared__ uint32_t wsum[16];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    if ((int)blockIdx.x >= nbands) {  // block-uniform
        const int y = (int)blockIdx.x - nbands;
        const uint32_t* row = rowpart + (size_t)y * nblk;
        uint32_t t = 0;
        for (int i = tid; i < nblk; i += 1024) t += row[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
        if (lane == 0) wsum[w] = t;
        __syncthreads();
        if (tid == 0) {
            uint32_t sum = 0;
            for (int k = 0; k < 16; ++k) sum += wsum[k];
            if (sum) atomicAdd(row_hist + y, sum);
        }
        return;
    }
    uint32_t* col = partials + (size_t)blockIdx.x * nblk;
    uint32_t carry = 0;
    for (int base = 0; base < nblk; base += 1024) {
        const int i = base + tid;
        const uint32_t v = i < nblk ? col[i] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int k = 0; k < 16; ++k) {
            pre += k < w ? wsum[k] : 0u;
            tot += wsum[k];
        }
        if (i < nblk) col[i] = carry + pre + x - v;
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) {
        uint32_t* hdr = reinterpret_cast<uint32_t*>(send + (size_t)blockIdx.x * block_bytes);
        hdr[0] = carry;
        hdr[1] = 0u;
        hdr[2] = 0u;
        hdr[3] = 0u;
    }
}

// Scatter: every splat of band b goes to slot partials[b][blk] + (earlier waves' and lanes'
// splats of the band), in shard order; slot_of[b * P + g] remembers it for B2's band sum.
__global__ __launch_bounds__(kB) void pack_scatter_kernel(const uint32_t* __restrict__ tiles,
                                                          const uint4* __restrict__ rect,
                                                          const uint32_t* __restrict__ depth_key,
                                                          const float4* __restrict__ rec, int P, BandRows br,
                                                          const uint32_t* __restrict__ partials, int nblk,
                                                          char* __restrict__ send, size_t block_bytes, int pair_cap,
                                                          uint32_t* __restrict__ slot_of) {
    __shared__ uint32_t cnt[kWaves][kMaxBands];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int base = blockIdx.x * kPackTile + w * (kI * 64);
    // pass 1: this wave's count per band (for the wave offsets)
    uint32_t c[kMaxBands];
#pragma unroll
    for (int b = 0; b < kMaxBands; ++b) c[b] = 0u;
    for (int r = 0; r < kI; ++r) {
        const int g = base + r * 64 + lane;
        int b_lo = kMaxBands, b_hi = -1;
        if (g < P && tiles[g] != 0u) {
            const uint4 rr = rect[g];
            band_span(br, rr.x >> 16, rr.y >> 16, b_lo, b_hi);
        }
#pragma unroll
        for (int b = 0; b < kMaxBands; ++b)
            if (b < br.n) c[b] += (uint32_t)__popcll(__ballot(b >= b_lo && b <= b_hi));
    }
    if (lane == 0)
        for (int b = 0; b < br.n; ++b) cnt[w][b] = c[b];
    __syncthreads();
    uint32_t pos[kMaxBands];
#pragma unroll
    for (int b = 0; b < kMaxBands; ++b) {
        pos[b] = 0u;
        if (b < br.n) {
            pos[b] = partials[b * nblk + blockIdx.x];
            for (int k = 0; k < w; ++k) pos[b] += cnt[k][b];
        }
    }
    const uint64_t lt = lanemask_lt();
    for (int r = 0; r < kI; ++r) {
        const int g = base + r * 64 + lane;
        int b_lo = kMaxBands, b_hi = -1;
        uint4 rr = make_uint4(0u, 0u, 0u, 0u);
        if (g < P && tiles[g] != 0u) {
            rr = rect[g];
            band_span(br, rr.x >> 16, rr.y >> 16, b_lo, b_hi);
        }
        float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0;
        uint32_t dk = 0u;
        if (b_lo <= b_hi) {
            r0 = rec[3 * (size_t)g];
            r1 = rec[3 * (size_t)g + 1];
            r2 = rec[3 * (size_t)g + 2];
            dk = depth_key[g];
        }
#pragma unroll
        for (int b = 0; b < kMaxBands; ++b) {
            if (b >= br.n) continue;  // grid-uniform
            const bool in = b >= b_lo && b <= b_hi;
            const uint64_t m = __ballot(in);
            if (in) {
                const uint32_t slot = pos[b] + (uint32_t)__popcll(m & lt);
                slot_of[(size_t)b * P + g] = slot;
                if (slot < (uint32_t)pair_cap) {
                    float4* dst = reinterpret_cast<float4*>(send + (size_t)b * block_bytes + kSplatBytes +
                                                            (size_t)slot * kSplatBytes);
                    dst[0] = r0;
                    dst[1] = r1;
                    dst[2] = r2;
                    dst[3] = make_float4(__uint_as_float(dk), __uint_as_float(rr.x), __uint_as_float(rr.y), 0.f);
                }
            }
            pos[b] += (uint32_t)__popcll(m);
        }
    }
}

// Band owner: local index i = src * pair_cap + slot.  Live slots get their record, depth key,
// rect and the tile count of the rect clipped to the band's rows; empty slots get no tiles.
// Band side.  With rb_hist (the grid then covers every slot once, 256 per block): also each
// block's splats per band row (the row-bucketed binning's pass-A counts, as F1 writes them on a
// single GPU) and its tiles_touched sum (the F2 scan's block partial).
__global__ __launch_bounds__(256) void unpack_kernel(const char* __restrict__ recv, size_t block_bytes, int nsrc,
                                                     int pair_cap, int ty0, int ty1, float4* __restrict__ rec,
                                                     uint32_t* __restrict__ depth_key, uint32_t* __restrict__ tiles,
                                                     uint4* __restrict__ rect, uint32_t* __restrict__ rb_hist,
                                                     uint32_t* __restrict__ bsum) {
    const long long n = (long long)nsrc * pair_cap;
    if (rb_hist) {  // grid-uniform
        __shared__ uint32_t rows[kRbMaxRows];
        __shared__ uint32_t ws[4];
        rows[threadIdx.x] = 0u;
        __syncthreads();
        const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
        uint32_t nt = 0;
        if (i < n) {
            const int src = (int)(i / pair_cap), slot = (int)(i - (long long)src * pair_cap);
            const char* blk = recv + (size_t)src * block_bytes;
            const uint32_t count = *reinterpret_cast<const uint32_t*>(blk);
            if ((uint32_t)slot < count) {
                const float4* sp = reinterpret_cast<const float4*>(blk + kSplatBytes + (size_t)slot * kSplatBytes);
                const float4 a = sp[3];
                rec[3 * i] = sp[0];
                rec[3 * i + 1] = sp[1];
                rec[3 * i + 2] = sp[2];
                const uint32_t lo = __float_as_uint(a.y), hi = __float_as_uint(a.z);
                depth_key[i] = __float_as_uint(a.x);
                rect[i] = make_uint4(lo, hi, 0u, 0u);
                const int miny = (int)(lo >> 16), maxy = (int)(hi >> 16);
                const int y0 = miny > ty0 ? miny : ty0, y1 = maxy < ty1 ? maxy : ty1;
                nt = y1 > y0 ? ((hi & 0xFFFF) - (lo & 0xFFFF)) * (uint32_t)(y1 - y0) : 0u;
                tiles[i] = nt;
                if (nt)
                    for (int r = y0; r < y1; ++r) atomicAdd(&rows[r - ty0], 1u);
            } else {
                depth_key[i] = 0xFFFFFFFFu;
                tiles[i] = 0u;
            }
        }
        uint32_t t = nt;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
        if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = t;
        __syncthreads();
        if ((int)threadIdx.x < ty1 - ty0) rb_hist[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = rows[threadIdx.x];
        if (threadIdx.x == 0) bsum[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
        return;
    }
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const int src = (int)(i / pair_cap), slot = (int)(i - (long long)src * pair_cap);
        const char* blk = recv + (size_t)src * block_bytes;
        const uint32_t count = *reinterpret_cast<const uint32_t*>(blk);
        if ((uint32_t)slot < count) {
            const float4* sp = reinterpret_cast<const float4*>(blk + kSplatBytes + (size_t)slot * kSplatBytes);
            const float4 a = sp[3];
            rec[3 * i] = sp[0];
            rec[3 * i + 1] = sp[1];
            rec[3 * i + 2] = sp[2];
            const uint32_t lo = __float_as_uint(a.y), hi = __float_as_uint(a.z);
            depth_key[i] = __float_as_uint(a.x);
            rect[i] = make_uint4(lo, hi, 0u, 0u);
            const int miny = (int)(lo >> 16), maxy = (int)(hi >> 16);
            const int y0 = miny > ty0 ? miny : ty0, y1 = maxy < ty1 ? maxy : ty1;
            tiles[i] = y1 > y0 ? ((hi & 0xFFFF) - (lo & 0xFFFF)) * (uint32_t)(y1 - y0) : 0u;
        } else {
            depth_key[i] = 0xFFFFFFFFu;
            tiles[i] = 0u;
        }
    }
}

// ---- the multi-GPU step's glue around the exchanges (gsr.h gsr_band_publish / gsr_gather_finish):
// one launch each instead of ~20 small copies, reductions and clears per step ----

// This rank's all-gather row: its band's pixel rows [py0, py1) of the 3 x H x W image into the
// row's 3 x tall x W head, then the status words (send-header counts, band K) at status_off.
__global__ __launch_bounds__(256) void band_publish_kernel(const float* __restrict__ color, int W, int H, int py0,
                                                          int py1, int tall, float* __restrict__ mine,
                                                          long long status_off, const char* __restrict__ send,
                                                          size_t block_bytes, int nbands,
                                                          const uint32_t* __restrict__ K_dev) {
    const long long per = (long long)(py1 - py0) * W, total = 3 * per;
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += stride) {
        const long long c = i / per, r = i - c * per;
        mine[c * (long long)tall * W + r] = color[c * (long long)H * W + (long long)py0 * W + r];
    }
    if (blockIdx.x == 0 && threadIdx.x <= nbands) {
        uint32_t* st = reinterpret_cast<uint32_t*>(mine + status_off);
        st[threadIdx.x] = threadIdx.x < nbands
                              ? *reinterpret_cast<const uint32_t*>(send + (size_t)threadIdx.x * block_bytes)
                              : *K_dev;
    }
}

// From the gathered rows (world x row_floats): every rank's band into the image, the agreed
// overflow word (ranks whose header counts exceed pair_cap or whose K exceeds the capacity, read
// from every rank's status words: the same value on every rank) and the next step's row
// statistics cleared (the statistics words of this rank's own row).
__global__ __launch_bounds__(256) void gather_finish_kernel(const float* __restrict__ gathered, long long row_floats,
                                                           long long status_off, int world, BandRows br, int W, int H,
                                                           int tall, float* __restrict__ image, uint32_t pair_cap,
                                                           uint32_t capacity, int32_t* __restrict__ guard,
                                                           float* __restrict__ zero, int nzero) {
    const int r = blockIdx.y;
    const int a = br.row[r] * kTile < H ? br.row[r] * kTile : H;
    const int b = br.row[r + 1] * kTile < H ? br.row[r + 1] * kTile : H;
    const long long per = (long long)(b - a) * W, total = 3 * per;
    const float* src = gathered + (long long)r * row_floats;
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += stride) {
        const long long c = i / per, q = i - c * per;
        image[c * (long long)H * W + (long long)a * W + q] = src[c * (long long)tall * W + q];
    }
    if (blockIdx.x == 0 && r == 0) {
        if (threadIdx.x < 64) {  // one lane per rank
            bool bad = false;
            if ((int)threadIdx.x < world) {
                const uint32_t* st = reinterpret_cast<const uint32_t*>(gathered + (long long)threadIdx.x * row_floats +
                                                                       status_off);
                for (int k = 0; k < world; ++k) bad |= st[k] > pair_cap;
                bad |= st[world] > capacity;
            }
            const uint64_t m = __ballot(bad);
            if (threadIdx.x == 0) guard[0] = (int32_t)__popcll(m);
        }
        for (int i = threadIdx.x; i < nzero; i += 256) zero[i] = 0.0f;
    }
}

}  // namespace

int launch_band_publish(const float* color, int W, int H, int py0, int py1, int tall, float* mine,
                        long long status_off, const char* send, size_t block_bytes, int nbands, const uint32_t* K_dev,
                        hipStream_t s) {
    const long long total = 3LL * (py1 > py0 ? py1 - py0 : 0) * W;
    const long long blocks = total > 0 ? ((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048) : 1;
    hipLaunchKernelGGL(band_publish_kernel, dim3((unsigned)blocks), dim3(256), 0, s, color, W, H, py0,
                       py1 > py0 ? py1 : py0, tall, mine, status_off, send, block_bytes, nbands, K_dev);
    return (int)hipGetLastError();
}

int launch_gather_finish(const float* gathered, long long row_floats, long long status_off, int world,
                         const BandRows& br, int W, int H, int tall, float* image, uint32_t pair_cap,
                         uint32_t capacity, int32_t* guard, float* zero, int nzero, hipStream_t s) {
    const long long total = 3LL * tall * W;
    const long long blocks = total > 0 ? ((total + 255) / 256 < 512 ? (total + 255) / 256 : 512) : 1;
    hipLaunchKernelGGL(gather_finish_kernel, dim3((unsigned)blocks, world), dim3(256), 0, s, gathered, row_floats,
                       status_off, world, br, W, H, tall, image, pair_cap, capacity, guard, zero, nzero);
    return (int)hipGetLastError();
}

int launch_pack_splats(const uint32_t* tiles, const uint4* rect, const uint32_t* depth_key, const float4* rec, int P,
                       const BandRows& br, uint32_t* partials, char* send, int pair_cap, uint32_t* slot_of,
                       uint32_t* row_hist, int grid_y, bool spans, hipStream_t s, uint32_t* rowpart) {
    const size_t bb = exchange_block_bytes(pair_cap);
    if (P <= 0) {  // empty shard: zero headers
        for (int b = 0; b < br.n; ++b)
            if (hipError_t e = hipMemsetAsync(send + (size_t)b * bb, 0, kSplatBytes, s)) return (int)e;
        return 0;
    }
    const int nblk = pack_blocks(P);
    const int hrows = row_hist ? (spans ? 3 : 1) * grid_y : 0;
    uint32_t* rp = hrows > 0 && hrows <= kRbMaxRows ? rowpart : nullptr;  // rowpart: [256][nblk] words
    if (spans && row_hist)
        hipLaunchKernelGGL(pack_count_kernel<true>, dim3(nblk), dim3(kB), 0, s, tiles, rect, P, br, partials, nblk,
                           row_hist, grid_y, rp);
    else
        hipLaunchKernelGGL(pack_count_kernel<false>, dim3(nblk), dim3(kB), 0, s, tiles, rect, P, br, partials, nblk,
                           row_hist, grid_y, rp);
    hipLaunchKernelGGL(pack_scan_kernel, dim3(br.n + (rp ? hrows : 0)), dim3(1024), 0, s, partials, nblk, send, bb,
                       br.n, rp, row_hist);
    hipLaunchKernelGGL(pack_scatter_kernel, dim3(nblk), dim3(kB), 0, s, tiles, rect, depth_key, rec, P, br, partials,
                       nblk, send, bb, pair_cap, slot_of);
    return (int)hipGetLastError();
}

int launch_unpack_splats(const char* recv, int nsrc, int pair_cap, int ty0, int ty1, float4* rec, uint32_t* depth_key,
                         uint32_t* tiles, uint4* rect, hipStream_t s, uint32_t* rb_hist, uint32_t* bsum) {
    const long long n = (long long)nsrc * pair_cap;
    if (n <= 0) return 0;
    const long long blocks = (n + 255) / 256;
    if (rb_hist && ty1 - ty0 > kRbMaxRows) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)(rb_hist || blocks < 8192 ? blocks : 8192)), dim3(256), 0, s, recv,
                       exchange_block_bytes(pair_cap), nsrc, pair_cap, ty0, ty1, rec, depth_key, tiles, rect, rb_hist,
                       bsum);
    return (int)hipGetLastError();
}

}  // namespace gsr

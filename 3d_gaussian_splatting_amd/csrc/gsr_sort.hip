// gsr_sort.hip -- binning on gfx950: scan, duplicateWithKeys, LSD radix sort, tile ranges,
// per-tile depth order.
//
// Canonical instance order is (tile, depth bits, gid) (SURVEY §8a notes).  It is reached
// with far fewer sorted bytes than one 45-bit key sort over K instances:
//   1. inclusive scan of tiles_touched in gid order           -> offsets (K = last)
//   2. duplicate: Gaussian g emits its band-clipped rect row-major at offsets[g-1] (coalesced
//      reads of tiles / rects, wave-cooperative expansion)
//   3. stable LSD over the ceil(log2 tiles)-bit tile key only (2 passes at 1080p), values =
//      the instance's Gaussian id -> grouped by tile, gid order inside a tile
//   4. finalize: tile ranges from key boundaries
//   5. per tile, a stable LDS radix sort of the slice by the 32-bit depth key alone (ties keep
//      gid order) -> (tile, depth, gid)
// (B1 recovers an instance's emission index j from its Gaussian's rect, so no permutation
// array is carried through the sort.)
//
// K never has to reach the host: the scan writes it to a device word (total_out), and every
// later stage is launched for the binning's capacity and reads the live count from that word
// (instances past the capacity are dropped -- an overflow the caller detects from K).
//
// Radix sort = reduce-then-scan per 8-bit digit: upsweep (per-block digit counts), column
// scan (per digit over blocks), downsweep (stable wave64 ranking: 8 ballots give each lane
// its peer mask, popcount below it is its rank in the round; per-wave running counters in
// LDS; digit base = scanned counts).  All integer work: HBM / issue-bound, no MFMA.
#include <cstdlib>

#include "gsr_kernels.h"

namespace gsr {
namespace {

constexpr int kB = kSortBlock;       // 256 threads = 4 waves
constexpr int kI = kSortItems;       // 16 rounds per wave
constexpr int kWaves = kB / 64;
constexpr int kWaveItems = kI * 64;  // 1024 contiguous items per wave

__device__ inline uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return (lane == 0) ? 0ull : (~0ull >> (64 - lane));
}

// live item count: the host bound, or the device count clamped to it
__device__ __forceinline__ long long live_count(long long cap, const uint32_t* __restrict__ n_dev) {
    if (!n_dev) return cap;
    const long long n = (long long)*n_dev;
    return n < cap ? n : cap;
}

// lanes (among `active`) holding the same digit as this lane (digits of up to MAXB bits)
template <int MAXB = 8>
__device__ inline uint64_t match_digit(uint32_t d, int nbits, uint64_t active) {
    uint64_t peers = active;
#pragma unroll
    for (int b = 0; b < MAXB; ++b) {
        if (b < nbits) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
    }
    return peers;
}

// Chunk of the key array a radix block works on.  Blocks are dealt to the 8 XCDs round-robin
// (b % 8), so neighbouring chunks would sit in different L2s; with the remap each XCD takes a
// contiguous run of chunks, and the partial 64-B lines at the ends of a chunk's digit runs (the
// downsweep's scatter) and of its histogram column entries meet their neighbours' halves in the
// same L2 before write-back.
// (1M / 1080p tile sort 0.1145 -> 0.102 ms, 5M 0.496 -> 0.475; the same remap of the per-tile
// depth sort's tiles measured no change.)
__device__ __forceinline__ int radix_chunk(int b, int nb) {
    const int q = nb / 8, r = nb % 8, xcd = b % 8, local = b / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// ---- upsweep: per-block digit histogram, written digit-major hist[d * nb + b] ----
// Counting needs no stable rank, so per-wave LDS sub-histograms with atomics suffice (the
// 8-ballot peer match of the downsweep measured slower here).  Blocks past the live count
// write zero columns.
// RI: rounds of 64 keys per wave (kRadixItems, or kRadixItemsSmall for small sorts)
template <int RI>
__global__ __launch_bounds__(kB) void radix_upsweep(const uint32_t* __restrict__ keys, long long cap,
                                                    const uint32_t* __restrict__ n_dev, int shift, int nbits,
                                                    int nb, uint32_t* __restrict__ hist) {
    __shared__ uint32_t cnt[kWaves][256];
    const int tid = threadIdx.x, w = tid >> 6;
    const long long n = live_count(cap, n_dev);
#pragma unroll
    for (int k = 0; k < kWaves; ++k) cnt[k][tid] = 0;
    __syncthreads();
    const uint32_t mask = (1u << nbits) - 1u;
    const int chunk = radix_chunk(blockIdx.x, nb);
    const long long base = (long long)chunk * (kB * RI) + (long long)w * (64 * RI);
    // all RI loads in flight before the first atomic (one HBM round trip per wave, not RI / 4)
    uint32_t k[RI];
#pragma unroll
    for (int r = 0; r < RI; ++r) {
        const long long idx = base + r * 64 + (tid & 63);
        k[r] = idx < n ? keys[idx] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int r = 0; r < RI; ++r) {
        const long long idx = base + r * 64 + (tid & 63);
        if (idx < n) atomicAdd(&cnt[w][(k[r] >> shift) & mask], 1u);
    }
    __syncthreads();
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) s += cnt[k][tid];
    hist[(size_t)tid * nb + chunk] = s;
}

// ---- column scan: block d turns hist[d*nb .. +nb) into an exclusive scan; totals[d] ----
// Four consecutive counts per thread per round (1024 per block round: 8 rounds for the 7936
// blocks of a 5M / 1080p tile sort instead of 31).
constexpr int kColQ = 4;
__global__ __launch_bounds__(kB) void radix_colscan(uint32_t* __restrict__ hist, int nb,
                                                    uint32_t* __restrict__ totals) {
    __shared__ uint32_t wsum[kWaves];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    uint32_t* col = hist + (size_t)blockIdx.x * nb;
    uint32_t carry = 0;
    for (int base = 0; base < nb; base += kB * kColQ) {
        const int i0 = base + tid * kColQ;
        uint32_t v[kColQ], sv = 0;
#pragma unroll
        for (int q = 0; q < kColQ; ++q) {
            v[q] = i0 + q < nb ? col[i0 + q] : 0u;
            sv += v[q];
        }
        // inclusive wave scan of the per-thread sums
        uint32_t x = sv;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint32_t pre = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) pre += (k < w) ? wsum[k] : 0u;
        uint32_t run = carry + pre + x - sv;
#pragma unroll
        for (int q = 0; q < kColQ; ++q) {
            if (i0 + q < nb) col[i0 + q] = run;
            run += v[q];
        }
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) tot += wsum[k];
        __syncthreads();
        carry += tot;
    }
    if (tid == 0) totals[blockIdx.x] = carry;
}

// ---- downsweep: stable scatter, reordered through LDS so global writes are coalesced ----
template <int RI>
__global__ __launch_bounds__(kB) void radix_downsweep(const uint32_t* __restrict__ keys_in,
                                                      const uint32_t* __restrict__ vals_in,
                                                      uint32_t* __restrict__ keys_out,
                                                      uint32_t* __restrict__ vals_out, long long cap,
                                                      const uint32_t* __restrict__ n_dev, int shift, int nbits,
                                                      int nb, const uint32_t* __restrict__ hist,
                                                      const uint32_t* __restrict__ totals) {
    __shared__ uint32_t wcnt[kWaves][256];
    __shared__ uint32_t gbase[256];   // global position of this block's first item of digit d
    __shared__ uint32_t lbase[256];   // block-local position of the first item of digit d
    __shared__ uint32_t wsum[kWaves];
    constexpr int TILE = kB * RI;
    __shared__ uint32_t skey[TILE];
    __shared__ uint32_t sval[TILE];
    const long long n = live_count(cap, n_dev);
    const int chunk = radix_chunk(blockIdx.x, nb);
    const long long bbase = (long long)chunk * TILE;
    if (bbase >= n) return;  // block-uniform: nothing of this block is live
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t mask = (1u << nbits) - 1u;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) wcnt[k][tid] = 0;
    // global digit base: exclusive scan of totals + this block's scanned count
    {
        const uint32_t v = totals[tid];
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint32_t pre = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) pre += (k < w) ? wsum[k] : 0u;
        gbase[tid] = pre + x - v + hist[(size_t)tid * nb + chunk];
    }
    __syncthreads();
    const long long base = bbase + (long long)w * (64 * RI);
    uint32_t key[RI], val[RI], rank[RI];
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int r = 0; r < RI; ++r) {
        const long long idx = base + r * 64 + lane;
        const bool valid = idx < n;
        key[r] = valid ? keys_in[idx] : 0xFFFFFFFFu;
        val[r] = valid ? (vals_in ? vals_in[idx] : (uint32_t)idx) : 0u;
    }
#pragma unroll
    for (int r = 0; r < RI; ++r) {
        const long long idx = base + r * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = (key[r] >> shift) & mask;
        const uint64_t active = __ballot(valid);
        const uint64_t peers = match_digit(d, nbits, active);
        const uint32_t old = wcnt[w][d];
        rank[r] = old + (uint32_t)__popcll(peers & lt);
        if (valid && (peers & lt) == 0) wcnt[w][d] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    {
        // per digit: wave prefixes (in place) and the block count; block-local digit starts
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) {
            const uint32_t t = wcnt[k][tid];
            wcnt[k][tid] = c;
            c += t;
        }
        uint32_t x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        __syncthreads();  // wsum reuse
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint32_t pre = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) pre += (k < w) ? wsum[k] : 0u;
        lbase[tid] = pre + x - c;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RI; ++r) {
        const long long idx = base + r * 64 + lane;
        if (idx < n) {
            const uint32_t d = (key[r] >> shift) & mask;
            const uint32_t lp = lbase[d] + wcnt[w][d] + rank[r];
            skey[lp] = key[r];
            sval[lp] = val[r];
        }
    }
    __syncthreads();
    const int count = (n - bbase) < TILE ? (int)(n - bbase) : TILE;
#pragma unroll 4
    for (int i = tid; i < count; i += kB) {
        const uint32_t k = skey[i];
        const uint32_t d = (k >> shift) & mask;
        const uint32_t pos = gbase[d] + (uint32_t)i - lbase[d];
        keys_out[pos] = k;
        vals_out[pos] = sval[i];
    }
}

// ---- F2 scan of tiles_touched (gid order): reduce / partial scan / downsweep ----
__device__ inline uint32_t block_exclusive_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    const int nw = blockDim.x >> 6;
    for (int k = 0; k < nw; ++k) {
        pre += (k < w) ? wsum[k] : 0u;
        tot += wsum[k];
    }
    __syncthreads();
    *total = tot;
    return pre + x - v;
}

__global__ __launch_bounds__(kB) void scan_reduce(const uint32_t* __restrict__ in, int n,
                                                  uint32_t* __restrict__ partials) {
    __shared__ uint32_t wsum[kWaves];
    const int base = blockIdx.x * kSortTile;
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < kI; ++r) {
        const int i = base + r * kB + threadIdx.x;
        if (i < n) s += in[i];
    }
    uint32_t tot;
    block_exclusive_scan(s, wsum, &tot);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

// Exclusive scan of n words in place by one block of 1024 threads, kScanQ contiguous words per
// thread per round (all of a round's loads issued before its block scan): one load latency and
// one block scan per 8192 words, not per 1024 (the F2 block sums at 5M: 19.5k words).
// Up to kScanQ1 x 1024 words (5M: 19.5k) in one round: Q = ceil(n / 1024) consecutive words per
// thread, one load latency, one block scan, one store pass (three serial rounds of 8192 took
// ~7 us each at 5M).
#ifndef GSR_SCAN_ONE_ROUND
#define GSR_SCAN_ONE_ROUND 1
#endif
constexpr int kScanQ = 8, kScanQ1 = 32;
__device__ __forceinline__ uint32_t wide_block_scan(uint32_t* __restrict__ a, int n, uint32_t* wsum) {
    if (GSR_SCAN_ONE_ROUND && n <= 1024 * kScanQ1) {
        const int Q = (n + 1023) / 1024;
        const int i0 = (int)threadIdx.x * Q;
        uint32_t v[kScanQ1], sv = 0;
#pragma unroll
        for (int q = 0; q < kScanQ1; ++q) {
            v[q] = q < Q && i0 + q < n ? a[i0 + q] : 0u;
            sv += v[q];
        }
        uint32_t tot;
        uint32_t run = block_exclusive_scan(sv, wsum, &tot);
#pragma unroll
        for (int q = 0; q < kScanQ1; ++q) {
            if (q < Q && i0 + q < n) a[i0 + q] = run;
            run += v[q];
        }
        return tot;
    }
    uint32_t carry = 0;
    for (int base = 0; base < n; base += 1024 * kScanQ) {
        const int i0 = base + (int)threadIdx.x * kScanQ;
        uint32_t v[kScanQ], sv = 0;
#pragma unroll
        for (int q = 0; q < kScanQ; ++q) {
            v[q] = i0 + q < n ? a[i0 + q] : 0u;
            sv += v[q];
        }
        uint32_t tot;
        uint32_t run = carry + block_exclusive_scan(sv, wsum, &tot);
#pragma unroll
        for (int q = 0; q < kScanQ; ++q) {
            if (i0 + q < n) a[i0 + q] = run;
            run += v[q];
        }
        carry += tot;
    }
    return carry;
}

// The single-round scan through LDS (dynamic LDS of n words, n <= kScanQ1 x 1024): the array is
// loaded and stored coalesced (word i by thread i mod 1024), and each thread scans its Q
// consecutive words out of LDS -- the direct form's loads of Q consecutive words per thread touch
// a different cache line in every lane of every load instruction.
#ifndef GSR_SCAN_LDS
#define GSR_SCAN_LDS 1
#endif
__device__ __forceinline__ uint32_t wide_block_scan_lds(uint32_t* __restrict__ a, int n, uint32_t* wsum,
                                                        uint32_t* buf) {
    for (int i = (int)threadIdx.x; i < n; i += 1024) buf[i] = a[i];
    __syncthreads();
    const int Q = (n + 1023) / 1024;
    const int i0 = (int)threadIdx.x * Q;
    uint32_t v[kScanQ1], sv = 0;
#pragma unroll
    for (int q = 0; q < kScanQ1; ++q) {
        v[q] = q < Q && i0 + q < n ? buf[i0 + q] : 0u;
        sv += v[q];
    }
    uint32_t tot;
    uint32_t run = block_exclusive_scan(sv, wsum, &tot);
#pragma unroll
    for (int q = 0; q < kScanQ1; ++q) {
        if (q < Q && i0 + q < n) buf[i0 + q] = run;
        run += v[q];
    }
    __syncthreads();
    for (int i = (int)threadIdx.x; i < n; i += 1024) a[i] = buf[i];
    return tot;
}
__host__ __device__ constexpr bool scan_lds_fits(long long n) { return GSR_SCAN_LDS && n <= 1024LL * kScanQ1; }

// exclusive scan of the nb block totals in place; the grand total to *total_out
__global__ __launch_bounds__(1024) void scan_partials(uint32_t* __restrict__ partials, int nb,
                                                      uint32_t* __restrict__ total_out) {
    extern __shared__ uint32_t sbuf[];
    __shared__ uint32_t wsum[16];
    const uint32_t carry = scan_lds_fits(nb) ? wide_block_scan_lds(partials, nb, wsum, sbuf)
                                             : wide_block_scan(partials, nb, wsum);
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

// the row-bucketed binning's column scan: row r's per-block pair counts (histA[r][*]) in place,
// the row total to totA[r]; one 1024-thread block per row
__global__ __launch_bounds__(1024) void rb_colscan(uint32_t* __restrict__ hist, int nb, uint32_t* __restrict__ totals) {
    extern __shared__ uint32_t sbuf[];
    __shared__ uint32_t wsum[16];
    uint32_t* const a = hist + (size_t)blockIdx.x * nb;
    const uint32_t carry = scan_lds_fits(nb) ? wide_block_scan_lds(a, nb, wsum, sbuf) : wide_block_scan(a, nb, wsum);
    if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}
static size_t scan_lds_bytes(long long n) { return scan_lds_fits(n) ? sizeof(uint32_t) * (size_t)n : 0; }

__global__ __launch_bounds__(kB) void scan_downsweep(const uint32_t* __restrict__ in, int n,
                                                     const uint32_t* __restrict__ partials,
                                                     uint32_t* __restrict__ out) {
    __shared__ uint32_t buf[kSortTile + kSortTile / 32];
    __shared__ uint32_t wsum[kWaves];
    const int base = blockIdx.x * kSortTile;
    const int tid = threadIdx.x;
    auto pad = [](int i) { return i + (i >> 5); };
#pragma unroll
    for (int r = 0; r < kI; ++r) {
        const int i = r * kB + tid;
        const int g = base + i;
        buf[pad(i)] = g < n ? in[g] : 0u;
    }
    __syncthreads();
    uint32_t v[kI];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kI; ++k) {
        v[k] = buf[pad(tid * kI + k)];
        s += v[k];
        v[k] = s;  // thread-local inclusive
    }
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan(s, wsum, &tot) + partials[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kI; ++k) buf[pad(tid * kI + k)] = v[k] + ex;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kI; ++r) {
        const int i = r * kB + tid;
        if (base + i < n) out[base + i] = buf[pad(i)];
    }
}

// ---- F3 duplicate: wave-cooperative expansion (one wave = 64 consecutive Gaussians, whose
// instances are contiguous; lanes write consecutive instances -> coalesced stores) ----
__device__ __forceinline__ uint32_t udiv_small(uint32_t a, uint32_t b) {
    // a / b for a < 2^20, 1 <= b < 2^12: the float quotient of (a + 0.5) is at least 0.5 / b
    // away from an integer and rcp is accurate to ~1 ulp, so truncation is exact
    return (uint32_t)(((float)a + 0.5f) * __builtin_amdgcn_rcpf((float)b));
}

// Emission of one wave's instances [first, first + wtotal): lane i finds its owner -- the last
// lane whose start (s_start, relative to `first`) is <= i -- by binary search in LDS and writes
// (tile key, gid).  Instances at or past `cap` are dropped (binning overflow).
__device__ __forceinline__ void emit_wave(const uint32_t* s_start, const uint32_t* s_g, const uint32_t* s_w,
                                          const uint32_t* s_x0, const uint32_t* s_y0, uint32_t first,
                                          uint32_t wtotal, int grid_x, long long cap, uint32_t* __restrict__ tkey,
                                          uint32_t* __restrict__ tgid) {
    const int lane = threadIdx.x & 63;
    for (uint32_t i = lane; i < wtotal; i += 64) {
        if ((long long)first + i >= cap) break;
        int o = 0;  // lanes without instances never own one (their start is 0xFFFFFFFF)
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
            if (s_start[o + step] <= i) o += step;
        const uint32_t local = i - s_start[o];
        const uint32_t wd = s_w[o];
        const uint32_t dy = udiv_small(local, wd), dx = local - dy * wd;
        tkey[first + i] = (s_y0[o] + dy) * (uint32_t)grid_x + s_x0[o] + dx;
        tgid[first + i] = s_g[o];
    }
}

// ---- fused F2 + F3: scan of tiles_touched in gid order + duplicate, one kernel ----
// Block b (in launch order, atomic ticket) owns Gaussians [256 b, 256 b + 256): it scans their
// tiles_touched, finds the instances of all earlier blocks by a wave-parallel decoupled
// look-back (64 predecessors per probe; relaxed agent-scope atomics on packed flag|count
// words), writes offsets / inst_start, and emits its own instances exactly as
// duplicate_kernel does.  Replaces three scan kernels + a second pass over the Gaussians; shipped
// for n <= 2^19 (a full 1M scene's look-back chain over n / 256 blocks costs more than the
// three-kernel scan: 0.102 vs 0.084 ms).
constexpr uint32_t kAgg = 1u << 30, kInc = 2u << 30, kCntMask = kAgg - 1u;

__global__ __launch_bounds__(256) void scan_duplicate_kernel(const uint32_t* __restrict__ tiles,
                                                             uint4* __restrict__ rect, int n,
                                                             int grid_x, int ty0,
                                                             uint32_t* __restrict__ offsets,
                                                             uint32_t* __restrict__ tkey,
                                                             uint32_t* __restrict__ tgid, long long cap,
                                                             uint32_t* __restrict__ status,
                                                             uint32_t* __restrict__ ticket,
                                                             uint32_t* __restrict__ total_out) {
    __shared__ uint32_t s_start[kWaves][64], s_g[kWaves][64], s_w[kWaves][64], s_x0[kWaves][64],
        s_y0[kWaves][64];
    __shared__ uint32_t wsum[kWaves];
    __shared__ uint32_t s_excl;
    __shared__ int s_b;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    if (tid == 0) s_b = (int)atomicAdd(ticket, 1u);
    __syncthreads();
    const int b = s_b;
    const int g = b * 256 + tid;
    const bool valid = g < n;
    uint32_t nt = 0, minx = 0, maxx = 0, y0 = 0;
    if (valid) {
        nt = tiles[g];
        if (nt) {
            const uint4 rr = rect[g];
            minx = rr.x & 0xFFFF;
            maxx = rr.y & 0xFFFF;
            const uint32_t miny = rr.x >> 16;
            y0 = miny > (uint32_t)ty0 ? miny : (uint32_t)ty0;
        }
    }
    // block scan
    uint32_t x = nt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t pre = 0, total = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) {
        pre += (k < w) ? wsum[k] : 0u;
        total += wsum[k];
    }
    // look-back (wave 0)
    if (w == 0) {
        uint32_t excl = 0;
        if (b == 0) {
            if (lane == 0) __hip_atomic_store(status, kInc | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(status + b, kAgg | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int pos = b - 1;
            uint32_t spins = 0;
            while (true) {
                const int idx = pos - lane;
                uint32_t v = kInc;  // before block 0: an inclusive zero
                if (idx >= 0) v = __hip_atomic_load(status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                while (__ballot((v & ~kCntMask) == 0u)) {  // some predecessor not published yet
                    if (++spins > (1u << 24)) break;     // never expected; bounded so a bug cannot hang
                    __builtin_amdgcn_s_sleep(1);
                    if (idx >= 0 && (v & ~kCntMask) == 0u)
                        v = __hip_atomic_load(status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                const uint64_t inc = __ballot((v & kInc) != 0u);
                const int k = inc ? __builtin_ctzll(inc) : 64;  // nearest inclusive predecessor
                uint32_t c = lane <= k ? (v & kCntMask) : 0u;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
                excl += c;
                if (inc || spins > (1u << 24)) break;
                pos -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(status + b, kInc | (excl + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_excl = excl;
    }
    __syncthreads();
    const uint32_t excl = s_excl;
    const uint32_t lex = pre + x - nt;  // block-local exclusive offset
    if (valid) {
        offsets[g] = excl + lex + nt;
        if (nt) rect[g].z = excl + lex;  // inst_start
    }
    if (total_out && tid == 0 && (b + 1) * 256 >= n) *total_out = excl + total;  // the last block: K
    // emission: this wave's instances [excl + pre_w, + wsum[w]) with pre_w = first lane's lex
    const uint32_t wbase = pre;  // = lex of lane 0 of this wave
    // the owner search needs starts non-decreasing across the wave: a Gaussian without tiles
    // keeps its (shared) start and never owns an instance; lanes past n sort last
    s_start[w][lane] = valid ? lex - wbase : 0xFFFFFFFFu;
    s_g[w][lane] = (uint32_t)g;
    s_w[w][lane] = maxx - minx;
    s_x0[w][lane] = minx;
    s_y0[w][lane] = y0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    emit_wave(s_start[w], s_g[w], s_w[w], s_x0[w], s_y0[w], excl + wbase, wsum[w], grid_x, cap, tkey, tgid);
}

// RANKED (presort mode): lane i is depth rank i; its tiles / rect / gid come from the rank-order
// payload (rtiles / rrect, coalesced) and inst_start goes to rect[gid] (one scattered word).
// RANKED also scans: `bexcl` holds the exclusive offsets of the 256-rank blocks (rank_payload_kernel
// summed each block, scan_partials scanned the sums), the block scans its own ranks and writes
// `offsets` (the gather reads them) -- the three-kernel scan's reduce and downsweep passes gone.
template <bool RANKED>
__global__ __launch_bounds__(256) void duplicate_kernel(uint32_t* __restrict__ offsets,
                                                        const uint32_t* __restrict__ tiles,
                                                        uint4* __restrict__ rect, const uint4* __restrict__ rrect,
                                                        int P, int grid_x, int ty0,
                                                        uint32_t* __restrict__ tkey, uint32_t* __restrict__ tgid,
                                                        long long cap, const uint32_t* __restrict__ bexcl) {
    __shared__ uint32_t s_start[kWaves][64], s_g[kWaves][64], s_w[kWaves][64], s_x0[kWaves][64],
        s_y0[kWaves][64];
    __shared__ uint32_t wsum[kWaves];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int i = blockIdx.x * 256 + tid;  // gid, or depth rank (RANKED)
    const bool valid = i < P;
    uint32_t nt = 0, end = 0, g = (uint32_t)i;
    if (RANKED) {
        if (valid) nt = tiles[i];
        uint32_t tot;
        end = bexcl[blockIdx.x] + block_exclusive_scan(nt, wsum, &tot) + nt;
        if (valid) offsets[i] = end;
    } else if (valid) {
        nt = tiles[i];
        end = offsets[i];
    }
    uint32_t minx = 0, maxx = 0, y0 = 0;
    if (nt) {
        uint4 rr;
        if (RANKED) {
            rr = rrect[i];
            g = rr.z;
            rect[g].z = end - nt;  // inst_start
        } else {
            rect[g].z = end - nt;  // inst_start
            rr = rect[g];
        }
        minx = rr.x & 0xFFFF;
        maxx = rr.y & 0xFFFF;
        const uint32_t miny = rr.x >> 16;
        y0 = miny > (uint32_t)ty0 ? miny : (uint32_t)ty0;
    }
    const uint32_t first = (uint32_t)__builtin_amdgcn_readfirstlane((int)(end - nt));
    const uint64_t vmask = __ballot(valid);
    if (vmask == 0) return;
    const int last_lane = 63 - __builtin_clzll(vmask);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)end, last_lane) - first;
    s_start[w][lane] = valid ? end - nt - first : 0xFFFFFFFFu;
    s_g[w][lane] = g;
    s_w[w][lane] = maxx - minx;
    s_x0[w][lane] = minx;
    s_y0[w][lane] = y0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    emit_wave(s_start[w], s_g[w], s_w[w], s_x0[w], s_y0[w], first, total, grid_x, cap, tkey, tgid);
}

// ---- presort: each depth rank's binning payload, gathered once into rank order ----
// rtiles[r] = tiles[g], rrect[r] = (rect lo, rect hi, g, 0) for g = the sorted gid at rank r.  The
// reads are random (16 B per visible Gaussian, L2 / MALL-resident), the writes coalesced; the
// scan, F3 and the gather then stream the payload instead of each making random reads.
// It also sums each 256-rank block's tiles_touched into bsum[block] (for the ranked F3's scan).
__global__ __launch_bounds__(256) void rank_payload_kernel(const uint32_t* __restrict__ sgid,
                                                           const uint32_t* __restrict__ tiles,
                                                           const uint4* __restrict__ rect, int n,
                                                           uint32_t* __restrict__ rtiles,
                                                           uint4* __restrict__ rrect, uint32_t* __restrict__ bsum) {
    __shared__ uint32_t wsum[kWaves];
    const int r = blockIdx.x * 256 + threadIdx.x;
    uint32_t nt = 0;
    if (r < n) {
        const uint32_t g = sgid[r];
        nt = tiles[g];
        uint4 q = make_uint4(0u, 0u, g, 0u);
        if (nt) {
            const uint4 rr = rect[g];
            q.x = rr.x;
            q.y = rr.y;
        }
        rtiles[r] = nt;
        rrect[r] = q;
    }
    uint32_t s = nt;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// ---- row-bucketed binning: F3 + the tile sort + F5 in two counting passes ----
// The stable tile-key sort of the K emitted instances (two LSD passes over 8-byte records, ~340 MB
// of traffic at 1M / 1080p) is replaced by two counting passes that each touch far fewer bytes:
//   A. (Gaussian, tile row) pairs -- ~2.8 per visible Gaussian against ~7.5 instances -- bucketed by
//      row: a per-block row count (rb_rows_count), the radix column scan, and a placement that
//      takes each pair's slot from an LDS counter of its row (rb_rows_place).  A pair is
//      (gid, x0 | x1 << 16): its columns, not expanded.
//   B. per chunk of kRbChunk pairs of one row: the pairs' columns counted (rb_chunks_count), every
//      row's [column][chunk] counts scanned flat with a look-back over rows (rb_tiles_scan, which
//      also writes the tile ranges), and each chunk's instances placed from LDS column counters,
//      staged in LDS and written as coalesced column runs (rb_chunks_place).
// Result: every tile's entries contiguous, the ranges F5 would write, the tile keys -- ~140 MB of
// traffic and no separate F3 / F5 -- but a tile's entries in arbitrary order: the per-tile depth
// sort that follows orders them by the whole (depth, gid) key (the register form; the LDS forms
// add gid passes, `unordered`), so the canonical list is the radix path's bit for bit.  Used when
// the image has at most kRbMaxRows tile rows and kRbMaxCols tile columns (row / column ids fit one
// byte; tall grids of at most kRbMaxRows tile rows -- views mode's stacked images included -- take
// it too), outside presort mode, below kRbMaxCap instances (gsr_api.cpp expected_layout; recorded
// in gsr_buffers.layout).
constexpr int kRbChunk = kRbChunkPairs;  // pairs per pass-B block (4 per thread)
// GSR_RB_STAGE32 1: pass B stages (pair index | column << 16) as one word per instance (no
// sub-dword LDS stores from neighbouring lanes into one dword)
#ifndef GSR_RB_STAGE32
#define GSR_RB_STAGE32 1
#endif
static_assert(kRbChunk % 256 == 0 && kRbMaxRows == 256 && kRbMaxCols == 256, "one row / column per thread");
#ifndef GSR_RB_STAGE_A
#define GSR_RB_STAGE_A 1024
#endif
// LDS staging (pairs) of a pass-A block (~720 at 1M / 1080p; a block past it writes unstaged):
// 1024 keeps the block at 16 KB, 8 waves per SIMD (2048: 30 KB, 5)
constexpr int kRbStageA = GSR_RB_STAGE_A;
#ifndef GSR_RB_STAGE_B
#define GSR_RB_STAGE_B 4096
#endif
constexpr int kRbStage = GSR_RB_STAGE_B;  // LDS staging (instances) of a pass-B block (~2800 at 1M / 1080p)
constexpr uint32_t kRbAgg = 1u << 30, kRbInc = 2u << 30, kRbCntMask = kRbAgg - 1u;

// rows of one block's Gaussians -> histA[r * nbA + b] (F1 writes the same counts itself when it
// ran for these Gaussians: PreOut.rb_hist; this kernel serves the band side, whose splats arrive
// from the exchange)
__global__ __launch_bounds__(256) void rb_rows_count(const uint32_t* __restrict__ tiles, const uint4* __restrict__ rect,
                                                     int n, int ty0, int ty1, uint32_t* __restrict__ histA, int nbA) {
    __shared__ uint32_t cnt[kRbMaxRows];
    const int tid = threadIdx.x, R = ty1 - ty0;
    cnt[tid] = 0u;
    __syncthreads();
    const int g = blockIdx.x * 256 + tid;
    if (g < n) {
        const uint32_t nt = tiles[g];
        if (nt) {
            const uint4 rr = rect[g];
            const int miny = (int)(rr.x >> 16), maxy = (int)(rr.y >> 16);
            const int by0 = miny > ty0 ? miny : ty0, by1 = maxy < ty1 ? maxy : ty1;
            for (int r = by0; r < by1; ++r) atomicAdd(&cnt[r - ty0], 1u);
        }
    }
    __syncthreads();
    if (tid < R) histA[(size_t)tid * nbA + blockIdx.x] = cnt[tid];
}

// Pairs of the block's 256 Gaussians placed row by row: the block counts its pairs per row in
// LDS, takes each row's global base (the column-scanned counts), and every lane walks its own
// rows, taking a slot of its row from an LDS counter -- the order of a row's pairs inside the
// block is arbitrary (the per-tile sort that follows orders each tile by (depth, gid) itself),
// so no per-row ballot sweep is needed.  Staged in LDS by row, written as coalesced row runs.
__global__ __launch_bounds__(256) void rb_rows_place(const uint32_t* __restrict__ tiles, uint4* __restrict__ rect,
                                                     uint32_t* __restrict__ offsets, const uint32_t* __restrict__ bsum,
                                                     int n, int ty0, int ty1,
                                                     const uint32_t* __restrict__ histA,
                                                     const uint32_t* __restrict__ totA, int nbA,
                                                     uint32_t* __restrict__ pgid, uint32_t* __restrict__ pxr,
                                                     long long pcap, const uint32_t* __restrict__ depth_key,
                                                     uint2* __restrict__ ppair) {
    __shared__ uint32_t cnt[kRbMaxRows];  // pairs per row, then the running staging slot
    __shared__ uint32_t gb[kRbMaxRows];   // global position of the block's first pair of row r
    __shared__ uint32_t lb[kRbMaxRows];   // staging position of the block's first pair of row r
    __shared__ uint32_t sg[kRbStageA], sx[kRbStageA], sk[kRbStageA];
    __shared__ uint8_t sr[kRbStageA];
    __shared__ uint32_t wsum[kWaves];
    const int tid = threadIdx.x, R = ty1 - ty0;
    cnt[tid] = 0u;
    // the row totals and this block's column of the scanned counts: loads issued first (they do
    // not depend on the Gaussians), waited for at the block scan
    const uint32_t ta = tid < R ? totA[tid] : 0u;
    const uint32_t ha = tid < R ? histA[(size_t)tid * nbA + blockIdx.x] : 0u;
    const int g = blockIdx.x * 256 + tid;
    int by0 = 0, by1 = 0;  // band-relative rows
    uint32_t xr = 0;
    const uint32_t nt = g < n ? tiles[g] : 0u;
    uint32_t incl;  // F2: the inclusive scan of tiles_touched at g
    if (bsum) {     // from F1's scanned block sums: this block's base + the in-block scan
        const uint32_t bb = bsum[blockIdx.x];
        uint32_t tdum;
        incl = bb + block_exclusive_scan(nt, wsum, &tdum) + nt;
        if (g < n) offsets[g] = incl;
    } else {
        incl = g < n ? offsets[g] : 0u;  // the three-kernel scan's
    }
    if (nt) {
        const uint4 rr = rect[g];
        rect[g].z = incl - nt;  // inst_start: the emission index of the first instance (F3's)
        const int miny = (int)(rr.x >> 16), maxy = (int)(rr.y >> 16);
        by0 = (miny > ty0 ? miny : ty0) - ty0;
        by1 = (maxy < ty1 ? maxy : ty1) - ty0;
        xr = (rr.x & 0xFFFFu) | (rr.y << 16);
    }
    const uint32_t dk = ppair && nt ? depth_key[g] : 0u;  // the pair's depth key (ppair: for pass B)
    __syncthreads();
    for (int r = by0; r < by1; ++r) atomicAdd(&cnt[r], 1u);
    __syncthreads();
    uint32_t tot;
    {
        const uint32_t c = cnt[tid];
        uint32_t sdum;
        const uint32_t rowbase = block_exclusive_scan(ta, wsum, &sdum);
        gb[tid] = tid < R ? rowbase + ha : 0u;
        lb[tid] = block_exclusive_scan(c, wsum, &tot);
        cnt[tid] = 0u;
    }
    __syncthreads();
    const bool staged = tot <= (uint32_t)kRbStageA;  // block-uniform
    for (int r = by0; r < by1; ++r) {
        const uint32_t k = atomicAdd(&cnt[r], 1u);
        if (staged) {
            sg[lb[r] + k] = (uint32_t)g;
            sx[lb[r] + k] = xr;
            if (ppair) sk[lb[r] + k] = dk;
            sr[lb[r] + k] = (uint8_t)r;
        } else {
            const long long pos = (long long)gb[r] + k;
            if (pos < pcap) {
                if (ppair) ppair[pos] = make_uint2((uint32_t)g, dk);
                else pgid[pos] = (uint32_t)g;
                pxr[pos] = xr;
            }
        }
    }
    if (!staged) return;
    __syncthreads();
    for (int i = tid; i < (int)tot; i += 256) {
        const int rr = sr[i];
        const long long pos = (long long)gb[rr] + (uint32_t)i - lb[rr];
        if (pos < pcap) {
            if (ppair) ppair[pos] = make_uint2(sg[i], sk[i]);
            else pgid[pos] = sg[i];
            pxr[pos] = sx[i];
        }
    }
}

// Pass-B chunk numbering (every pass-B kernel the same): row r holds ceil(pairs_r / kRbChunk)
// chunks of its pairs (pairs clamped to the pair capacity), numbered in row order.  Each block
// builds the rows' pair and chunk bases once in LDS (two block scans over the rows) and then finds
// a chunk's row by a binary search there.
struct RbRows {
    uint32_t pbase[kRbMaxRows];  // the row's first pair
    uint32_t cbase[kRbMaxRows];  // the row's first chunk
    uint32_t npair[kRbMaxRows];  // the row's pairs (clamped)
    uint32_t wsum[kWaves];
    uint32_t nchunks;            // all rows' chunks
};

__device__ __forceinline__ void rb_rows_table(const uint32_t* __restrict__ totA, int R, long long pcap, RbRows& t) {
    const int tid = threadIdx.x;
    const uint32_t ta = tid < R ? totA[tid] : 0u;
    uint32_t tp;
    const uint32_t pb = block_exclusive_scan(ta, t.wsum, &tp);
    const long long avail = pcap - (long long)pb;
    const uint32_t tc = avail <= 0 ? 0u : (avail < (long long)ta ? (uint32_t)avail : ta);
    uint32_t tcs;
    const uint32_t cb = block_exclusive_scan((tc + kRbChunk - 1) / kRbChunk, t.wsum, &tcs);
    t.pbase[tid] = pb;
    t.cbase[tid] = tid < R ? cb : 0xFFFFFFFFu;  // rows past R never match
    t.npair[tid] = tc;
    if (tid == 0) t.nchunks = tcs;
    __syncthreads();
}

struct RbChunk {
    int r, k, nch;
    uint32_t p0, p1, cp;  // pairs [p0, p1); cp: the row's first chunk
};

__device__ __forceinline__ RbChunk rb_chunk(const RbRows& t, uint32_t b) {
    // the last row whose first chunk is <= b: a row without chunks shares its first chunk number with
    // the next row that has some, so the last such row is the one holding chunk b
    int r = 0;
#pragma unroll
    for (int step = kRbMaxRows / 2; step > 0; step >>= 1)
        if (t.cbase[r + step] <= b) r += step;
    RbChunk ch;
    ch.r = r;
    ch.cp = t.cbase[r];
    ch.k = (int)(b - ch.cp);
    ch.nch = (int)((t.npair[r] + kRbChunk - 1) / kRbChunk);
    ch.p0 = t.pbase[r] + (uint32_t)ch.k * kRbChunk;
    const uint32_t end = t.pbase[r] + t.npair[r];
    ch.p1 = ch.p0 + kRbChunk < end ? ch.p0 + kRbChunk : end;
    return ch;
}

// pass B, counts: instances of each chunk per column -> histB[gx * cp + c * nch + k].  Blocks walk
// the chunks (grid-stride), so a grid sized for the worst case costs no empty blocks.
__global__ __launch_bounds__(256) void rb_chunks_count(const uint32_t* __restrict__ pxr, const uint32_t* __restrict__ totA,
                                                       int R, int gx, long long pcap, uint32_t* __restrict__ histB) {
    __shared__ RbRows t;
    __shared__ uint32_t cnt[kRbMaxCols];
    const int tid = threadIdx.x;
    rb_rows_table(totA, R, pcap, t);
    for (uint32_t b = blockIdx.x; b < t.nchunks; b += gridDim.x) {
        const RbChunk ch = rb_chunk(t, b);
        cnt[tid] = 0u;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kRbChunk / 256; ++q) {
            const uint32_t p = ch.p0 + q * 256 + tid;
            if (p < ch.p1) {
                const uint32_t xr = pxr[p];
                for (uint32_t c = xr & 0xFFFFu; c < (xr >> 16); ++c) atomicAdd(&cnt[c], 1u);
            }
        }
        __syncthreads();
        if (tid < gx) histB[(size_t)gx * ch.cp + (size_t)tid * ch.nch + ch.k] = cnt[tid];
    }
}

// pass B, scan: the [column][chunk] counts of every row, flat, in R x G partitions -- partition
// p = r G + g holds columns [g gx / G, (g + 1) gx / G) of row r, contiguous in the flat order.
// Each block scans one partition (exclusive), takes its global base by a decoupled look-back over
// the partitions before it (in dispatch order: a ticket), and stores global positions in place;
// then the tile ranges of its columns ((0, 0) for an empty tile, as F5 leaves it; clamped to
// cap).  G > 1 spreads a row over several CUs: a band of 8 tile rows was 8 blocks on the chip
// (~22 us at 5M, the same as 68 rows of the full image).
constexpr int kRbScanThreads = 1024, kRbScanQ = 32;
// The look-back's status words pack a 30-bit count: the layout word keeps this binning to
// capacities below 2^30 (gsr_api.cpp expected_layout), so a step within its capacity never
// counts past it.  A look-back that spins past its bound (never expected) publishes what it has
// and marks the step: K_dev = UINT32_MAX, which every reader of K takes for an overflow
// (gsr_read_num_rendered names the cause), so the ranges it leaves are never trusted silently.
__global__ __launch_bounds__(kRbScanThreads) void rb_tiles_scan(const uint32_t* __restrict__ totA, int R, int gx,
                                                                int ty0, long long pcap, long long cap,
                                                                uint32_t* __restrict__ histB,
                                                                uint32_t* __restrict__ status,
                                                                uint32_t* __restrict__ ticket,
                                                                uint2* __restrict__ ranges,
                                                                uint32_t* __restrict__ K_dev, int G) {
    __shared__ uint32_t wsum[kRbScanThreads / 64];
    __shared__ uint32_t tstart[kRbMaxCols];
    __shared__ uint32_t s_row[2];
    __shared__ int s_p;
    __shared__ uint32_t s_base;
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid == 0) s_p = (int)atomicAdd(ticket, 1u);  // partitions in dispatch order (the look-back's progress)
    __syncthreads();
    const int p = s_p, r = p / G, gi = p - r * G;
    const int c0 = gi * gx / G, c1 = (gi + 1) * gx / G;  // this partition's columns
    // the row's chunks, as rb_rows_table numbers them
    {
        const uint32_t ta = tid < R ? totA[tid] : 0u;
        uint32_t tp;
        const uint32_t pb = block_exclusive_scan(ta, wsum, &tp);
        const long long avail = pcap - (long long)pb;
        const uint32_t tc = avail <= 0 ? 0u : (avail < (long long)ta ? (uint32_t)avail : ta);
        const uint32_t nc = (tc + kRbChunk - 1) / kRbChunk;
        uint32_t tcs;
        const uint32_t cb = block_exclusive_scan(nc, wsum, &tcs);
        if (tid == r) {
            s_row[0] = nc;
            s_row[1] = cb;
        }
        __syncthreads();
    }
    const uint32_t nch = s_row[0], cp = s_row[1];
    uint32_t* const h = histB + (size_t)gx * cp + (size_t)c0 * nch;  // the partition's counts
    const uint32_t E = (uint32_t)(c1 - c0) * nch;
    // the common case: the partition's counts in registers, Q consecutive ones per thread (up to
    // kRbScanQ x 1024), one block scan and one write of the final positions
    const uint32_t Q = (E + kRbScanThreads - 1) / kRbScanThreads;
    const bool one = Q <= (uint32_t)(GSR_SCAN_ONE_ROUND ? kRbScanQ : 4);
    const uint32_t i0 = Q * tid;
    uint32_t cnts[kRbScanQ], excl = 0, carry = 0;
    if (one) {
        uint32_t sv = 0;
#pragma unroll
        for (int q = 0; q < kRbScanQ; ++q) {
            cnts[q] = (uint32_t)q < Q && i0 + q < E ? h[i0 + q] : 0u;
            sv += cnts[q];
        }
        excl = block_exclusive_scan(sv, wsum, &carry);
    } else {
        for (uint32_t base = 0; base < E; base += 4 * kRbScanThreads) {
            const uint32_t j0 = base + 4 * tid;  // (partitions past kRbScanQ x 1024 counts: rounds of 4 per thread)
            uint32_t v[4], sv = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[q] = j0 + q < E ? h[j0 + q] : 0u;
                sv += v[q];
            }
            uint32_t tot;
            uint32_t run = carry + block_exclusive_scan(sv, wsum, &tot);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (j0 + q < E) h[j0 + q] = run;  // partition-relative for now
                run += v[q];
            }
            carry += tot;
        }
    }
    // look-back (wave 0): the instances of the partitions before p
    if (tid < 64) {
        uint32_t excl = 0;
        if (p == 0) {
            if (lane == 0) __hip_atomic_store(status, kRbInc | carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(status + p, kRbAgg | carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int pos = p - 1;
            uint32_t spins = 0;
            while (true) {
                const int idx = pos - lane;
                uint32_t v = kRbInc;
                if (idx >= 0) v = __hip_atomic_load(status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                while (__ballot((v & ~kRbCntMask) == 0u)) {
                    if (++spins > (1u << 24)) break;  // never expected; bounded so a bug cannot hang
                    __builtin_amdgcn_s_sleep(1);
                    if (idx >= 0 && (v & ~kRbCntMask) == 0u)
                        v = __hip_atomic_load(status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                const uint64_t inc = __ballot((v & kRbInc) != 0u);
                const int k = inc ? __builtin_ctzll(inc) : 64;
                uint32_t c = lane <= k ? (v & kRbCntMask) : 0u;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
                excl += c;
                if (inc || spins > (1u << 24)) break;
                pos -= 64;
            }
            if (lane == 0) __hip_atomic_store(status + p, kRbInc | (excl + carry), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (spins > (1u << 24) && lane == 0 && K_dev) *K_dev = 0xFFFFFFFFu;  // the step is void
        }
        if (lane == 0) s_base = excl;
    }
    __syncthreads();
    const uint32_t pbase = s_base;  // the global position of the partition's first instance
    if (one) {
        uint32_t run = pbase + excl;
        uint32_t c = i0 / (nch ? nch : 1u), k = i0 - c * nch;  // column (partition-relative) and chunk of i0
#pragma unroll
        for (int q = 0; q < kRbScanQ; ++q) {
            if ((uint32_t)q < Q && i0 + q < E) {
                h[i0 + q] = run;
                if (k == 0) tstart[c0 + c] = run;
                run += cnts[q];
                if (++k == nch) k = 0, ++c;
            }
        }
    } else {
        for (uint32_t i = tid; i < E; i += kRbScanThreads) h[i] += pbase;
        __syncthreads();
        if (tid >= c0 && tid < c1 && nch) tstart[tid] = h[(size_t)(tid - c0) * nch];
    }
    __syncthreads();
    // tile c of the partition: [its first chunk's base, the next tile's); the partition's last
    // tile ends where the next partition starts (flat order)
    if (tid >= c0 && tid < c1) {
        const uint32_t a = nch ? tstart[tid] : pbase, e = tid + 1 < c1 && nch ? tstart[tid + 1] : pbase + carry;
        const long long a2 = a < cap ? a : cap, e2 = e < cap ? e : cap;
        ranges[(size_t)(ty0 + r) * gx + tid] = e2 > a2 ? make_uint2((uint32_t)a2, (uint32_t)e2) : make_uint2(0u, 0u);
    }
}

// pass B, placement: each chunk's instances, a slot per instance from its column's LDS counter
// (order inside a tile is free, as in pass A), staged in LDS by column and written as coalesced
// column runs (tile key and gid; with tpair the (gid, depth key) pair, the key from pass A's
// ppair, so the per-tile sort that follows reads its keys coalesced instead of gathering one
// behind every gid load, one 8-B store per instance).  The staging holds each instance's pair
// index (u16) and column; the chunk's pairs (gid, key) sit in LDS beside it.
#ifndef GSR_RB_PLACE_WPE
#define GSR_RB_PLACE_WPE 1
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSR_RB_PLACE_WPE))) void rb_chunks_place(const uint32_t* __restrict__ pgid, const uint32_t* __restrict__ pxr,
                                                       const uint32_t* __restrict__ totA, int R, int gx, int ty0,
                                                       long long pcap, long long cap,
                                                       const uint32_t* __restrict__ histB,
                                                       uint32_t* __restrict__ tkey, uint32_t* __restrict__ tgid,
                                                       const uint2* __restrict__ ppair,
                                                       uint2* __restrict__ tpair) {
    __shared__ RbRows t;
    __shared__ uint32_t cnt[kRbMaxCols];  // instances per column, then the running staging slot
    __shared__ uint32_t lb[kRbMaxCols];   // staging start of column c
    __shared__ uint32_t gb[kRbMaxCols];   // global position of the chunk's first instance of column c
    __shared__ uint32_t pg[kRbChunk], pk[kRbChunk];  // the chunk's pairs: gid, depth key
#if GSR_RB_STAGE32
    __shared__ uint32_t spc[kRbStage];                // staged instance: pair index | column << 16
#else
    __shared__ uint16_t sp[kRbStage];                 // staged instance: its pair (index in the chunk)
    __shared__ uint8_t sc[kRbStage];
#endif
    __shared__ uint32_t wsum[kWaves];
    static_assert(kRbChunk <= 65536, "u16 pair index");
    const int tid = threadIdx.x;
    const bool keys = tpair != nullptr;  // launch-uniform
    rb_rows_table(totA, R, pcap, t);
    constexpr int kQ = kRbChunk / 256;
    // the next chunk's pairs are loaded while this one is placed (register double buffer)
    uint32_t nxr[kQ], ngg[kQ], nkk[kQ];
    auto load_pairs = [&](uint32_t b) {
        const RbChunk c = rb_chunk(t, b);
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const uint32_t p = c.p0 + q * 256 + tid;
            nxr[q] = p < c.p1 ? pxr[p] : 0u;  // 0: no columns
            if (keys) {
                const uint2 pp = p < c.p1 ? ppair[p] : make_uint2(0u, 0u);
                ngg[q] = pp.x;
                nkk[q] = pp.y;
            } else {
                ngg[q] = p < c.p1 ? pgid[p] : 0u;
                nkk[q] = 0u;
            }
        }
    };
    if (blockIdx.x < t.nchunks) load_pairs(blockIdx.x);
    for (uint32_t b = blockIdx.x; b < t.nchunks; b += gridDim.x) {
        const RbChunk ch = rb_chunk(t, b);
        cnt[tid] = 0u;
        const uint32_t hb = tid < gx ? histB[(size_t)gx * ch.cp + (size_t)tid * ch.nch + ch.k] : 0u;
        uint32_t xr[kQ], gg[kQ], kk[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            xr[q] = nxr[q];
            gg[q] = ngg[q];
            kk[q] = nkk[q];
        }
        if (b + gridDim.x < t.nchunks) load_pairs(b + gridDim.x);
        __syncthreads();  // cnt zeroed (and the previous chunk's staging read out)
#pragma unroll
        for (int q = 0; q < kQ; ++q)
            for (uint32_t c = xr[q] & 0xFFFFu; c < (xr[q] >> 16); ++c) atomicAdd(&cnt[c], 1u);
        __syncthreads();
        uint32_t tot;
        {
            const uint32_t c = cnt[tid];
            lb[tid] = block_exclusive_scan(c, wsum, &tot);
            gb[tid] = hb;
            cnt[tid] = 0u;
        }
        __syncthreads();
        const bool staged = tot <= (uint32_t)kRbStage;  // block-uniform
        const uint32_t row_tile = (uint32_t)(ty0 + ch.r) * (uint32_t)gx;
        if (staged) {
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                pg[q * 256 + tid] = gg[q];
                if (keys) pk[q * 256 + tid] = kk[q];
            }
        }
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            for (uint32_t c = xr[q] & 0xFFFFu; c < (xr[q] >> 16); ++c) {
                const uint32_t k = atomicAdd(&cnt[c], 1u);
                if (staged) {
#if GSR_RB_STAGE32
                    spc[lb[c] + k] = (uint32_t)(q * 256 + tid) | (c << 16);
#else
                    sp[lb[c] + k] = (uint16_t)(q * 256 + tid);
                    sc[lb[c] + k] = (uint8_t)c;
#endif
                } else {
                    const long long pos = (long long)gb[c] + k;
                    if (pos < cap) {
                        if (tkey) tkey[pos] = row_tile + c;
                        if (keys) tpair[pos] = make_uint2(gg[q], kk[q]);
                        else tgid[pos] = gg[q];
                    }
                }
            }
        }
        if (staged) {
            __syncthreads();
            for (int i = tid; i < (int)tot; i += 256) {
#if GSR_RB_STAGE32
                const uint32_t pc = spc[i];
                const int c = (int)(pc >> 16);
#else
                const int c = sc[i];
#endif
                const long long pos = (long long)gb[c] + ((uint32_t)i - lb[c]);
                if (pos < cap) {
                    if (tkey) tkey[pos] = row_tile + (uint32_t)c;
#if GSR_RB_STAGE32
                    const int pi = (int)(pc & 0xFFFFu);
#else
                    const int pi = sp[i];
#endif
                    if (keys) tpair[pos] = make_uint2(pg[pi], pk[pi]);
                    else tgid[pos] = pg[pi];
                }
            }
        }
        __syncthreads();  // cnt / lb / gb / staging reused by the next chunk
    }
}

// ---- F5 finalize: tile ranges from the sorted keys ----
// Four sorted keys per thread (one 16-B load; the sorted array is 16-B aligned), the neighbours
// across the quad from the adjacent words (cache hits): 0.075 -> ~0.03 ms at 5M / 1080p.
constexpr int kFinQ = 4;
__global__ __launch_bounds__(256) void finalize_kernel(const uint32_t* __restrict__ stile, long long cap,
                                                       const uint32_t* __restrict__ n_dev,
                                                       uint2* __restrict__ ranges) {
    const long long K = live_count(cap, n_dev);
    const long long i0 = ((long long)blockIdx.x * 256 + threadIdx.x) * kFinQ;
    if (i0 >= K) return;
    uint32_t t[kFinQ];
    if (i0 + kFinQ <= K) {
        const uint4 q = *reinterpret_cast<const uint4*>(stile + i0);
        t[0] = q.x, t[1] = q.y, t[2] = q.z, t[3] = q.w;
    } else {
#pragma unroll
        for (int j = 0; j < kFinQ; ++j) t[j] = i0 + j < K ? stile[i0 + j] : 0xFFFFFFFFu;
    }
    uint32_t prev = i0 > 0 ? stile[i0 - 1] : 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < kFinQ; ++j) {
        const long long i = i0 + j;
        if (i >= K) break;
        const uint32_t next = j + 1 < kFinQ ? t[j + 1] : (i + 1 < K ? stile[i + 1] : 0xFFFFFFFFu);
        if (i == 0 || prev != t[j]) ranges[t[j]].x = (uint32_t)i;
        if (i == K - 1 || next != t[j]) ranges[t[j]].y = (uint32_t)(i + 1);
        prev = t[j];
    }
}

// ---- per-tile depth order (canonical (tile, depth bits, gid) without a global depth sort) ----
// After the stable tile-bits sort of instances emitted in gid order, each tile's slice holds
// its Gaussians in gid order, so a stable LSD sort of the 32-bit depth keys alone gives
// (depth, gid) order.  Each pass is ranked exactly as radix_downsweep ranks (wave64 ballot
// peer match, per-wave digit counters, a digit-major block scan), in LDS: ~20 B of LDS traffic
// per key per pass, against ~log2(n)^2 / 2 x 12 B for a bitonic network, which is
// LDS-bandwidth-bound.  Passes whose digit is equal for every key of the slice are skipped, so
// 9-bit digits need 3 passes for the <= 27 differing bits of a 0.2 .. 100 depth range.
// Measured at 1M/1080p: 9-bit radix 0.098 ms, 8-bit 0.102 ms, bitonic 0.130 ms; the radix form
// is latency-bound per block (dependent LDS counter updates per 64-key round, ~6 syncs per
// pass), not by LDS bandwidth.
// NT threads, I items per thread: CAP = NT * I keys; wave w owns the contiguous run
// [w * 64 I, (w + 1) * 64 I) of the slice, ranked round by round in index order (stable).
// One slice [rg.x, rg.y) of n <= NT * I entries, sorted by the whole block.  Ends with every
// LDS access behind a barrier, so a block may call it again for another slice.
// Runs of equal depth keys in a depth-sorted slice (skey, sval in LDS, n entries) into gid order.
// The thread holding a run's first entry sorts the run by insertion when it is at most
// kTieRunMax long (runs are disjoint, so no two threads touch the same entries); if any run is
// longer, the whole slice goes through an all-ascending bitonic network on the 64-bit (depth,
// gid) keys in place (a degenerate slice: many Gaussians at one depth).  Ends behind a barrier.
// lo_bit > 0 (a truncated sort, radix_sort_slice): the slice was ordered by the key bits at and
// above lo_bit only, so a run is a group of equal TRUNCATED keys, and it is insertion-sorted by the
// whole (depth, gid) pair (lo_bit = 0: runs of equal keys, sorted by gid -- the same thing).
constexpr int kTieRunMax = 32;
// (A truncated sort that meets a long group -- clustered depths, thousands of keys within one
// truncated step -- takes the bitonic fallback on the whole pair as well.  Re-sorting such a slice
// on every bit from the registers instead was tried in round 6 and faulted on the GPU in the
// clustered-depth parity test; it is not used.)
__device__ __forceinline__ void tie_fixup(uint32_t* skey, uint32_t* sval, int n, int nt, int lo_bit = 0) {
    int longrun = 0;
    for (int i = threadIdx.x; i + 1 < n; i += nt) {
        const uint32_t k = skey[i] >> lo_bit;
        if ((skey[i + 1] >> lo_bit) != k || (i > 0 && (skey[i - 1] >> lo_bit) == k)) continue;  // not a run start
        int e = i + 2;
        while (e < n && (skey[e] >> lo_bit) == k && e - i <= kTieRunMax) ++e;
        if (e - i > kTieRunMax) {
            longrun = 1;
            continue;
        }
        for (int a = i + 1; a < e; ++a) {  // insertion sort of (skey, sval)[i, e) by the 64-bit pair
            const uint32_t ka = skey[a], va = sval[a];
            const uint64_t x = ((uint64_t)ka << 32) | va;
            int b = a;
            while (b > i && ((((uint64_t)skey[b - 1]) << 32) | sval[b - 1]) > x) {
                skey[b] = skey[b - 1];
                sval[b] = sval[b - 1];
                --b;
            }
            skey[b] = ka;
            sval[b] = va;
        }
    }
    if (!__syncthreads_or(longrun)) return;
    int m = 1;
    while (m < n) m <<= 1;
    auto cex = [&](int i, int j) {  // i < j; j >= n is +inf padding
        if (j >= n) return;
        const uint64_t a = ((uint64_t)skey[i] << 32) | sval[i], b = ((uint64_t)skey[j] << 32) | sval[j];
        if (a > b) {
            skey[i] = (uint32_t)(b >> 32), sval[i] = (uint32_t)b;
            skey[j] = (uint32_t)(a >> 32), sval[j] = (uint32_t)a;
        }
    };
    for (int size = 2; size <= m; size <<= 1) {
        for (int d = size >> 1; d >= 1; d >>= 1) {
            const bool flip = d == (size >> 1);
            for (int t = threadIdx.x; t < (m >> 1); t += nt) {
                const int i = ((t & ~(d - 1)) << 1) | (t & (d - 1));
                cex(i, flip ? (i ^ (size - 1)) : (i + d));
            }
            __syncthreads();
        }
    }
}

// out of line for the register-heavy slice kernels (its few live values cross the call)
__device__ __attribute__((noinline)) void tile_tie_fixup(uint32_t* skey, uint32_t* sval, int n, int nt, int lo_bit) {
    tie_fixup(skey, sval, n, nt, lo_bit);
}

// Truncated passes (unordered slices only): the LSD passes cover the top slice_passes(cap) * DB
// differing key bits and tie_fixup orders the groups of equal truncated keys by the whole
// (depth, gid) pair -- at 5M / 1080p (~4000-entry slices, 25 differing depth bits) two 9-bit
// passes instead of three leave ~3 % of the entries in groups of 2-3.  Longer slices keep more
// bits (a 8192-entry slice 3 x 8, so its groups stay as short); the 16384-entry form keeps all.
// GSR_SLICE_TRUNC 0: every differing bit everywhere.
#ifndef GSR_SLICE_TRUNC
#define GSR_SLICE_TRUNC 1
#endif
#ifndef GSR_SLICE_PASSES_8K
#define GSR_SLICE_PASSES_8K 3
#endif
__host__ __device__ constexpr int slice_passes(int cap) {
    return !GSR_SLICE_TRUNC ? 0 : cap <= 4096 ? 2 : cap <= 8192 ? GSR_SLICE_PASSES_8K : 0;
}

template <int NT, int I, int DB>
struct SliceLds {
    uint32_t wcnt[NT / 64][1 << DB];
    uint32_t lbase[1 << DB];
    uint32_t red[2][NT / 64];
    uint32_t skey[NT * I];
    uint32_t sval[NT * I];
};

template <int NT, int I, int DB, bool kFixInline = false>
__device__ __forceinline__ void radix_sort_slice(const uint2 rg, const uint32_t* __restrict__ depth_key,
                                                 uint32_t* __restrict__ gid, SliceLds<NT, I, DB>& lds,
                                                 bool unordered = false) {
    constexpr int NWV = NT / 64, BINS = 1 << DB;
    constexpr uint32_t DMASK = BINS - 1u;
    auto& wcnt = lds.wcnt;
    auto& lbase = lds.lbase;
    auto& red = lds.red;
    auto& skey = lds.skey;
    auto& sval = lds.sval;
    const int n = (int)(rg.y - rg.x);
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    // wave w owns [w * per, (w + 1) * per): per = the slice split evenly over the waves in whole
    // 64-lane rounds (<= 64 I since n <= CAP)
    const int per = (n + NWV * 64 - 1) / (NWV * 64) * 64;
    const int base = w * per;
    const int end = base + per < n ? base + per : n;
    uint32_t key[I], val[I], rank[I];
    uint32_t kor = 0u, kand = 0xFFFFFFFFu;
#pragma unroll
    for (int r = 0; r < I; ++r) {
        const int idx = base + r * 64 + lane;
        const bool valid = idx < end;
        val[r] = valid ? gid[rg.x + idx] : 0u;
        key[r] = valid ? depth_key[val[r]] : 0xFFFFFFFFu;
        if (valid) {
            kor |= key[r];
            kand &= key[r];
        }
    }
    // bits where the slice's keys differ: passes over constant digits are no-ops (stable)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        kor |= __shfl_xor(kor, o, 64);
        kand &= __shfl_xor(kand, o, 64);
    }
    if (lane == 0) {
        red[0][w] = kor;
        red[1][w] = kand;
    }
    __syncthreads();
    uint32_t diff = 0u;
    {
        uint32_t o_ = 0u, a_ = 0xFFFFFFFFu;
#pragma unroll
        for (int k = 0; k < NWV; ++k) {
            o_ |= red[0][k];
            a_ &= red[1][k];
        }
        diff = o_ ^ a_;
    }
    const uint64_t lt = lanemask_lt();
    // The (stable) depth passes alone: a gid-ordered slice ends in (depth, gid) order.  An
    // unordered one (the row-bucketed binning leaves a tile's entries in arbitrary order) ends in
    // depth order with each run of equal depth keys in arbitrary gid order; tile_tie_fixup puts
    // those runs in gid order afterwards (ties are rare and short: an LSD pass over the gid bits
    // per 8-9 of them would cost as much as the depth passes again).  An unordered slice is also
    // sorted on its top slice_passes * DB differing bits only (lo_bit): the fix-up then orders the
    // groups of equal truncated keys by the whole pair.
    const int hb = diff ? 31 - __clz(diff) : 0;  // the highest differing bit
    constexpr int KB = slice_passes(NT * I) * DB;  // kept bits (0: all)
    const int lo_bit = (unordered && KB > 0 && hb + 1 > KB) ? hb + 1 - KB : 0;
    bool ran = false;
    for (int shift = lo_bit; shift < 32 && shift <= hb; shift += DB) {
        if (((diff >> shift) & DMASK) == 0u) continue;  // block-uniform
        ran = true;
        for (int d = tid; d < NWV * BINS; d += NT) (&wcnt[0][0])[d] = 0u;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < I; ++r) {
            if (base + r * 64 >= end) break;  // wave-uniform: only the rounds holding keys
            const int idx = base + r * 64 + lane;
            const bool valid = idx < end;
            const uint32_t d = (key[r] >> shift) & DMASK;
            const uint64_t peers = match_digit<DB>(d, DB, __ballot(valid));
            const uint32_t old = wcnt[w][d];
            rank[r] = old + (uint32_t)__popcll(peers & lt);
            if (valid && (peers & lt) == 0) wcnt[w][d] = old + (uint32_t)__popcll(peers);
        }
        __syncthreads();
        // per digit: wave prefixes in place, then the digit-major block scan -> lbase
        for (int d = tid; d < BINS; d += NT) {
            uint32_t c = 0;
#pragma unroll
            for (int k = 0; k < NWV; ++k) {
                const uint32_t t = wcnt[k][d];
                wcnt[k][d] = c;
                c += t;
            }
            lbase[d] = c;
        }
        __syncthreads();
        if (tid < 64) {  // exclusive scan of the BINS digit totals, BINS / 64 per lane
            constexpr int Q = BINS / 64;
            uint32_t c4[Q], s4 = 0;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                c4[q] = lbase[Q * tid + q];
                s4 += c4[q];
            }
            uint32_t x = s4;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            uint32_t run = x - s4;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                lbase[Q * tid + q] = run;
                run += c4[q];
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < I; ++r) {
            const int idx = base + r * 64 + lane;
            if (idx < end) {
                const uint32_t d = (key[r] >> shift) & DMASK;
                const uint32_t lp = lbase[d] + wcnt[w][d] + rank[r];
                skey[lp] = key[r];
                sval[lp] = val[r];
            }
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < I; ++r) {
            const int idx = base + r * 64 + lane;
            if (idx < end) {
                key[r] = skey[idx];
                val[r] = sval[idx];
            }
        }
        __syncthreads();  // skey / sval / wcnt are rewritten by the next pass
    }
    if (unordered && n > 1) {
        if (!ran) {  // every key equal: the slice is one run, in LDS for the fix-up
#pragma unroll
            for (int r = 0; r < I; ++r) {
                const int idx = base + r * 64 + lane;
                if (idx < end) {
                    skey[idx] = key[r];
                    sval[idx] = val[r];
                }
            }
            __syncthreads();
        }
        if constexpr (kFixInline) tie_fixup(skey, sval, n, NT, lo_bit);
        else tile_tie_fixup(skey, sval, n, NT, lo_bit);
        for (int i = tid; i < n; i += NT) gid[rg.x + i] = sval[i];
        __syncthreads();  // skey / sval / red[] are rewritten by the next slice
        return;
    }
#pragma unroll
    for (int r = 0; r < I; ++r) {
        const int idx = base + r * 64 + lane;
        if (idx < end) gid[rg.x + idx] = val[r];
    }
    __syncthreads();  // red[] is rewritten by the next slice
}

// ---- per-tile depth order, register form: one wave per tile ----
// A slice of n <= 64 E entries (E = 1 .. 16, the smallest power of two that holds it)
// is sorted by one wave in VGPRs as 64-bit (depth << 32 | gid) keys with a bitonic network: lane l
// holds entries l E .. l E + E - 1, so exchanges at distances below E stay inside a lane and the
// rest go lane to lane by DPP (lane xor 1 / 2 / 3, row mirrors, row_ror 8), ds_swizzle (xor 4,
// 16, 31 inside 32-lane halves) and ds_bpermute (across the halves).  The gid in the low word
// makes every key distinct, so the result is the canonical (depth, gid) order whatever order the
// slice arrives in (no stability needed), and there is no LDS, no barrier and no per-pass
// histogram: ~log2(64 E)^2 / 2 compare-exchange stages of 5-6 VALU ops per key pair, against the
// LDS radix form's dependent counter updates and ~6 barriers per pass (latency-bound per block).
// "Flip" network (every merge ascending: its first stage pairs i with i ^ (k - 1), mirrored).
#ifndef GSR_TILE_WAVE_SORT
#define GSR_TILE_WAVE_SORT 1
#endif

// x from lane (lane ^ M) of the wave, M = 2^a - 1 (mirror stages) or 2^a (half cleaners)
template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x) {
    static_assert(M >= 1 && M <= 63, "lane_xor distance");
    if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
    else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);
    else if constexpr (M == 3) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x1B, 0xF, 0xF, false);
    else if constexpr (M == 7) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);
    else if constexpr (M == 15) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);
    else if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);
    else if constexpr (M == 4 || M == 16 || M == 31)  // bit mode: and 0x1f, xor M, inside 32-lane halves
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (M << 10));
    else return (uint32_t)__shfl_xor((int)x, M, 64);  // 32, 63: across the halves
}

template <int M>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t x) {
    return ((uint64_t)lane_xor<M>((uint32_t)(x >> 32)) << 32) | lane_xor<M>((uint32_t)x);
}

// flip = 0: keep min(a, b); flip = ~0: keep max(a, b).  Keys are below 2^63 (a positive float's
// bits over a gid; padding 2^63 - 1), so the sign of a - b orders them; the select is a bit
// insert on that sign -- VALU only (a compare into an SGPR mask and a scalar XOR with the lane
// side would put a VALU -> SALU -> VALU round trip on every element).
// (m & x) | (~m & y) in one v_bfi_b32 (written out, the compiler turns it back into a compare
// into an SGPR mask + v_cndmask, with its s_nop hazard per element)
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(x), "v"(y));
    return r;
}

__device__ __forceinline__ uint64_t keep_side(uint64_t a, uint64_t b, uint32_t flip) {
    const uint32_t m = (uint32_t)((int64_t)(a - b) >> 63) ^ flip;  // ~0: keep a
    return ((uint64_t)bfi(m, (uint32_t)(a >> 32), (uint32_t)(b >> 32)) << 32) | bfi(m, (uint32_t)a, (uint32_t)b);
}

__device__ __forceinline__ void cas_up(uint64_t& a, uint64_t& b) {
    const uint32_t m = (uint32_t)((int64_t)(a - b) >> 63);  // ~0: a < b
    const uint32_t ah = (uint32_t)(a >> 32), al = (uint32_t)a, bh = (uint32_t)(b >> 32), bl = (uint32_t)b;
    a = ((uint64_t)bfi(m, ah, bh) << 32) | bfi(m, al, bl);
    b = ((uint64_t)bfi(m, bh, ah) << 32) | bfi(m, bl, al);
}

// half cleaners of distance J, J / 2, .., 1
template <int E, int J>
__device__ __forceinline__ void wave_half_cleaners(uint64_t (&v)[E], int lane) {
    if constexpr (J >= 1) {
        if constexpr (J >= E) {
            constexpr int L = J / E;
            const uint32_t flip = (lane & L) ? ~0u : 0u;
#pragma unroll
            for (int e = 0; e < E; ++e) v[e] = keep_side(v[e], lane_xor64<L>(v[e]), flip);
        } else {
#pragma unroll
            for (int e = 0; e < E; ++e)
                if ((e & J) == 0) cas_up(v[e], v[e ^ J]);
        }
        wave_half_cleaners<E, J / 2>(v, lane);
    }
}

// merges of size K, 2K, .., 64 E
template <int E, int K>
__device__ __forceinline__ void wave_bitonic(uint64_t (&v)[E], int lane) {
    if constexpr (K <= 64 * E) {
        if constexpr (K <= E) {
#pragma unroll
            for (int e = 0; e < E; ++e)
                if ((e & (K / 2)) == 0) cas_up(v[e], v[e ^ (K - 1)]);
        } else {
            // entry i = lane E + e pairs with i ^ (K - 1): lane ^ (K / E - 1), entry E - 1 - e
            constexpr int M = K / E - 1;
            const uint32_t flip = (lane & (K / (2 * E))) ? ~0u : 0u;
            if constexpr (E == 1) {
                v[0] = keep_side(v[0], lane_xor64<M>(v[0]), flip);
            } else {
#pragma unroll
                for (int e = 0; e < E / 2; ++e) {
                    const uint64_t pa = lane_xor64<M>(v[E - 1 - e]), pb = lane_xor64<M>(v[e]);
                    v[e] = keep_side(v[e], pa, flip);
                    v[E - 1 - e] = keep_side(v[E - 1 - e], pb, flip);
                }
            }
        }
        wave_half_cleaners<E, K / 4>(v, lane);
        wave_bitonic<E, 2 * K>(v, lane);
    }
}

// The slice is read coalesced (entry e * 64 + lane into register e: the network sorts whatever
// order it is given) and, sorted (rank lane E + e in register e), written back through the wave's
// LDS rows so the stores are coalesced too (`xs`: 64 E + 64 E / 32 words, rows padded against bank
// conflicts).
template <int E>
__device__ __forceinline__ void wave_sort_slice(const uint2 rg, const uint32_t* __restrict__ depth_key,
                                                uint32_t* __restrict__ gid, int lane, uint32_t* xs,
                                                const uint2* __restrict__ src = nullptr) {
    const int n = (int)(rg.y - rg.x);
    uint64_t v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = e * 64 + lane;
        uint64_t k = 0x7FFFFFFFFFFFFFFFull;  // padding sorts last (no real key reaches it)
        if (i < n) {
            if (src) {  // the placed (gid, key) pairs
                const uint2 p = src[rg.x + i];
                k = ((uint64_t)p.y << 32) | p.x;
            } else {
                const uint32_t g = gid[rg.x + i];
                k = ((uint64_t)depth_key[g] << 32) | g;
            }
        }
        v[e] = k;
    }
    wave_bitonic<E, 2>(v, lane);
    auto pad = [](int i) { return i + (i >> 5); };
#pragma unroll
    for (int e = 0; e < E; ++e) xs[pad(lane * E + e)] = (uint32_t)v[e];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = e * 64 + lane;
        if (i < n) gid[rg.x + i] = xs[pad(i)];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // xs reused by the wave's next slice
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- the same network on 32-bit keys (slices of <= 1024 entries) ----
// Key = the slice's top 22 differing depth bits over the entry's slice position (10 bits): half
// the cross-lane traffic of the 64-bit key (one DPP / swizzle / bpermute per exchange, not two)
// and a compare-exchange of one v_min_u32 + one v_max_u32.  Entries whose truncated depths are
// equal (the depth bits below the top 22 differing ones, or the whole depth, tie) come out in
// slice-position order; they are put in (depth, gid) order afterwards from the full keys -- in
// place by the lane holding a run's first entry when the run is short, else by the 64-bit form.
constexpr int kWaveKeyBits = 22, kWaveRunMax = 16;

__device__ __forceinline__ void cas_up32(uint32_t& a, uint32_t& b) {
    const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}

__device__ __forceinline__ uint32_t keep_side32(uint32_t a, uint32_t b, uint32_t flip) {
    return bfi(flip, a > b ? a : b, a < b ? a : b);  // flip = ~0: max
}

template <int E, int J>
__device__ __forceinline__ void wave_half_cleaners32(uint32_t (&v)[E], int lane) {
    if constexpr (J >= 1) {
        if constexpr (J >= E) {
            constexpr int L = J / E;
            const uint32_t flip = (lane & L) ? ~0u : 0u;
#pragma unroll
            for (int e = 0; e < E; ++e) v[e] = keep_side32(v[e], lane_xor<L>(v[e]), flip);
        } else {
#pragma unroll
            for (int e = 0; e < E; ++e)
                if ((e & J) == 0) cas_up32(v[e], v[e ^ J]);
        }
        wave_half_cleaners32<E, J / 2>(v, lane);
    }
}

template <int E, int K>
__device__ __forceinline__ void wave_bitonic32(uint32_t (&v)[E], int lane) {
    if constexpr (K <= 64 * E) {
        if constexpr (K <= E) {
#pragma unroll
            for (int e = 0; e < E; ++e)
                if ((e & (K / 2)) == 0) cas_up32(v[e], v[e ^ (K - 1)]);
        } else {
            constexpr int M = K / E - 1;
            const uint32_t flip = (lane & (K / (2 * E))) ? ~0u : 0u;
            if constexpr (E == 1) {
                v[0] = keep_side32(v[0], lane_xor<M>(v[0]), flip);
            } else {
#pragma unroll
                for (int e = 0; e < E / 2; ++e) {
                    const uint32_t pa = lane_xor<M>(v[E - 1 - e]), pb = lane_xor<M>(v[e]);
                    v[e] = keep_side32(v[e], pa, flip);
                    v[E - 1 - e] = keep_side32(v[E - 1 - e], pb, flip);
                }
            }
        }
        wave_half_cleaners32<E, K / 4>(v, lane);
        wave_bitonic32<E, 2 * K>(v, lane);
    }
}

template <int E>
__device__ __forceinline__ void wave_sort_slice32(const uint2 rg, const uint32_t* __restrict__ depth_key,
                                                  uint32_t* __restrict__ gid, int lane, uint32_t* xs,
                                                  const uint2* __restrict__ src = nullptr) {
    static_assert(64 * E <= (1 << (32 - kWaveKeyBits)), "slice position bits");
    constexpr uint32_t kPos = (1u << (32 - kWaveKeyBits)) - 1u;
    const int n = (int)(rg.y - rg.x);
    uint32_t v[E], dk[E];
    uint32_t kor = 0u, kand = ~0u;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = e * 64 + lane;
        dk[e] = 0u;
        if (i < n) {
            dk[e] = src ? src[rg.x + i].y : depth_key[gid[rg.x + i]];
            kor |= dk[e];
            kand &= dk[e];
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        kor |= __shfl_xor(kor, o, 64);
        kand &= __shfl_xor(kand, o, 64);
    }
    const uint32_t dif = kor ^ kand;
    const int top = dif ? 32 - __clz(dif) : 0;  // differing bits [0, top)
    const int sh = top > kWaveKeyBits ? top - kWaveKeyBits : 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = e * 64 + lane;
        // padding ~0 sorts last: a real key reaches it only as the last of 1024 entries
        v[e] = i < n ? (((dk[e] >> sh) & ((1u << kWaveKeyBits) - 1u)) << (32 - kWaveKeyBits)) | (uint32_t)i : ~0u;
    }
    wave_bitonic32<E, 2>(v, lane);
    auto pad = [](int i) { return i + (i >> 5); };
#pragma unroll
    for (int e = 0; e < E; ++e) xs[pad(lane * E + e)] = v[e];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // runs of equal truncated keys: the lane holding a run's first entry orders it by the full
    // (depth, gid) key (insertion; the slice's gids are still in place in gid[])
    auto full = [&](uint32_t x) {
        if (src) {
            const uint2 p = src[rg.x + (x & kPos)];
            return ((uint64_t)p.y << 32) | p.x;
        }
        const uint32_t g = gid[rg.x + (x & kPos)];
        return ((uint64_t)depth_key[g] << 32) | g;
    };
    bool tie = false, longrun = false;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int r = lane * E + e;
        if (r + 1 < n && (v[e] >> (32 - kWaveKeyBits)) == (xs[pad(r + 1)] >> (32 - kWaveKeyBits))) tie = true;
    }
    if (__ballot(tie)) {  // wave-uniform; rare
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int r = lane * E + e;
            const uint32_t top_r = v[e] >> (32 - kWaveKeyBits);
            if (r + 1 >= n || (xs[pad(r + 1)] >> (32 - kWaveKeyBits)) != top_r) continue;
            if (r > 0 && (xs[pad(r - 1)] >> (32 - kWaveKeyBits)) == top_r) continue;  // not the run's first
            int end = r + 2;
            while (end < n && (xs[pad(end)] >> (32 - kWaveKeyBits)) == top_r && end - r <= kWaveRunMax) ++end;
            if (end - r > kWaveRunMax) {
                longrun = true;
                continue;
            }
            for (int a = r + 1; a < end; ++a) {
                const uint32_t x = xs[pad(a)];
                const uint64_t fx = full(x);
                int b = a;
                while (b > r && full(xs[pad(b - 1)]) > fx) {
                    xs[pad(b)] = xs[pad(b - 1)];
                    --b;
                }
                xs[pad(b)] = x;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (__ballot(longrun)) {  // many entries at one truncated depth: the 64-bit form
            wave_sort_slice<E>(rg, depth_key, gid, lane, xs, src);
            return;
        }
    }
    // every read of the slice's gids completes before the first store over them (the compiler
    // would otherwise store each result as soon as its own load returned, while later loads of the
    // same slice were still in flight)
    uint32_t og[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = e * 64 + lane;
        const uint32_t at = rg.x + (xs[pad(i)] & kPos);
        og[e] = i < n ? (src ? src[at].x : gid[at]) : 0u;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = e * 64 + lane;
        if (i < n) gid[rg.x + i] = og[e];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // xs reused by the wave's next slice
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef GSR_WAVE_KEY32
#define GSR_WAVE_KEY32 1
#endif

// Four tiles per 256-thread block, one per wave; slices longer than 1024 entries go to `ovf`.
__global__ __launch_bounds__(256) void tile_depth_wave(const uint2* __restrict__ ranges, int tile0, int ntiles,
                                                      const uint32_t* __restrict__ depth_key,
                                                      uint32_t* __restrict__ gid, uint32_t* __restrict__ ovf,
                                                      uint32_t* __restrict__ ovf_count,
                                                      const uint2* __restrict__ src) {
    __shared__ uint32_t xs_all[4][64 * 16 + 32];
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntiles) return;
    const int lane = threadIdx.x & 63;
    uint32_t* const xs = xs_all[threadIdx.x >> 6];
    const int tile = tile0 + t;
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    if (n <= 1 || n > 1024) {
        // src: the later forms sort in place in gid[] -- the slice's gids go there first
        if (src)
            for (int i = lane; i < n; i += 64) gid[rg.x + i] = src[rg.x + i].x;
        if (n > 1 && lane == 0) ovf[atomicAdd(ovf_count, 1u)] = (uint32_t)tile;
        return;
    }
    if (GSR_WAVE_KEY32) {
        if (n <= 64) wave_sort_slice32<1>(rg, depth_key, gid, lane, xs, src);
        else if (n <= 128) wave_sort_slice32<2>(rg, depth_key, gid, lane, xs, src);
        else if (n <= 256) wave_sort_slice32<4>(rg, depth_key, gid, lane, xs, src);
        else if (n <= 512) wave_sort_slice32<8>(rg, depth_key, gid, lane, xs, src);
        else wave_sort_slice32<16>(rg, depth_key, gid, lane, xs, src);
        return;
    }
    if (n <= 64) wave_sort_slice<1>(rg, depth_key, gid, lane, xs, src);
    else if (n <= 128) wave_sort_slice<2>(rg, depth_key, gid, lane, xs, src);
    else if (n <= 256) wave_sort_slice<4>(rg, depth_key, gid, lane, xs, src);
    else if (n <= 512) wave_sort_slice<8>(rg, depth_key, gid, lane, xs, src);
    else wave_sort_slice<16>(rg, depth_key, gid, lane, xs, src);
}

// The queued slices of 1025 .. 2048 entries, one wave each (a kernel of its own: the 32-entry-per-
// lane form needs ~230 VGPRs, which would cap the common form's occupancy at 2 waves per SIMD);
// longer ones go on to `ovf2` for the LDS form.  Launched only where the mean slice is near one
// wave's 1024 entries (multi-GPU bands at 1M: ~1060), where a good share of the slices exceed it;
// the queue length is on the device.
__global__ __launch_bounds__(256) void tile_depth_wave_queue(const uint2* __restrict__ ranges,
                                                            const uint32_t* __restrict__ depth_key,
                                                            uint32_t* __restrict__ gid,
                                                            const uint32_t* __restrict__ ovf,
                                                            const uint32_t* __restrict__ ovf_count,
                                                            uint32_t* __restrict__ ovf2,
                                                            uint32_t* __restrict__ ovf2_count) {
    __shared__ uint32_t xs_all[4][64 * 32 + 64];
    const uint32_t cnt = *ovf_count;
    const int lane = threadIdx.x & 63;
    uint32_t* const xs = xs_all[threadIdx.x >> 6];
    for (uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < cnt; q += gridDim.x * 4) {
        const uint32_t tile = ovf[q];
        const uint2 rg = ranges[tile];
        const int n = (int)(rg.y - rg.x);
        if (n > 2048) {
            if (lane == 0) ovf2[atomicAdd(ovf2_count, 1u)] = tile;
            continue;  // wave-uniform
        }
        wave_sort_slice<32>(rg, depth_key, gid, lane, xs);
    }
}

// ---- per-tile depth order, block form: slices of 1025 .. NW x 1024 entries (round 6) ----
// Each of the block's NW waves sorts 1024 entries of the slice with the register network on
// 32-bit keys (the slice's top differing depth bits over the entry's slice position, as the
// one-wave form: 20 bits over 12 at 4096 entries, 19 over 13 at 8192); the waves' runs are then
// merged by the same all-ascending network, its stages at distances >= 1024 exchanged through LDS
// (one write, a barrier and one read per entry; padded rows: conflict-free) and
// the rest inside each wave.  Against the LDS radix form (two or three counting passes of ~6
// barriers each, the digit-peer ballots, latency-bound per block, PMC round 6): ~log2(n)^2 / 2
// register stages, 3 (4096) or 6 (8192) LDS exchanges.  Runs of equal truncated keys are put in
// (depth, gid) order from the full keys by the thread holding a run's first entry; a run longer
// than kWaveRunMax (depths clustered inside one truncated step) leaves the slice untouched and
// hands the tile on (`false`) to the next queue, whose forms sort every bit.
// E: entries per lane (16: 1024 per wave; 8: 512 per wave, twice the waves per slice and one more
// level of LDS merges, for a shorter chain per block)
#ifndef GSR_BLOCK_E
#define GSR_BLOCK_E 16
#endif
constexpr int kBlkE = GSR_BLOCK_E;
__host__ __device__ constexpr int blk_pad(int i) { return i + (i >> 5); }
__host__ __device__ constexpr int ilog2c(int x) { return x <= 1 ? 0 : 1 + ilog2c(x >> 1); }
constexpr int kBlkW = 4096 / (64 * kBlkE), kBlkQW = 8192 / (64 * kBlkE);  // waves: <= 4096 / <= 8192
template <int NW>
struct BlockSortLds {
    uint32_t xs[blk_pad(NW * 64 * kBlkE)];
    uint32_t red[2][NW];
};

template <int NW>
__device__ __forceinline__ bool block_sort_slice(const uint2 rg, const uint32_t* __restrict__ depth_key,
                                                 uint32_t* __restrict__ gid, const uint2* __restrict__ src,
                                                 BlockSortLds<NW>& L) {
    constexpr int WE = 64 * kBlkE;  // entries per wave
    constexpr int CAP = NW * WE, NT = NW * 64;
    constexpr int PB = ilog2c(CAP);  // position bits
    constexpr int KB = 32 - PB;                           // truncated depth bits
    static_assert((1 << PB) == CAP, "position bits");
    constexpr uint32_t kPos = CAP - 1u;
    const int n = (int)(rg.y - rg.x);
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    // active waves: the power of two whose runs cover the slice (the rest only meet the barriers)
    int nwa = 1;
    while (nwa * WE < n) nwa <<= 1;
    const bool act = w < nwa;
    uint32_t v[kBlkE];
    uint32_t kor = 0u, kand = ~0u;
#pragma unroll
    for (int e = 0; e < kBlkE; ++e) {
        const int i = w * WE + e * 64 + lane;
        v[e] = 0u;
        if (i < n) {
            v[e] = src ? src[rg.x + i].y : depth_key[gid[rg.x + i]];
            kor |= v[e];
            kand &= v[e];
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        kor |= __shfl_xor(kor, o, 64);
        kand &= __shfl_xor(kand, o, 64);
    }
    if (lane == 0) {
        L.red[0][w] = kor;
        L.red[1][w] = kand;
    }
    __syncthreads();
    {
        uint32_t o_ = 0u, a_ = ~0u;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            o_ |= L.red[0][k];
            a_ &= L.red[1][k];
        }
        kor = o_;
        kand = a_;
    }
    const uint32_t dif = kor ^ kand;
    const int top = dif ? 32 - __clz(dif) : 0;  // differing bits [0, top)
    const int sh = top > KB ? top - KB : 0;
#pragma unroll
    for (int e = 0; e < kBlkE; ++e) {
        const int i = w * WE + e * 64 + lane;
        // padding ~0 sorts last: a real key reaches it only at position CAP - 1, i.e. n = CAP
        v[e] = i < n ? (((v[e] >> sh) & ((1u << KB) - 1u)) << PB) | (uint32_t)i : ~0u;
    }
    if (act) wave_bitonic32<kBlkE, 2>(v, lane);  // each active wave's WE entries, ascending
    // merges of the waves' runs: entry i = w WE + E lane + e
    const int i0 = w * WE + lane * kBlkE;
    uint32_t* const xs = L.xs;
    auto lds_stage = [&](int x, int h) {  // i <-> i ^ x, the lower of the pair (i & h == 0) keeps the min
        if (act) {
#pragma unroll
            for (int e = 0; e < kBlkE; ++e) xs[blk_pad(i0 + e)] = v[e];
        }
        __syncthreads();
        if (act) {
            const bool hi = (i0 & h) != 0;  // the same for the lane's E entries (h >= WE)
#pragma unroll
            for (int e = 0; e < kBlkE; ++e) {
                const uint32_t o = xs[blk_pad((i0 + e) ^ x)];
                v[e] = hi ? (v[e] > o ? v[e] : o) : (v[e] < o ? v[e] : o);
            }
        }
        __syncthreads();  // xs is rewritten by the next stage
    };
    for (int K = 2 * WE; K <= nwa * WE; K <<= 1) {  // block-uniform
        lds_stage(K - 1, K >> 1);                     // the mirror stage
        for (int J = K >> 2; J >= WE; J >>= 1) lds_stage(J, J);
        if (act) wave_half_cleaners32<kBlkE, WE / 2>(v, lane);
    }
    // the sorted keys by rank, then the runs of equal truncated keys
    if (act) {
#pragma unroll
        for (int e = 0; e < kBlkE; ++e) xs[blk_pad(i0 + e)] = v[e];
    }
    __syncthreads();
    bool tie = false;
    if (act) {
#pragma unroll
        for (int e = 0; e < kBlkE; ++e) {
            const int r = i0 + e;
            if (r + 1 < n && (v[e] >> PB) == (xs[blk_pad(r + 1)] >> PB)) tie = true;
        }
    }
    if (__syncthreads_or(tie)) {  // block-uniform
        auto full = [&](uint32_t x) {
            if (src) {
                const uint2 p = src[rg.x + (x & kPos)];
                return ((uint64_t)p.y << 32) | p.x;
            }
            const uint32_t g = gid[rg.x + (x & kPos)];
            return ((uint64_t)depth_key[g] << 32) | g;
        };
        bool longrun = false;
        if (act) {
#pragma unroll
            for (int e = 0; e < kBlkE; ++e) {
                const int r = i0 + e;
                const uint32_t top_r = v[e] >> PB;
                if (r + 1 >= n || (xs[blk_pad(r + 1)] >> PB) != top_r) continue;
                if (r > 0 && (xs[blk_pad(r - 1)] >> PB) == top_r) continue;  // not the run's first
                int end = r + 2;
                while (end < n && (xs[blk_pad(end)] >> PB) == top_r && end - r <= kWaveRunMax) ++end;
                if (end - r > kWaveRunMax) {
                    longrun = true;
                    continue;
                }
                if (end - r <= 4) {
                    // the common run (2 - 3 entries at 5M / 1080p): its full keys loaded together --
                    // one global round trip, not one per insertion step -- and a 4-entry network
                    uint32_t xx[4];
                    uint64_t fk[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const bool in = r + j < end;
                        xx[j] = in ? xs[blk_pad(r + j)] : 0u;
                        fk[j] = in ? full(xx[j]) : ~0ull;
                    }
                    auto cx = [&](int a, int b) {
                        if (fk[b] < fk[a]) {
                            const uint64_t t = fk[a];
                            fk[a] = fk[b];
                            fk[b] = t;
                            const uint32_t u = xx[a];
                            xx[a] = xx[b];
                            xx[b] = u;
                        }
                    };
                    cx(0, 1);
                    cx(2, 3);
                    cx(0, 2);
                    cx(1, 3);
                    cx(1, 2);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (r + j < end) xs[blk_pad(r + j)] = xx[j];
                    continue;
                }
                for (int a = r + 1; a < end; ++a) {  // insertion by the full (depth, gid) key
                    const uint32_t x = xs[blk_pad(a)];
                    const uint64_t fx = full(x);
                    int b = a;
                    while (b > r && full(xs[blk_pad(b - 1)]) > fx) {
                        xs[blk_pad(b)] = xs[blk_pad(b - 1)];
                        --b;
                    }
                    xs[blk_pad(b)] = x;
                }
            }
        }
        if (__syncthreads_or(longrun)) return false;  // nothing written: the next form sorts it
    }
    // out in rank order (in place without src: every thread's reads of the slice's gids complete,
    // block-wide, before the first store over them)
    uint32_t og[CAP / NT];
#pragma unroll
    for (int k = 0; k < CAP / NT; ++k) {
        const int r = k * NT + tid;
        const uint32_t at = rg.x + (xs[blk_pad(r < n ? r : 0)] & kPos);
        og[k] = r < n ? (src ? src[at].x : gid[at]) : 0u;
    }
    if (!src) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < CAP / NT; ++k) {
        const int r = k * NT + tid;
        if (r < n) gid[rg.x + r] = og[k];
    }
    __syncthreads();  // xs / red are rewritten by the block's next slice
    return true;
}

#ifndef GSR_TILE_BLOCK_SORT
#define GSR_TILE_BLOCK_SORT 1
#endif
// launches of fewer tiles (multi-GPU bands) sort every deep slice with the 8-wave form in one round
#ifndef GSR_BLOCK8_TILES
#define GSR_BLOCK8_TILES 4096
#endif

// One block of NW waves per tile of the launch (slices of up to NW x 1024 entries); longer slices,
// and those with long runs of equal truncated keys, go to `ovf`: NW = 4 (full images) hands them to
// the 8-wave queue below, which reads src too; NW = 8 (band launches, ~1000 tiles: one round of
// blocks instead of two, the first one's 4096-entry sorts and then the queued longer ones) hands
// them to tile_depth_sort_big, which sorts in place -- their gids are copied to gid[] first.
template <int NW>
__global__ __launch_bounds__(NW * 64) void tile_depth_block(const uint2* __restrict__ ranges, int tile0,
                                                           const uint32_t* __restrict__ depth_key,
                                                           uint32_t* __restrict__ gid, uint32_t* __restrict__ ovf,
                                                           uint32_t* __restrict__ ovf_count,
                                                           const uint2* __restrict__ src) {
    __shared__ BlockSortLds<NW> lds;
    const int tile = tile0 + blockIdx.x;
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    if (n <= 1) {
        if (n == 1 && src && threadIdx.x == 0) gid[rg.x] = src[rg.x].x;
        return;
    }
    if (n > NW * 64 * kBlkE || !block_sort_slice<NW>(rg, depth_key, gid, src, lds)) {  // block-uniform
        if (NW == kBlkQW && src)
            for (int i = threadIdx.x; i < n; i += NW * 64) gid[rg.x + i] = src[rg.x + i].x;
        if (threadIdx.x == 0) ovf[atomicAdd(ovf_count, 1u)] = (uint32_t)tile;
    }
}

// The queued slices of up to 8192 entries, eight waves per block, one queued tile per block (the
// grid covers every tile; blocks past the queue's length exit at once); longer ones and those with
// long truncated-key runs go on to `ovf2` (tile_depth_sort_big sorts every bit).
__global__ __launch_bounds__(64 * kBlkQW) void tile_depth_block_queue(const uint2* __restrict__ ranges,
                                                             const uint32_t* __restrict__ depth_key,
                                                             uint32_t* __restrict__ gid,
                                                             const uint32_t* __restrict__ ovf,
                                                             const uint32_t* __restrict__ ovf_count,
                                                             uint32_t* __restrict__ ovf2,
                                                             uint32_t* __restrict__ ovf2_count,
                                                             const uint2* __restrict__ src) {
    __shared__ BlockSortLds<kBlkQW> lds;
    if (blockIdx.x >= *ovf_count) return;
    const uint32_t tile = ovf[blockIdx.x];
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    if (n > 8192 || !block_sort_slice<kBlkQW>(rg, depth_key, gid, src, lds)) {  // block-uniform
        // tile_depth_sort_big sorts in place in gid[]: the slice's gids go there first
        if (src)
            for (int i = threadIdx.x; i < n; i += 64 * kBlkQW) gid[rg.x + i] = src[rg.x + i].x;
        if (threadIdx.x == 0) ovf2[atomicAdd(ovf2_count, 1u)] = tile;
    }
}

// One block per tile of the launch; slices longer than NT * I go to the queue `ovf`.
template <int NT, int I, int DB>
__global__ __launch_bounds__(NT) void tile_depth_radix(const uint2* __restrict__ ranges, int tile0,
                                                      const uint32_t* __restrict__ depth_key,
                                                      uint32_t* __restrict__ gid, uint32_t* __restrict__ ovf,
                                                      uint32_t* __restrict__ ovf_count, int unordered) {
    const int tile = tile0 + blockIdx.x;
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    if (n <= 1) return;
    if (n > NT * I) {
        if (threadIdx.x == 0) ovf[atomicAdd(ovf_count, 1u)] = (uint32_t)tile;
        return;
    }
    __shared__ SliceLds<NT, I, DB> lds;
    radix_sort_slice<NT, I, DB>(rg, depth_key, gid, lds, unordered != 0);
}

// The queued (longer) slices: blocks walk the queue; slices longer than NT * I go on to the
// second queue (ovf2), which the global-memory form drains.  The queue length is on the device,
// so blocks past it exit at once.
template <int NT, int I, int DB>
__global__ __launch_bounds__(NT) void tile_depth_radix_queue(const uint2* __restrict__ ranges,
                                                            const uint32_t* __restrict__ depth_key,
                                                            uint32_t* __restrict__ gid,
                                                            const uint32_t* __restrict__ ovf,
                                                            const uint32_t* __restrict__ ovf_count,
                                                            uint32_t* __restrict__ ovf2, uint32_t* __restrict__ ovf2_count,
                                                            int unordered) {
    __shared__ SliceLds<NT, I, DB> lds;
    const uint32_t cnt = *ovf_count;
    for (uint32_t q = blockIdx.x; q < cnt; q += gridDim.x) {
        const uint32_t tile = ovf[q];
        const uint2 rg = ranges[tile];
        if ((int)(rg.y - rg.x) > NT * I) {
            if (threadIdx.x == 0) ovf2[atomicAdd(ovf2_count, 1u)] = tile;
            continue;  // block-uniform
        }
        radix_sort_slice<NT, I, DB>(rg, depth_key, gid, lds, unordered != 0);
    }
}

// Slices of 8193 and more entries (dense tiles of training views): one kernel, 1024-thread
// blocks, 8 work items per queued tile.  A slice of <= 16384 entries is sorted whole in LDS by
// item 0 (~145 KB: gfx950 gives one workgroup up to 160 KiB).  A longer slice is cut into
// 16384-entry chunks, sorted in place by the tile's items in parallel (a chunk is in gid order,
// so the stable depth sort leaves it in (depth, gid) order), and the item that finishes last
// (a per-tile counter, device-scope fences on both sides) merges them: the rest of an
// all-ascending ("flip") bitonic network over the range padded to a power of two, whose stages
// through size 16384 the sorted chunks already satisfy.  Strides >= 16384 run in global memory
// on the 64-bit (depth << 32 | gid) key split over two u32 arrays (the tile sort's free
// ping-pong pair); shorter strides in LDS one chunk at a time.  A 40k-entry tile takes 3 global
// passes and 2 x 3 LDS chunk passes instead of the 136 global passes of a plain bitonic sort.
constexpr int kBigChunk = 16384;
using BigSliceLds = SliceLds<1024, 16, 8>;
static_assert(sizeof(BigSliceLds) >= kBigChunk * sizeof(uint64_t), "merge chunk aliases the slice LDS");

// One bitonic half-cleaner stage (pairs i <-> i + d) over the LDS chunk.  The chunk is padded
// with ~0 sentinels, which no real (depth, gid) pair reaches (gid < 2^32-1).
__device__ __forceinline__ void lds_half_cleaner(uint64_t* sk, int d) {
    for (int t = threadIdx.x; t < kBigChunk / 2; t += 1024) {
        const int i = ((t & ~(d - 1)) << 1) | (t & (d - 1));
        const uint64_t a = sk[i], b = sk[i + d];
        if (a > b) sk[i] = b, sk[i + d] = a;
    }
    __syncthreads();
}

// The big form's LDS: the slice sort's arrays, or the merge's 16384 packed keys.  At namespace
// scope so that the two out-of-line phases below address it as LDS directly; each has the
// 128-VGPR budget of a 1024-thread block to itself (inlined into one loop nest, the slice
// sort's 48 key / value / rank registers spilled).
__shared__ union BigLds {
    BigSliceLds slice;
    uint64_t sk[kBigChunk];
} g_big;

__device__ __attribute__((noinline)) void big_slice_sort(const uint2 rg, const uint32_t* __restrict__ depth_key,
                                                         uint32_t* __restrict__ gid, bool unordered) {
    radix_sort_slice<1024, 16, 8, true>(rg, depth_key, gid, g_big.slice, unordered);
}

__device__ __attribute__((noinline)) void merge_sorted_chunks(const uint2 r, const uint32_t* __restrict__ depth_key,
                                                              uint32_t* __restrict__ gid, uint32_t* __restrict__ hi,
                                                              uint32_t* __restrict__ lo) {
    uint64_t* const sk = g_big.sk;
    const int n = (int)(r.y - r.x);
    int m = kBigChunk;
    while (m < n) m <<= 1;
    const int nch = (n + kBigChunk - 1) / kBigChunk;
    uint32_t* H = hi + r.x;
    uint32_t* L = lo + r.x;
    for (int i = threadIdx.x; i < n; i += 1024) {
        const uint32_t g = gid[r.x + i];
        H[i] = depth_key[g];
        L[i] = g;
    }
    __syncthreads();
    auto cex = [&](int i, int j) {  // i < j; indices >= n are +inf padding
        if (j >= n) return;
        const uint64_t a = ((uint64_t)H[i] << 32) | L[i], b = ((uint64_t)H[j] << 32) | L[j];
        if (a > b) {
            H[i] = (uint32_t)(b >> 32), L[i] = (uint32_t)b;
            H[j] = (uint32_t)(a >> 32), L[j] = (uint32_t)a;
        }
    };
    for (int size = 2 * kBigChunk; size <= m; size <<= 1) {
        for (int d = size >> 1; d >= kBigChunk; d >>= 1) {
            const bool flip = d == (size >> 1);
            for (int t = threadIdx.x; t < (m >> 1); t += 1024) {
                const int i = ((t & ~(d - 1)) << 1) | (t & (d - 1));
                cex(i, flip ? (i ^ (size - 1)) : (i + d));
            }
            __syncthreads();
        }
        const bool last = size == m;
        for (int c = 0; c < nch; ++c) {
            const int base = c * kBigChunk;
            for (int i = threadIdx.x; i < kBigChunk; i += 1024)
                sk[i] = base + i < n ? (((uint64_t)H[base + i] << 32) | L[base + i]) : ~0ull;
            __syncthreads();
            for (int d = kBigChunk >> 1; d >= 1; d >>= 1) lds_half_cleaner(sk, d);
            for (int i = threadIdx.x; i < kBigChunk && base + i < n; i += 1024) {
                const uint64_t v = sk[i];
                if (last) {
                    gid[r.x + base + i] = (uint32_t)v;
                } else {
                    H[base + i] = (uint32_t)(v >> 32);
                    L[base + i] = (uint32_t)v;
                }
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(1024) void tile_depth_sort_big(const uint2* __restrict__ ranges,
                                                            const uint32_t* __restrict__ depth_key,
                                                            uint32_t* __restrict__ gid,
                                                            const uint32_t* __restrict__ ovf,
                                                            const uint32_t* __restrict__ ovf_count,
                                                            uint32_t* __restrict__ done,
                                                            uint32_t* __restrict__ hi, uint32_t* __restrict__ lo,
                                                            int unordered) {
    __shared__ uint32_t last;
    const uint32_t cnt = *ovf_count;
    // item-major: the first cnt work items are every tile's item 0, spread over all blocks
    for (uint32_t w = blockIdx.x; w < 8u * cnt; w += gridDim.x) {
        const uint32_t q = w % cnt, item = w / cnt;
        const uint2 r = ranges[ovf[q]];
        const uint32_t n = r.y - r.x;
        // a slice of <= kBigChunk entries is item 0's whole; a longer one is cut into chunks
        const bool whole = n <= (uint32_t)kBigChunk;
        const uint32_t nch = whole ? 1u : (n + kBigChunk - 1) / kBigChunk;
        const uint32_t parts = nch < 8u ? nch : 8u;
        if (item >= parts) continue;  // block-uniform
        for (uint32_t c0 = r.x + item * kBigChunk; c0 < r.y; c0 += 8u * kBigChunk) {
            const uint32_t c1 = whole || c0 + kBigChunk >= r.y ? r.y : c0 + kBigChunk;
            big_slice_sort(make_uint2(c0, c1), depth_key, gid, unordered != 0);
        }
        if (whole) continue;
        __threadfence();  // this item's chunks visible device-wide before it counts itself done
        __syncthreads();
        if (threadIdx.x == 0) last = atomicAdd(done + q, 1u) == parts - 1u ? 1u : 0u;
        __syncthreads();
        if (!last) continue;  // block-uniform
        __threadfence();      // acquire: the other items' chunks
        merge_sorted_chunks(r, depth_key, gid, hi, lo);
    }
}
}  // namespace

int radix_sort(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* k0, uint32_t* v0,
               uint32_t* k1, uint32_t* v1, long long cap, const uint32_t* n_dev, int nbits, uint32_t* hist,
               int* which, hipStream_t s) {
    *which = -1;
    if (cap <= 0) return 0;
    const int nb = radix_blocks(cap);
    uint32_t* totals = hist + (size_t)256 * (nb + 1);
    const uint32_t* kin = keys_in;
    const uint32_t* vin = vals_in;
    int dst = 0;
    // the fewest 8-bit-or-narrower passes, digits split evenly (13 tile bits: 7 + 6, not 8 + 5:
    // half the buckets in the first pass, so each block's runs to scatter are twice as long;
    // 0.114 vs 0.120 ms at 1M / 1080p, 0.486 vs 0.512 at 5M)
    const int passes = (nbits + 7) / 8, per = (nbits + passes - 1) / passes;
    for (int shift = 0; shift < nbits; shift += per) {
        const int bits = (nbits - shift) < per ? (nbits - shift) : per;
        uint32_t* ko = dst == 0 ? k0 : k1;
        uint32_t* vo = dst == 0 ? v0 : v1;
        if (radix_tile_for(cap) == kRadixTile) {
            hipLaunchKernelGGL(radix_upsweep<kRadixItems>, dim3(nb), dim3(kB), 0, s, kin, cap, n_dev, shift, bits, nb,
                               hist);
            hipLaunchKernelGGL(radix_colscan, dim3(256), dim3(kB), 0, s, hist, nb, totals);
            hipLaunchKernelGGL(radix_downsweep<kRadixItems>, dim3(nb), dim3(kB), 0, s, kin, vin, ko, vo, cap, n_dev,
                               shift, bits, nb, hist, totals);
        } else {
            hipLaunchKernelGGL(radix_upsweep<kRadixItemsSmall>, dim3(nb), dim3(kB), 0, s, kin, cap, n_dev, shift, bits,
                               nb, hist);
            hipLaunchKernelGGL(radix_colscan, dim3(256), dim3(kB), 0, s, hist, nb, totals);
            hipLaunchKernelGGL(radix_downsweep<kRadixItemsSmall>, dim3(nb), dim3(kB), 0, s, kin, vin, ko, vo, cap,
                               n_dev, shift, bits, nb, hist, totals);
        }
        kin = ko;
        vin = vo;
        *which = dst;
        dst ^= 1;
    }
    return (int)hipGetLastError();
}

int launch_scan(const uint32_t* tiles, int n, uint32_t* offsets, uint32_t* scan_partials_buf, uint32_t* total_out,
                hipStream_t s, bool fused_ok) {
    if (n <= 0) return (int)hipMemsetAsync(total_out, 0, sizeof(uint32_t), s);
    if (fused_ok && n <= kFusedScanMax) return 0;  // scanned by the fused kernel in launch_duplicate
    const int nb = sort_blocks(n);
    hipLaunchKernelGGL(scan_reduce, dim3(nb), dim3(kB), 0, s, tiles, n, scan_partials_buf);
    hipLaunchKernelGGL(scan_partials, dim3(1), dim3(1024), scan_lds_bytes(nb), s, scan_partials_buf, nb, total_out);
    hipLaunchKernelGGL(scan_downsweep, dim3(nb), dim3(kB), 0, s, tiles, n, scan_partials_buf, offsets);
    return (int)hipGetLastError();
}

// one block of 256 Gaussians: offsets = its scanned base + the in-block inclusive scan
__global__ __launch_bounds__(256) void block_offsets_kernel(const uint32_t* __restrict__ tiles, int n,
                                                            const uint32_t* __restrict__ bsum,
                                                            uint32_t* __restrict__ offsets) {
    __shared__ uint32_t wsum[kWaves];
    const int g = blockIdx.x * 256 + threadIdx.x;
    const uint32_t nt = g < n ? tiles[g] : 0u;
    uint32_t tdum;
    const uint32_t incl = bsum[blockIdx.x] + block_exclusive_scan(nt, wsum, &tdum) + nt;
    if (g < n) offsets[g] = incl;
}

int launch_scan_blocks(uint32_t* bsum, int n, uint32_t* total_out, hipStream_t s) {
    if (n <= 0) return (int)hipMemsetAsync(total_out, 0, sizeof(uint32_t), s);
    hipLaunchKernelGGL(scan_partials, dim3(1), dim3(1024), scan_lds_bytes(div_up(n, 256)), s, bsum, div_up(n, 256),
                       total_out);
    return (int)hipGetLastError();
}

int launch_block_offsets(const uint32_t* tiles, int n, const uint32_t* bsum, uint32_t* offsets, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(block_offsets_kernel, dim3(div_up(n, 256)), dim3(256), 0, s, tiles, n, bsum, offsets);
    return (int)hipGetLastError();
}

int launch_rb_binning(const uint32_t* tiles, uint4* rect, uint32_t* offsets, int n, int gx, int ty0, int ty1,
                      uint32_t* histA, uint32_t* histB, uint32_t* rb_status, uint32_t* pgid, uint32_t* pxr,
                      uint32_t* tkey, uint32_t* tgid, uint2* ranges, long long cap, hipStream_t s,
                      bool rows_counted, const uint32_t* bsum, uint32_t* K_dev, const uint32_t* depth_key,
                      uint2* ppair, uint2* tpair) {
    const int R = ty1 - ty0;
    if (!depth_key || !ppair || !tpair) ppair = tpair = nullptr;
    if (n <= 0 || R <= 0 || cap <= 0) return 0;  // ranges stay cleared
    if (R > kRbMaxRows || gx > kRbMaxCols || cap >= kRbMaxCap) return (int)hipErrorInvalidValue;
    const int nbA = div_up(n, 256);
    uint32_t* const totA = histA + (size_t)256 * nbA;
    if (!rows_counted)
        hipLaunchKernelGGL(rb_rows_count, dim3(nbA), dim3(256), 0, s, tiles, rect, n, ty0, ty1, histA, nbA);
    hipLaunchKernelGGL(rb_colscan, dim3(R), dim3(1024), scan_lds_bytes(nbA), s, histA, nbA, totA);
    hipLaunchKernelGGL(rb_rows_place, dim3(nbA), dim3(256), 0, s, tiles, rect, offsets, bsum, n, ty0, ty1, histA, totA,
                       nbA, pgid, pxr, cap, depth_key, ppair);
    // chunks: at most cap / kRbChunk full ones plus one partial per row; the blocks walk them, so
    // the grid is capped near what the chip holds at once (no tail of empty blocks)
    const int nch_max = div_up(cap, kRbChunk) + R;
    const int gcount = nch_max < 2048 ? nch_max : 2048, gplace = nch_max < 1280 ? nch_max : 1280;
    hipLaunchKernelGGL(rb_chunks_count, dim3(gcount), dim3(256), 0, s, pxr, totA, R, gx, cap, histB);
    // partitions per row: enough to spread a band's few rows over the chip, at most kRbScanSplit
    int G = kRbScanSplit < 256 / R ? kRbScanSplit : 256 / R;
    G = G < 1 ? 1 : G > gx ? gx : G;
    hipLaunchKernelGGL(rb_tiles_scan, dim3(R * G), dim3(kRbScanThreads), 0, s, totA, R, gx, ty0, cap, cap, histB,
                       rb_status + 16, rb_status, ranges, K_dev, G);
    hipLaunchKernelGGL(rb_chunks_place, dim3(gplace), dim3(256), 0, s, pgid, pxr, totA, R, gx, ty0, cap, cap, histB,
                       tkey, tgid, ppair, tpair);
    return (int)hipGetLastError();
}

int launch_duplicate(const uint32_t* tiles, uint4* rect, int n, int grid_x, int ty0, uint32_t* offsets,
                     uint32_t* lookback, uint32_t* tkey, uint32_t* tgid, long long cap, uint32_t* total_out,
                     hipStream_t s, bool scanned) {
    if (n <= 0) return 0;
    if (n <= kFusedScanMax && !scanned) {  // fused look-back scan + duplicate
        const int nb = div_up(n, 256);
        if (hipError_t e = hipMemsetAsync(lookback, 0, sizeof(uint32_t) * (16 + (size_t)nb), s)) return (int)e;
        hipLaunchKernelGGL(scan_duplicate_kernel, dim3(nb), dim3(256), 0, s, tiles, rect, n, grid_x, ty0, offsets,
                           tkey, tgid, cap, lookback + 16, lookback, total_out);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(duplicate_kernel<false>, dim3(div_up(n, 256)), dim3(256), 0, s, offsets, tiles, rect,
                       nullptr, n, grid_x, ty0, tkey, tgid, cap, nullptr);
    return (int)hipGetLastError();
}

int launch_depth_presort(const uint32_t* depth_key, const uint32_t* tiles, const uint4* rect, int n, uint32_t* dk0,
                         uint32_t* dv0, uint32_t* dk1, uint32_t* dv1, uint32_t* hist, uint32_t* rtiles, uint4* rrect,
                         uint32_t* bsum, uint32_t* total_out, hipStream_t s) {
    if (n <= 0) return (int)hipMemsetAsync(total_out, 0, sizeof(uint32_t), s);
    int which = -1;  // 4 passes of 8 bits: the result lands in (dk1, dv1)
    if (int e = radix_sort(depth_key, nullptr, dk0, dv0, dk1, dv1, n, nullptr, 32, hist, &which, s)) return e;
    const uint32_t* sgid = which == 0 ? dv0 : dv1;
    const int nb = div_up(n, 256);
    hipLaunchKernelGGL(rank_payload_kernel, dim3(nb), dim3(256), 0, s, sgid, tiles, rect, n, rtiles, rrect, bsum);
    // the 256-rank blocks' exclusive offsets and K: F3 (launch_duplicate_ranked) scans inside them
    hipLaunchKernelGGL(scan_partials, dim3(1), dim3(1024), scan_lds_bytes(nb), s, bsum, nb, total_out);
    return (int)hipGetLastError();
}

int launch_duplicate_ranked(const uint32_t* rtiles, const uint4* rrect, uint4* rect, int n, int grid_x, int ty0,
                            const uint32_t* bexcl, uint32_t* offsets, uint32_t* tkey, uint32_t* tgid, long long cap,
                            hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(duplicate_kernel<true>, dim3(div_up(n, 256)), dim3(256), 0, s, offsets, rtiles, rect, rrect, n,
                       grid_x, ty0, tkey, tgid, cap, bexcl);
    return (int)hipGetLastError();
}

// the gids of placed (gid, depth key) pairs, for the forms that sort gid[] in place
__global__ __launch_bounds__(256) void copy_pair_gids(const uint2* __restrict__ src, long long n,
                                                      uint32_t* __restrict__ gid) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) gid[i] = src[i].x;
}

// the LDS slice capacity the per-tile sort picks for a mean slice of K / ntiles entries
static int tile_sort_cap(long long K, int ntiles) {
    const long long mean = ntiles > 0 ? K / ntiles : K;
    int cap = 1024;
    while (cap < 4096 && cap < mean + mean / 2) cap <<= 1;
    return cap;
}

bool tile_wave_sort_eligible(long long K, int ntiles) { return GSR_TILE_WAVE_SORT && tile_sort_cap(K, ntiles) <= 2048; }

int launch_tile_depth_sort(const uint2* ranges, int tile0, int ntiles, long long K, const uint32_t* depth_key,
                           uint32_t* gid, uint32_t* ovf, uint32_t* ovf_count, uint32_t* ovf2, uint32_t* ovf2_count,
                           uint32_t* done, uint32_t* scratch_hi, uint32_t* scratch_lo, hipStream_t s,
                           bool unordered, const uint2* src) {
    if (ntiles <= 0 || K <= 0) return 0;
    const int uo = unordered ? 1 : 0;
    // one block per tile holding up to cap entries in LDS, a power of two >= 1.5x the mean slice
    // (1024 .. 4096: <= 43 KB of LDS, 3 blocks per CU); longer slices queue for 512-thread blocks
    // of up to 8192 (73 KB: 2 per CU) walking the queue, and beyond that for tile_depth_sort_big
    // (one 8192-entry block per tile at 5M / 1080p: 0.89 ms with 512 threads, 0.79 with 1024,
    // against 0.49 for 4096-entry blocks + the queue: 1 block per CU)
    const int cap = tile_sort_cap(K, ntiles);
    // slices of up to 1024 entries sorted in registers, one wave each, whenever the
    // mean slice leaves most tiles within that (the longer ones queue for the LDS forms below)
    if (tile_wave_sort_eligible(K, ntiles)) {
        hipLaunchKernelGGL(tile_depth_wave, dim3(div_up(ntiles, 4)), dim3(256), 0, s, ranges, tile0, ntiles, depth_key,
                           gid, ovf, ovf_count, src);
        // the slices past one wave's 1024 entries: where the mean is near 1024 (bands), many -- a
        // 2048-entry wave each, the rest on to the LDS form; elsewhere few (none at 1M / 1080p) --
        // all straight to the 1024-thread LDS form, one launch instead of two more near-empty
        // ones (~5 us each)
        const int bgrid = ntiles < 256 ? ntiles : 256;
        if (K / ntiles > 900) {
            const int wgrid = ntiles < 2048 ? div_up(ntiles, 4) : 512;
            hipLaunchKernelGGL(tile_depth_wave_queue, dim3(wgrid), dim3(256), 0, s, ranges, depth_key, gid, ovf,
                               ovf_count, ovf2, ovf2_count);
            hipLaunchKernelGGL(tile_depth_sort_big, dim3(bgrid), dim3(1024), 0, s, ranges, depth_key, gid, ovf2,
                               ovf2_count, done, scratch_hi, scratch_lo, uo);
        } else {
            hipLaunchKernelGGL(tile_depth_sort_big, dim3(bgrid), dim3(1024), 0, s, ranges, depth_key, gid, ovf,
                               ovf_count, done, scratch_hi, scratch_lo, uo);
        }
        return (int)hipGetLastError();
    } else {
#define GSR_TILE_RADIX(NT_, I_)                                                                       \
    hipLaunchKernelGGL((tile_depth_radix<NT_, I_, 9>), dim3(ntiles), dim3(NT_), 0, s, ranges, tile0, depth_key, \
                       gid, ovf, ovf_count, uo)
#ifndef GSR_BAND_SORT_NT
#define GSR_BAND_SORT_NT 512
#endif
// full images: 256-thread blocks, or 512 when the mean slice is long (cap 4096; 0 = that rule):
// 5M / 1080p 0.550 -> 0.490 ms with 512, 1M / 1080p (cap 2048) 0.103 -> 0.111 ms, so per cap
#ifndef GSR_FULL_SORT_NT
#define GSR_FULL_SORT_NT 0
#endif
    if (src && !(GSR_TILE_BLOCK_SORT && cap == 4096)) {  // the radix forms sort in place: gids first
        hipLaunchKernelGGL(copy_pair_gids, dim3(div_up(K, 256)), dim3(256), 0, s, src, K, gid);
        src = nullptr;
    }
    if (GSR_TILE_BLOCK_SORT && cap == 4096 && ntiles < GSR_BLOCK8_TILES) {  // bands: 8 waves per tile
        hipLaunchKernelGGL(tile_depth_block<kBlkQW>, dim3(ntiles), dim3(64 * kBlkQW), 0, s, ranges, tile0, depth_key, gid, ovf2,
                           ovf2_count, src);
        const int bgrid = ntiles < 256 ? ntiles : 256;
        hipLaunchKernelGGL(tile_depth_sort_big, dim3(bgrid), dim3(1024), 0, s, ranges, depth_key, gid, ovf2,
                           ovf2_count, done, scratch_hi, scratch_lo, uo);
        return (int)hipGetLastError();
    }
    if (GSR_TILE_BLOCK_SORT && cap == 4096) {  // deep slices: the block form, then its 8192-entry queue
        hipLaunchKernelGGL(tile_depth_block<kBlkW>, dim3(ntiles), dim3(64 * kBlkW), 0, s, ranges, tile0, depth_key, gid, ovf,
                           ovf_count, src);
        hipLaunchKernelGGL(tile_depth_block_queue, dim3(ntiles), dim3(64 * kBlkQW), 0, s, ranges, depth_key, gid, ovf,
                           ovf_count, ovf2, ovf2_count, src);
        const int bgrid = ntiles < 256 ? ntiles : 256;
        hipLaunchKernelGGL(tile_depth_sort_big, dim3(bgrid), dim3(1024), 0, s, ranges, depth_key, gid, ovf2,
                           ovf2_count, done, scratch_hi, scratch_lo, uo);
        return (int)hipGetLastError();
    }
    if (ntiles < 4096 && GSR_BAND_SORT_NT == 512) {  // band launches: fewer tiles, wider blocks
        if (cap == 1024) GSR_TILE_RADIX(512, 2);
        else if (cap == 2048) GSR_TILE_RADIX(512, 4);
        else GSR_TILE_RADIX(512, 8);
    } else if (ntiles < 4096 && GSR_BAND_SORT_NT == 1024) {
        if (cap == 1024) GSR_TILE_RADIX(1024, 1);
        else if (cap == 2048) GSR_TILE_RADIX(1024, 2);
        else GSR_TILE_RADIX(1024, 4);
    } else if (GSR_FULL_SORT_NT == 512 || (GSR_FULL_SORT_NT == 0 && cap == 4096)) {
        if (cap == 1024) GSR_TILE_RADIX(512, 2);
        else if (cap == 2048) GSR_TILE_RADIX(512, 4);
        else GSR_TILE_RADIX(512, 8);
    } else if (GSR_FULL_SORT_NT == 1024) {
        if (cap == 1024) GSR_TILE_RADIX(1024, 1);
        else if (cap == 2048) GSR_TILE_RADIX(1024, 2);
        else GSR_TILE_RADIX(1024, 4);
    } else if (cap == 1024) GSR_TILE_RADIX(256, 4);
    else if (cap == 2048) GSR_TILE_RADIX(256, 8);
    else GSR_TILE_RADIX(256, 16);
#undef GSR_TILE_RADIX
    }
    const int qgrid = ntiles < 512 ? ntiles : 512;
    hipLaunchKernelGGL((tile_depth_radix_queue<512, 16, 8>), dim3(qgrid), dim3(512), 0, s, ranges, depth_key, gid, ovf,
                       ovf_count, ovf2, ovf2_count, uo);
    // slices beyond 8192: the 16384-entry LDS form and the chunked form (tile_depth_sort_big)
    const int bgrid = ntiles < 256 ? ntiles : 256;
    hipLaunchKernelGGL(tile_depth_sort_big, dim3(bgrid), dim3(1024), 0, s, ranges, depth_key, gid, ovf2, ovf2_count,
                       done, scratch_hi, scratch_lo, uo);
    return (int)hipGetLastError();
}

// The tile key of every listed instance from the ranges (the row-bucketed binning does not write
// them in the step: only the GSR_VIEW_SORTED_TILE accessor reads them)
__global__ __launch_bounds__(256) void tile_keys_from_ranges(const uint2* __restrict__ ranges, long long cap,
                                                             uint32_t* __restrict__ tkey) {
    const uint2 rg = ranges[blockIdx.x];
    const uint32_t e = rg.y < cap ? rg.y : (uint32_t)cap;
    for (uint32_t i = rg.x + threadIdx.x; i < e; i += 256) tkey[i] = blockIdx.x;
}

int launch_tile_keys_from_ranges(const uint2* ranges, int tiles, long long cap, uint32_t* tkey, hipStream_t s) {
    if (tiles <= 0 || cap <= 0) return 0;
    hipLaunchKernelGGL(tile_keys_from_ranges, dim3(tiles), dim3(256), 0, s, ranges, cap, tkey);
    return (int)hipGetLastError();
}

int launch_finalize(const uint32_t* sorted_tile, long long cap, const uint32_t* K_dev, uint2* ranges, hipStream_t s) {
    if (cap <= 0) return 0;
    hipLaunchKernelGGL(finalize_kernel, dim3(div_up(div_up(cap, kFinQ), 256)), dim3(256), 0, s, sorted_tile, cap, K_dev,
                       ranges);
    return (int)hipGetLastError();
}

}  // namespace gsr

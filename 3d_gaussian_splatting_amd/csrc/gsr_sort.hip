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

// exclusive scan of the nb block totals in place; the grand total to *total_out
__global__ __launch_bounds__(1024) void scan_partials(uint32_t* __restrict__ partials, int nb,
                                                      uint32_t* __restrict__ total_out) {
    __shared__ uint32_t wsum[16];
    uint32_t carry = 0;
    for (int base = 0; base < nb; base += 1024) {
        const int i = base + threadIdx.x;
        const uint32_t v = i < nb ? partials[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(v, wsum, &tot);
        if (i < nb) partials[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

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
template <int NT, int I, int DB>
struct SliceLds {
    uint32_t wcnt[NT / 64][1 << DB];
    uint32_t lbase[1 << DB];
    uint32_t red[2][NT / 64];
    uint32_t skey[NT * I];
    uint32_t sval[NT * I];
};

template <int NT, int I, int DB>
__device__ __forceinline__ void radix_sort_slice(const uint2 rg, const uint32_t* __restrict__ depth_key,
                                                 uint32_t* __restrict__ gid, SliceLds<NT, I, DB>& lds) {
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
    for (int shift = 0; shift < 32; shift += DB) {
        if (((diff >> shift) & DMASK) == 0u) continue;  // block-uniform
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
#pragma unroll
    for (int r = 0; r < I; ++r) {
        const int idx = base + r * 64 + lane;
        if (idx < end) gid[rg.x + idx] = val[r];
    }
    __syncthreads();  // red[] is rewritten by the next slice
}

// One block per tile of the launch; slices longer than NT * I go to the queue `ovf`.
template <int NT, int I, int DB>
__global__ __launch_bounds__(NT) void tile_depth_radix(const uint2* __restrict__ ranges, int tile0,
                                                      const uint32_t* __restrict__ depth_key,
                                                      uint32_t* __restrict__ gid, uint32_t* __restrict__ ovf,
                                                      uint32_t* __restrict__ ovf_count) {
    const int tile = tile0 + blockIdx.x;
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    if (n <= 1) return;
    if (n > NT * I) {
        if (threadIdx.x == 0) ovf[atomicAdd(ovf_count, 1u)] = (uint32_t)tile;
        return;
    }
    __shared__ SliceLds<NT, I, DB> lds;
    radix_sort_slice<NT, I, DB>(rg, depth_key, gid, lds);
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
                                                            uint32_t* __restrict__ ovf2, uint32_t* __restrict__ ovf2_count) {
    __shared__ SliceLds<NT, I, DB> lds;
    const uint32_t cnt = *ovf_count;
    for (uint32_t q = blockIdx.x; q < cnt; q += gridDim.x) {
        const uint32_t tile = ovf[q];
        const uint2 rg = ranges[tile];
        if ((int)(rg.y - rg.x) > NT * I) {
            if (threadIdx.x == 0) ovf2[atomicAdd(ovf2_count, 1u)] = tile;
            continue;  // block-uniform
        }
        radix_sort_slice<NT, I, DB>(rg, depth_key, gid, lds);
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
                                                         uint32_t* __restrict__ gid) {
    radix_sort_slice<1024, 16, 8>(rg, depth_key, gid, g_big.slice);
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
                                                            uint32_t* __restrict__ hi, uint32_t* __restrict__ lo) {
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
            big_slice_sort(make_uint2(c0, c1), depth_key, gid);
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
                hipStream_t s) {
    if (n <= 0) return (int)hipMemsetAsync(total_out, 0, sizeof(uint32_t), s);
    if (n <= kFusedScanMax) return 0;  // scanned by the fused kernel in launch_duplicate
    const int nb = sort_blocks(n);
    hipLaunchKernelGGL(scan_reduce, dim3(nb), dim3(kB), 0, s, tiles, n, scan_partials_buf);
    hipLaunchKernelGGL(scan_partials, dim3(1), dim3(1024), 0, s, scan_partials_buf, nb, total_out);
    hipLaunchKernelGGL(scan_downsweep, dim3(nb), dim3(kB), 0, s, tiles, n, scan_partials_buf, offsets);
    return (int)hipGetLastError();
}

int launch_duplicate(const uint32_t* tiles, uint4* rect, int n, int grid_x, int ty0, uint32_t* offsets,
                     uint32_t* lookback, uint32_t* tkey, uint32_t* tgid, long long cap, uint32_t* total_out,
                     hipStream_t s) {
    if (n <= 0) return 0;
    if (n <= kFusedScanMax) {  // fused look-back scan + duplicate
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
    hipLaunchKernelGGL(scan_partials, dim3(1), dim3(1024), 0, s, bsum, nb, total_out);
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

int launch_tile_depth_sort(const uint2* ranges, int tile0, int ntiles, long long K, const uint32_t* depth_key,
                           uint32_t* gid, uint32_t* ovf, uint32_t* ovf_count, uint32_t* ovf2, uint32_t* ovf2_count,
                           uint32_t* done, uint32_t* scratch_hi, uint32_t* scratch_lo,
                           hipStream_t s) {
    if (ntiles <= 0 || K <= 0) return 0;
    // one block per tile holding up to cap entries in LDS, a power of two >= 1.5x the mean slice
    // (1024 .. 4096: <= 43 KB of LDS, 3 blocks per CU); longer slices queue for 512-thread blocks
    // of up to 8192 (73 KB: 2 per CU) walking the queue, and beyond that for tile_depth_sort_big
    const long long mean = K / ntiles;
    int cap = 1024;
    // (one 8192-entry block per tile at 5M / 1080p: 0.89 ms with 512 threads, 0.79 with 1024,
    // against 0.49 for 4096-entry blocks + the queue: 1 block per CU)
    while (cap < 4096 && cap < mean + mean / 2) cap <<= 1;
#define GSR_TILE_RADIX(NT_, I_)                                                                          \
    hipLaunchKernelGGL((tile_depth_radix<NT_, I_, 9>), dim3(ntiles), dim3(NT_), 0, s, ranges, tile0, depth_key, \
                       gid, ovf, ovf_count)
#ifndef GSR_BAND_SORT_NT
#define GSR_BAND_SORT_NT 512
#endif
// full images: 256-thread blocks, or 512 when the mean slice is long (cap 4096; 0 = that rule):
// 5M / 1080p 0.550 -> 0.490 ms with 512, 1M / 1080p (cap 2048) 0.103 -> 0.111 ms, so per cap
#ifndef GSR_FULL_SORT_NT
#define GSR_FULL_SORT_NT 0
#endif
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
    const int qgrid = ntiles < 512 ? ntiles : 512;
    hipLaunchKernelGGL((tile_depth_radix_queue<512, 16, 8>), dim3(qgrid), dim3(512), 0, s, ranges, depth_key, gid, ovf,
                       ovf_count, ovf2, ovf2_count);
    // slices beyond 8192: the 16384-entry LDS form and the chunked form (tile_depth_sort_big)
    const int bgrid = ntiles < 256 ? ntiles : 256;
    hipLaunchKernelGGL(tile_depth_sort_big, dim3(bgrid), dim3(1024), 0, s, ranges, depth_key, gid, ovf2, ovf2_count,
                       done, scratch_hi, scratch_lo);
    return (int)hipGetLastError();
}

int launch_finalize(const uint32_t* sorted_tile, long long cap, const uint32_t* K_dev, uint2* ranges, hipStream_t s) {
    if (cap <= 0) return 0;
    hipLaunchKernelGGL(finalize_kernel, dim3(div_up(div_up(cap, kFinQ), 256)), dim3(256), 0, s, sorted_tile, cap, K_dev,
                       ranges);
    return (int)hipGetLastError();
}

}  // namespace gsr

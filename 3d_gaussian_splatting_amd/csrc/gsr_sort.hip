// gsr_sort.hip -- binning on gfx950: scan, duplicateWithKeys, LSD radix sort, tile ranges,
// per-tile depth order.
//
// Canonical instance order is (tile, depth bits, gid) (SURVEY §8a notes).  It is reached
// with far fewer sorted bytes than one 45-bit key sort over K instances (shipped binning,
// GSR_BIN_VARIANT 1, gsr_api.cpp):
//   1. inclusive scan of tiles_touched in gid order           -> offsets (K = last)
//   2. duplicate: Gaussian g emits its band-clipped rect row-major at offsets[g-1] (coalesced
//      reads of tiles / rects, wave-cooperative expansion)
//   3. stable LSD over the ceil(log2 tiles)-bit tile key only (2 passes at 1080p), values =
//      the instance's Gaussian id -> grouped by tile, gid order inside a tile
//   4. finalize: tile ranges from key boundaries
//   5. per tile, a stable LDS radix sort of the slice by the 32-bit depth key alone (ties keep
//      gid order) -> (tile, depth, gid)
// (B1 recovers an instance's emission index j from its Gaussian's rect, so no permutation
// array is carried through the sort.)  The older order -- a global depth sort of the P keys
// first, then emission in depth order (variant 0) -- and a count binning (variant 2) are kept
// for A/B.
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

// ---- upsweep: per-block digit histogram, written digit-major hist[d * nb + b] ----
__global__ __launch_bounds__(kB) void radix_upsweep(const uint32_t* __restrict__ keys, long long n,
                                                    int shift, int nbits, int nb,
                                                    uint32_t* __restrict__ hist) {
    __shared__ uint32_t cnt[kWaves][256];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) cnt[k][tid] = 0;
    __syncthreads();
    const uint32_t mask = (1u << nbits) - 1u;
    const long long base = (long long)blockIdx.x * kSortTile + (long long)w * kWaveItems;
    for (int r = 0; r < kI; ++r) {
        const long long idx = base + r * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = valid ? (keys[idx] >> shift) & mask : 0u;
        const uint64_t active = __ballot(valid);
        if (active == 0) break;
        const uint64_t peers = match_digit(d, nbits, active);
        if (valid && (peers & lanemask_lt()) == 0) cnt[w][d] += (uint32_t)__popcll(peers);
    }
    __syncthreads();
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) s += cnt[k][tid];
    hist[(size_t)tid * nb + blockIdx.x] = s;
}

// Same counts with LDS atomics (per-wave sub-histograms): counting needs no stable rank, so
// the 8-ballot peer match of radix_upsweep is not needed here.
__global__ __launch_bounds__(kB) void radix_upsweep_atomic(const uint32_t* __restrict__ keys, long long n,
                                                           int shift, int nbits, int nb,
                                                           uint32_t* __restrict__ hist) {
    __shared__ uint32_t cnt[kWaves][256];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) cnt[k][tid] = 0;
    __syncthreads();
    const uint32_t mask = (1u << nbits) - 1u;
    const long long base = (long long)blockIdx.x * kSortTile + (long long)w * kWaveItems;
#pragma unroll 4
    for (int r = 0; r < kI; ++r) {
        const long long idx = base + r * 64 + lane;
        if (idx < n) atomicAdd(&cnt[w][(keys[idx] >> shift) & mask], 1u);
    }
    __syncthreads();
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) s += cnt[k][tid];
    hist[(size_t)tid * nb + blockIdx.x] = s;
}

// ---- column scan: block d turns hist[d*nb .. +nb) into an exclusive scan; totals[d] ----
__global__ __launch_bounds__(kB) void radix_colscan(uint32_t* __restrict__ hist, int nb,
                                                    uint32_t* __restrict__ totals) {
    __shared__ uint32_t wsum[kWaves];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    uint32_t* col = hist + (size_t)blockIdx.x * nb;
    uint32_t carry = 0;
    for (int base = 0; base < nb; base += kB) {
        const int i = base + tid;
        const uint32_t v = i < nb ? col[i] : 0u;
        // inclusive wave scan
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
        if (i < nb) col[i] = carry + pre + x - v;
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) tot += wsum[k];
        __syncthreads();
        carry += tot;
    }
    if (tid == 0) totals[blockIdx.x] = carry;
}

// ---- downsweep: stable scatter, reordered through LDS so global writes are coalesced ----
template <bool V2>
__global__ __launch_bounds__(kB) void radix_downsweep(const uint32_t* __restrict__ keys_in,
                                                      const uint32_t* __restrict__ vals_in,
                                                      uint32_t* __restrict__ keys_out,
                                                      uint32_t* __restrict__ vals_out, long long n,
                                                      int shift, int nbits, int nb,
                                                      const uint32_t* __restrict__ hist,
                                                      const uint32_t* __restrict__ totals,
                                                      const uint32_t* __restrict__ v2_in,
                                                      uint32_t* __restrict__ v2_out) {
    __shared__ uint32_t wcnt[kWaves][256];
    __shared__ uint32_t gbase[256];   // global position of this block's first item of digit d
    __shared__ uint32_t lbase[256];   // block-local position of the first item of digit d
    __shared__ uint32_t wsum[kWaves];
    __shared__ uint32_t skey[kSortTile];
    __shared__ uint32_t sval[kSortTile];
    __shared__ uint32_t sv2[V2 ? kSortTile : 1];  // second value array (V2)
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
        gbase[tid] = pre + x - v + hist[(size_t)tid * nb + blockIdx.x];
    }
    __syncthreads();
    const long long bbase = (long long)blockIdx.x * kSortTile;
    const long long base = bbase + (long long)w * kWaveItems;
    uint32_t key[kI], val[kI], rank[kI], v2[kI];
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int r = 0; r < kI; ++r) {
        const long long idx = base + r * 64 + lane;
        const bool valid = idx < n;
        key[r] = valid ? keys_in[idx] : 0xFFFFFFFFu;
        val[r] = valid ? (vals_in ? vals_in[idx] : (uint32_t)idx) : 0u;
        v2[r] = (V2 && valid) ? v2_in[idx] : 0u;
    }
#pragma unroll
    for (int r = 0; r < kI; ++r) {
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
    for (int r = 0; r < kI; ++r) {
        const long long idx = base + r * 64 + lane;
        if (idx < n) {
            const uint32_t d = (key[r] >> shift) & mask;
            const uint32_t lp = lbase[d] + wcnt[w][d] + rank[r];
            skey[lp] = key[r];
            sval[lp] = val[r];
            if (V2) sv2[lp] = v2[r];
        }
    }
    __syncthreads();
    const int count = (n - bbase) < kSortTile ? (int)(n - bbase) : kSortTile;
#pragma unroll 4
    for (int i = tid; i < count; i += kB) {
        const uint32_t k = skey[i];
        const uint32_t d = (k >> shift) & mask;
        const uint32_t pos = gbase[d] + (uint32_t)i - lbase[d];
        keys_out[pos] = k;
        vals_out[pos] = sval[i];
        if (V2) v2_out[pos] = sv2[i];
    }
}

// ---- onesweep LSD radix sort: one kernel per 8-bit pass ----
// Global digit histograms for every pass come from one read of the keys (radix_hist_all);
// each pass then needs a single kernel: a block takes the next tile in launch order (atomic
// ticket, so every tile it waits on is already resident), ranks its 4096 keys exactly as
// radix_downsweep does, publishes its per-digit counts, and finds the count of each digit
// in all earlier tiles by decoupled look-back over their published (flag | count) words
// (relaxed agent-scope atomics, the packed word makes flag and count one atomic).  Each pass
// reads and writes the keys/values once -- the reduce-then-scan form reads the keys twice
// and runs three kernels per pass.
constexpr uint32_t kAgg = 1u << 30, kInc = 2u << 30, kCntMask = kAgg - 1u;

__global__ __launch_bounds__(kB) void radix_hist_all(const uint32_t* __restrict__ keys, long long n,
                                                     int nbits, uint32_t* __restrict__ ghist) {
    __shared__ uint32_t h[4][256];
    const int tid = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 4; ++p) h[p][tid] = 0;
    __syncthreads();
    const int npass = (nbits + 7) / 8;
    const long long base = (long long)blockIdx.x * kSortTile;
#pragma unroll 4
    for (int r = 0; r < kI; ++r) {
        const long long idx = base + r * kB + tid;
        if (idx < n) {
            const uint32_t k = keys[idx];
            for (int p = 0; p < npass; ++p) {
                const int bits = (nbits - 8 * p) < 8 ? (nbits - 8 * p) : 8;
                atomicAdd(&h[p][(k >> (8 * p)) & ((1u << bits) - 1u)], 1u);
            }
        }
    }
    __syncthreads();
    for (int p = 0; p < npass; ++p)
        if (h[p][tid]) atomicAdd(&ghist[p * 256 + tid], h[p][tid]);
}

template <int KI, int LB>
__global__ __launch_bounds__(kB) void radix_onesweep(const uint32_t* __restrict__ keys_in,
                                                     const uint32_t* __restrict__ vals_in,
                                                     uint32_t* __restrict__ keys_out,
                                                     uint32_t* __restrict__ vals_out, long long n,
                                                     int shift, int nbits,
                                                     const uint32_t* __restrict__ ghist,
                                                     uint32_t* __restrict__ status,
                                                     uint32_t* __restrict__ ticket) {
    __shared__ uint32_t wcnt[kWaves][256];
    __shared__ uint32_t gbase[256];
    __shared__ uint32_t lbase[256];
    __shared__ uint32_t wsum[kWaves];
    constexpr int TILE = kB * KI, WITEMS = KI * 64;
    __shared__ uint32_t skey[TILE];
    __shared__ uint32_t sval[TILE];
    __shared__ int s_tile;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t mask = (1u << nbits) - 1u;
    if (tid == 0) s_tile = (int)atomicAdd(ticket, 1u);
#pragma unroll
    for (int k = 0; k < kWaves; ++k) wcnt[k][tid] = 0;
    __syncthreads();
    const int tile = s_tile;
    const long long bbase = (long long)tile * TILE;
    const long long base = bbase + (long long)w * WITEMS;
    uint32_t key[KI], val[KI], rank[KI];
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int r = 0; r < KI; ++r) {
        const long long idx = base + r * 64 + lane;
        const bool valid = idx < n;
        key[r] = valid ? keys_in[idx] : 0xFFFFFFFFu;
        val[r] = valid ? (vals_in ? vals_in[idx] : (uint32_t)idx) : 0u;
    }
#pragma unroll
    for (int r = 0; r < KI; ++r) {
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
    uint32_t c = 0;  // this tile's count of digit `tid`
#pragma unroll
    for (int k = 0; k < kWaves; ++k) {
        const uint32_t t = wcnt[k][tid];
        wcnt[k][tid] = c;
        c += t;
    }
    // publish, then look back over earlier tiles for digit `tid`
    uint32_t* my = status + (size_t)tile * 256 + tid;
    uint32_t excl = 0;
    if (tile == 0) {
        __hip_atomic_store(my, kInc | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __hip_atomic_store(my, kAgg | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int t = tile - 1;
        uint32_t spins = 0;
        if (LB == 1) {
            while (t >= 0) {
                const uint32_t v = __hip_atomic_load(status + (size_t)t * 256 + tid, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                if ((v & ~kCntMask) == 0u) {
                    if (++spins > (1u << 26)) break;  // never expected: bounded so a bug cannot hang the GPU
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += v & kCntMask;
                if (v & kInc) break;
                --t;
            }
        } else {
            // windowed look-back: LB predecessors' words per probe, all loads in flight at
            // once; consume them nearest-first up to the first inclusive prefix (done) or the
            // first unpublished word (re-probe from there).  Before tile 0: an inclusive zero.
            while (t >= 0) {
                uint32_t v[LB];
#pragma unroll
                for (int j = 0; j < LB; ++j)
                    v[j] = (t - j >= 0) ? __hip_atomic_load(status + (size_t)(t - j) * 256 + tid, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT)
                                        : kInc;
                int used = 0;
                bool done = false;
                for (; used < LB; ++used) {
                    const uint32_t x = v[used];
                    if ((x & ~kCntMask) == 0u) break;
                    excl += x & kCntMask;
                    if (x & kInc) {
                        done = true;
                        break;
                    }
                }
                if (done) break;
                if (used == 0) {
                    if (++spins > (1u << 26)) break;  // never expected: bounded so a bug cannot hang the GPU
                    __builtin_amdgcn_s_sleep(1);
                }
                t -= used;
            }
        }
        __hip_atomic_store(my, kInc | (excl + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    {
        // global digit base = exclusive scan of the pass histogram + earlier tiles' count
        const uint32_t v = ghist[tid];
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
        gbase[tid] = pre + x - v + excl;
        __syncthreads();  // wsum reuse
        // block-local digit starts
        uint32_t y = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t z = __shfl_up(y, o, 64);
            if (lane >= o) y += z;
        }
        if (lane == 63) wsum[w] = y;
        __syncthreads();
        uint32_t pre2 = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) pre2 += (k < w) ? wsum[k] : 0u;
        lbase[tid] = pre2 + y - c;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < KI; ++r) {
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

// ---- scan (gathered input): reduce / partial scan / downsweep ----
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

__global__ __launch_bounds__(kB) void scan_reduce(const uint32_t* __restrict__ in,
                                                  const uint32_t* __restrict__ idx, int n,
                                                  uint32_t* __restrict__ partials) {
    __shared__ uint32_t wsum[kWaves];
    const int base = blockIdx.x * kSortTile;
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < kI; ++r) {
        const int i = base + r * kB + threadIdx.x;
        if (i < n) s += in[idx ? idx[i] : i];
    }
    uint32_t tot;
    block_exclusive_scan(s, wsum, &tot);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void scan_partials(uint32_t* __restrict__ partials, int nb) {
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
}

__global__ __launch_bounds__(kB) void scan_downsweep(const uint32_t* __restrict__ in,
                                                     const uint32_t* __restrict__ idx, int n,
                                                     const uint32_t* __restrict__ partials,
                                                     uint32_t* __restrict__ out,
                                                     uint32_t* __restrict__ iota_out) {
    __shared__ uint32_t buf[kSortTile + kSortTile / 32];
    __shared__ uint32_t wsum[kWaves];
    const int base = blockIdx.x * kSortTile;
    const int tid = threadIdx.x;
    auto pad = [](int i) { return i + (i >> 5); };
#pragma unroll
    for (int r = 0; r < kI; ++r) {
        const int i = r * kB + tid;
        const int g = base + i;
        buf[pad(i)] = g < n ? in[idx ? idx[g] : g] : 0u;
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
        if (base + i < n) {
            out[base + i] = buf[pad(i)];
            if (iota_out) iota_out[base + i] = (uint32_t)(base + i);
        }
    }
}

// ---- F3 duplicate: wave-cooperative expansion (one wave = 64 consecutive ranks, whose
// instances are contiguous; lanes write consecutive instances -> coalesced stores) ----
__device__ __forceinline__ uint32_t udiv_small(uint32_t a, uint32_t b) {
    // a / b for a < 2^20, 1 <= b < 2^12: the float quotient of (a + 0.5) is at least 0.5 / b
    // away from an integer and rcp is accurate to ~1 ulp, so truncation is exact
    return (uint32_t)(((float)a + 0.5f) * __builtin_amdgcn_rcpf((float)b));
}

// ---- fused F2 + F3: scan of tiles_touched in rank order + duplicate, one kernel ----
// Block b (in launch order, atomic ticket) owns ranks [256 b, 256 b + 256): it scans their
// tiles_touched, finds the instances of all earlier blocks by a wave-parallel decoupled
// look-back (64 predecessors per probe; relaxed agent-scope atomics on packed flag|count
// words), writes offsets / inst_start, and emits its own instances exactly as
// duplicate_kernel does.  Replaces three scan kernels + a second pass over the ranks.

__global__ __launch_bounds__(256) void scan_duplicate_kernel(const uint32_t* __restrict__ gid_by_rank,
                                                             const uint32_t* __restrict__ tiles,
                                                             uint4* __restrict__ rect, int n,
                                                             int grid_x, int ty0,
                                                             uint32_t* __restrict__ offsets,
                                                             uint32_t* __restrict__ tkey,
                                                             uint32_t* __restrict__ inst_gid,
                                                             uint32_t* __restrict__ status,
                                                             uint32_t* __restrict__ ticket,
                                                             uint32_t* __restrict__ tcount,
                                                             const uint32_t* __restrict__ depth_key,
                                                             uint32_t* __restrict__ inst_depth) {
    __shared__ uint32_t s_start[kWaves][64], s_g[kWaves][64], s_w[kWaves][64], s_x0[kWaves][64],
        s_y0[kWaves][64], s_dk[kWaves][64];
    __shared__ uint32_t wsum[kWaves];
    __shared__ uint32_t s_excl;
    __shared__ int s_b;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    if (tid == 0) s_b = (int)atomicAdd(ticket, 1u);
    __syncthreads();
    const int b = s_b;
    const int r = b * 256 + tid;
    const bool valid = r < n;
    uint32_t g = 0, nt = 0, minx = 0, maxx = 0, y0 = 0;
    if (valid) {
        g = gid_by_rank[r];
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
        offsets[r] = excl + lex + nt;
        if (nt) rect[g].z = excl + lex;  // inst_start
    }
    // emission: this wave's instances [excl + pre_w, + wsum[w]) with pre_w = first lane's lex
    const uint32_t wbase = pre;  // = lex of lane 0 of this wave
    const uint32_t wtotal = wsum[w];
    s_start[w][lane] = (valid && nt) ? lex - wbase : 0xFFFFFFFFu;
    s_g[w][lane] = g;
    s_w[w][lane] = maxx - minx;
    s_x0[w][lane] = minx;
    s_y0[w][lane] = y0;
    s_dk[w][lane] = (inst_depth && nt) ? depth_key[g] : 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t first = excl + wbase;
    for (uint32_t i = lane; i < wtotal; i += 64) {
        int o = 0;  // owner = last lane whose start <= i (lanes without instances never own one)
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
            if (s_start[w][o + step] <= i) o += step;
        const uint32_t local = i - s_start[w][o];
        const uint32_t wd = s_w[w][o];
        const uint32_t dy = udiv_small(local, wd), dx = local - dy * wd;
        const uint32_t tk = (s_y0[w][o] + dy) * (uint32_t)grid_x + s_x0[w][o] + dx;
        tkey[first + i] = tk;
        inst_gid[first + i] = s_g[w][o];
        if (tcount) atomicAdd(tcount + tk, 1u);  // count binning: no-return atomic
        if (inst_depth) inst_depth[first + i] = s_dk[w][o];  // per-tile depth sort keys
    }
}

// ---- band candidates: order-preserving compaction of the Gaussians with tiles in the band ----
// A block owns kSortTile consecutive gids; wave w handles the contiguous 1024-gid run
// [w*1024, (w+1)*1024) of it in 16 rounds of 64 lanes, so ballot prefix counts keep gid order.
__global__ __launch_bounds__(kB) void compact_count(const uint32_t* __restrict__ tiles, int n,
                                                   uint32_t* __restrict__ partials) {
    __shared__ uint32_t wsum[kWaves];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int base = blockIdx.x * kSortTile + w * kWaveItems;
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < kI; ++r) {
        const int g = base + r * 64 + lane;
        c += __popcll(__ballot(g < n && tiles[g] != 0u));
    }
    if (lane == 0) wsum[w] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < kWaves; ++k) t += wsum[k];
        partials[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kB) void compact_scatter(const uint32_t* __restrict__ tiles,
                                                     const uint32_t* __restrict__ depth_key, int n,
                                                     const uint32_t* __restrict__ partials,
                                                     uint32_t* __restrict__ keys_out,
                                                     uint32_t* __restrict__ gids_out,
                                                     uint32_t* __restrict__ count_out) {
    __shared__ uint32_t wsum[kWaves];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int base = blockIdx.x * kSortTile + w * kWaveItems;
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < kI; ++r) {
        const int g = base + r * 64 + lane;
        c += __popcll(__ballot(g < n && tiles[g] != 0u));
    }
    if (lane == 0) wsum[w] = c;
    __syncthreads();
    uint32_t pos = partials[blockIdx.x];
    for (int k = 0; k < w; ++k) pos += wsum[k];
#pragma unroll
    for (int r = 0; r < kI; ++r) {
        const int g = base + r * 64 + lane;
        const bool keep = g < n && tiles[g] != 0u;
        const uint64_t m = __ballot(keep);
        if (keep) {
            const uint32_t at = pos + (uint32_t)__popcll(m & lanemask_lt());
            keys_out[at] = depth_key[g];
            gids_out[at] = (uint32_t)g;
        }
        pos += (uint32_t)__popcll(m);
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kB - 1) *count_out = pos;
}

__global__ __launch_bounds__(256) void duplicate_kernel(const uint32_t* __restrict__ gid_by_rank,
                                                        const uint32_t* __restrict__ offsets,
                                                        const uint32_t* __restrict__ tiles,
                                                        uint4* __restrict__ rect, int P,
                                                        int grid_x, int ty0, int ty1,
                                                        uint32_t* __restrict__ tkey,
                                                        uint32_t* __restrict__ inst_gid,
                                                        uint32_t* __restrict__ tcount,
                                                        const uint32_t* __restrict__ depth_key,
                                                        uint32_t* __restrict__ inst_depth) {
    __shared__ uint32_t s_start[kWaves][64], s_g[kWaves][64], s_w[kWaves][64], s_x0[kWaves][64],
        s_y0[kWaves][64], s_dk[kWaves][64];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int r = blockIdx.x * 256 + tid;
    const bool valid = r < P;
    uint32_t g = 0, nt = 0, end = 0;
    if (valid) {
        g = gid_by_rank[r];
        nt = tiles[g];
        end = offsets[r];
    }
    uint32_t minx = 0, maxx = 0, y0 = 0;
    if (nt) {
        rect[g].z = end - nt;  // inst_start
        const uint4 rr = rect[g];
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
    s_dk[w][lane] = (inst_depth && nt) ? depth_key[g] : 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t i = lane; i < total; i += 64) {
        // owner = last lane whose start <= i (lanes with no instances never own one)
        int o = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)
            if (s_start[w][o + step] <= i) o += step;
        const uint32_t local = i - s_start[w][o];
        const uint32_t wd = s_w[w][o];
        const uint32_t dy = udiv_small(local, wd), dx = local - dy * wd;
        const uint32_t tk = (s_y0[w][o] + dy) * (uint32_t)grid_x + s_x0[w][o] + dx;
        tkey[first + i] = tk;
        inst_gid[first + i] = s_g[w][o];
        if (tcount) atomicAdd(tcount + tk, 1u);  // count binning: no-return atomic
        if (inst_depth) inst_depth[first + i] = s_dk[w][o];  // per-tile depth sort keys
    }
    (void)ty1;
}

// ---- F5 finalize: tile ranges from the sorted keys ----
__global__ __launch_bounds__(256) void finalize_kernel(const uint32_t* __restrict__ stile, long long K,
                                                       uint2* __restrict__ ranges) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= K) return;
    const uint32_t t = stile[i];
    if (i == 0 || stile[i - 1] != t) ranges[t].x = (uint32_t)i;
    if (i == K - 1 || stile[i + 1] != t) ranges[t].y = (uint32_t)(i + 1);
}


// ---- count binning (GSR_BIN_VARIANT 2, shipped): the instance list grouped by tile without a
// key sort.  F3 adds every instance into its tile's counter (no-return atomics); one block
// scans the counts into the tile ranges and turns each count into a cursor; the scatter claims
// a slot per instance with a returning atomic on its tile's cursor.  Order inside a tile is
// arbitrary here -- the per-tile (depth, gid) sort below makes it canonical -- so no stability
// is needed, and the K (tile, gid) pairs are read and written once instead of two LSD passes
// (each a read, a histogram pass and a write) plus the finalize pass.
__global__ __launch_bounds__(1024) void tile_offsets_kernel(uint32_t* __restrict__ tcount, int t0, int nt,
                                                            uint2* __restrict__ ranges) {
    __shared__ uint32_t wsum[16];
    uint32_t carry = 0;
    for (int base = 0; base < nt; base += 1024) {
        const int i = base + threadIdx.x;
        const uint32_t v = i < nt ? tcount[t0 + i] : 0u;
        uint32_t tot;
        const uint32_t ex = carry + block_exclusive_scan(v, wsum, &tot);
        if (i < nt) {
            ranges[t0 + i] = make_uint2(ex, ex + v);
            tcount[t0 + i] = ex;  // the tile's scatter cursor
        }
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void tile_scatter_kernel(const uint32_t* __restrict__ tkey,
                                                           const uint32_t* __restrict__ gid, long long K,
                                                           uint32_t* __restrict__ cursor,
                                                           uint32_t* __restrict__ stile,
                                                           uint32_t* __restrict__ sgid) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= K) return;
    const uint32_t t = tkey[i];
    const uint32_t pos = atomicAdd(cursor + t, 1u);
    stile[pos] = t;
    sgid[pos] = gid[i];
}

// ---- per-tile depth order (canonical (tile, depth bits, gid) without a global depth sort) ----
// After the stable tile-bits sort of instances emitted in gid order, each tile's slice holds
// its Gaussians in gid order; sorting the slice by the unique 64-bit key (depth bits << 32 |
// gid) gives exactly the canonical order.  Bitonic network in the all-ascending ("flip")
// form, so padding keys (all ones) stay at the top and a virtually padded global slice needs
// no storage beyond its n entries.  Integer work: LDS-latency-bound, no MFMA.
// key of slice entry i: the depth key carried through the tile sort (sdepth, contiguous) or,
// without it, gathered per instance from the Gaussian's depth key (random 4-B reads)
__device__ __forceinline__ uint64_t depth_gid_key(const uint32_t* __restrict__ depth_key,
                                                  const uint32_t* __restrict__ sdepth, uint32_t pos, uint32_t g) {
    return ((uint64_t)(sdepth ? sdepth[pos] : depth_key[g]) << 32) | g;
}

template <int NT>
__device__ __forceinline__ void bitonic_lds(uint64_t* k, int m) {
    for (int size = 2; size <= m; size <<= 1) {
        const int half = size >> 1;
        for (int t = threadIdx.x; t < (m >> 1); t += NT) {
            const int i = ((t & ~(half - 1)) << 1) | (t & (half - 1));
            const int j = i ^ (size - 1);  // mirror partner within the size block
            const uint64_t a = k[i], b = k[j];
            if (a > b) {
                k[i] = b;
                k[j] = a;
            }
        }
        __syncthreads();
        for (int d = half >> 1; d >= 1; d >>= 1) {
            for (int t = threadIdx.x; t < (m >> 1); t += NT) {
                const int i = ((t & ~(d - 1)) << 1) | (t & (d - 1));
                const int j = i + d;
                const uint64_t a = k[i], b = k[j];
                if (a > b) {
                    k[i] = b;
                    k[j] = a;
                }
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ int pow2_at_least(int n) {
    int m = 1;
    while (m < n) m <<= 1;
    return m;
}

// Small form: one block of NT threads per tile, slices of up to CAP instances in LDS; longer
// slices are queued for tile_depth_sort_large.  The host picks CAP from the mean instances per
// tile (launch_tile_depth_sort), so the queue stays empty on ordinary scenes.
template <int CAP, int NT>
__global__ __launch_bounds__(NT) void tile_depth_sort_small(const uint2* __restrict__ ranges, int tile0,
                                                            const uint32_t* __restrict__ depth_key,
                                                            const uint32_t* __restrict__ sdepth,
                                                            uint32_t* __restrict__ gid, uint32_t* __restrict__ ovf,
                                                            uint32_t* __restrict__ ovf_count) {
    __shared__ uint64_t k[CAP];
    const int tile = tile0 + blockIdx.x;
    const uint2 r = ranges[tile];
    const int n = (int)(r.y - r.x);
    if (n <= 1) return;
    if (n > CAP) {
        if (threadIdx.x == 0) ovf[atomicAdd(ovf_count, 1u)] = (uint32_t)tile;
        return;
    }
    const int m = pow2_at_least(n);
    for (int i = threadIdx.x; i < m; i += NT)
        k[i] = i < n ? depth_gid_key(depth_key, sdepth, r.x + i, gid[r.x + i]) : ~0ull;
    __syncthreads();
    bitonic_lds<NT>(k, m);
    for (int i = threadIdx.x; i < n; i += NT) gid[r.x + i] = (uint32_t)k[i];
}

// Radix form (shipped for stable input): when the tile's slice is already in gid order (the
// stable tile-key sort of gid-order emissions, GSR_BIN_VARIANT 1), a stable LSD sort of the
// 32-bit depth keys alone gives (depth, gid) order.  Four 8-bit passes in LDS, each ranked
// exactly as radix_downsweep ranks (wave64 ballot peer match, per-wave digit counters, a
// digit-major block scan): ~20 B of LDS traffic per key per pass, against ~log2(n)^2 / 2 x 12 B
// for the bitonic network, which is LDS-bandwidth-bound.  Passes whose digit is equal for every
// key of the slice are skipped, so 9-bit digits need 3 passes for the <= 27 differing bits of
// a 0.2 .. 100 depth range.  Measured at 1M/1080p: 9-bit radix 0.098 ms, 8-bit 0.102 ms,
// bitonic 0.130 ms; the radix form is latency-bound per block (dependent LDS counter updates
// per 64-key round, ~6 syncs per pass), not by LDS bandwidth.
// NT threads, I items per thread: CAP = NT * I keys; wave w owns the contiguous run
// [w * 64 I, (w + 1) * 64 I) of the slice, ranked round by round in index order (stable).
// One slice [rg.x, rg.y) of n <= NT * I entries, sorted by the whole block.  Ends with every
// LDS access behind a barrier, so a block may call it again for another slice.
template <int NT, int I, int DB>
__device__ __forceinline__ void radix_sort_slice(const uint2 rg, const uint32_t* __restrict__ depth_key,
                                                 const uint32_t* __restrict__ sdepth, uint32_t* __restrict__ gid) {
    constexpr int NWV = NT / 64, CAP = NT * I, BINS = 1 << DB;
    constexpr uint32_t DMASK = BINS - 1u;
    __shared__ uint32_t wcnt[NWV][BINS];
    __shared__ uint32_t lbase[BINS];
    __shared__ uint32_t red[2][NWV];
    __shared__ uint32_t skey[CAP];
    __shared__ uint32_t sval[CAP];
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
        key[r] = valid ? (sdepth ? sdepth[rg.x + idx] : depth_key[val[r]]) : 0xFFFFFFFFu;
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
                                                      const uint32_t* __restrict__ sdepth,
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
    radix_sort_slice<NT, I, DB>(rg, depth_key, sdepth, gid);
}

// The queued (longer) slices: blocks walk the queue; slices longer than NT * I go on to the
// second queue (ovf2), which the global-memory form drains.  The queue length is on the device,
// so blocks past it exit at once.
template <int NT, int I, int DB>
__global__ __launch_bounds__(NT) void tile_depth_radix_queue(const uint2* __restrict__ ranges,
                                                            const uint32_t* __restrict__ depth_key,
                                                            const uint32_t* __restrict__ sdepth,
                                                            uint32_t* __restrict__ gid,
                                                            const uint32_t* __restrict__ ovf,
                                                            const uint32_t* __restrict__ ovf_count,
                                                            uint32_t* __restrict__ ovf2, uint32_t* __restrict__ ovf2_count) {
    const uint32_t cnt = *ovf_count;
    for (uint32_t q = blockIdx.x; q < cnt; q += gridDim.x) {
        const uint32_t tile = ovf[q];
        const uint2 rg = ranges[tile];
        if ((int)(rg.y - rg.x) > NT * I) {
            if (threadIdx.x == 0) ovf2[atomicAdd(ovf2_count, 1u)] = tile;
            continue;  // block-uniform
        }
        radix_sort_slice<NT, I, DB>(rg, depth_key, sdepth, gid);
    }
}


// Large form: the queued tiles, 1024 threads per block.  Up to kLargeLds instances in LDS;
// beyond that (dense real scenes) the same network runs on the slice in global memory, with
// the key split into two u32 arrays (the tile sort's free ping-pong pair), virtually padded.
constexpr int kLargeLds = 8192;
__global__ __launch_bounds__(1024) void tile_depth_sort_large(const uint2* __restrict__ ranges,
                                                              const uint32_t* __restrict__ depth_key,
                                                              const uint32_t* __restrict__ sdepth,
                                                              uint32_t* __restrict__ gid,
                                                              const uint32_t* __restrict__ ovf,
                                                              const uint32_t* __restrict__ ovf_count,
                                                              uint32_t* __restrict__ hi, uint32_t* __restrict__ lo) {
    extern __shared__ uint64_t kl[];
    const uint32_t cnt = *ovf_count;
    for (uint32_t q = blockIdx.x; q < cnt; q += gridDim.x) {
        const uint2 r = ranges[ovf[q]];
        const int n = (int)(r.y - r.x);
        const int m = pow2_at_least(n);
        if (m <= kLargeLds) {
            for (int i = threadIdx.x; i < m; i += 1024)
                kl[i] = i < n ? depth_gid_key(depth_key, sdepth, r.x + i, gid[r.x + i]) : ~0ull;
            __syncthreads();
            bitonic_lds<1024>(kl, m);
            for (int i = threadIdx.x; i < n; i += 1024) gid[r.x + i] = (uint32_t)kl[i];
            __syncthreads();
            continue;
        }
        uint32_t* H = hi + r.x;
        uint32_t* L = lo + r.x;
        for (int i = threadIdx.x; i < n; i += 1024) {
            const uint32_t g = gid[r.x + i];
            H[i] = sdepth ? sdepth[r.x + i] : depth_key[g];
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
        for (int size = 2; size <= m; size <<= 1) {
            const int half = size >> 1;
            for (int t = threadIdx.x; t < (m >> 1); t += 1024) {
                const int i = ((t & ~(half - 1)) << 1) | (t & (half - 1));
                cex(i, i ^ (size - 1));
            }
            __threadfence_block();
            __syncthreads();
            for (int d = half >> 1; d >= 1; d >>= 1) {
                for (int t = threadIdx.x; t < (m >> 1); t += 1024) {
                    const int i = ((t & ~(d - 1)) << 1) | (t & (d - 1));
                    cex(i, i + d);
                }
                __threadfence_block();
                __syncthreads();
            }
        }
        for (int i = threadIdx.x; i < n; i += 1024) gid[r.x + i] = L[i];
        __syncthreads();
    }
}
}  // namespace

// A/B selector (bench/ablation only; read per call like the blend variants):
// 0 = reduce-then-scan everywhere, 1 = onesweep everywhere, 2 (shipped) = onesweep for the
// depth sort (P keys: latency-bound, one kernel per pass wins) and reduce-then-scan for the
// tile sort (K keys: the look-back chain over ~1600 tiles costs more than the extra read).
static bool use_onesweep(bool depth_sort) {
    const char* e = std::getenv("GSR_SORT_VARIANT");
    const int v = e ? std::atoi(e) : 2;
    return v == 1 || (v == 2 && depth_sort);
}

// onesweep: ghist (4 x 256) | tickets (16) | status (passes x nb x 256); one memset per sort
// reduce-then-scan upsweep: LDS-atomic counts (1, shipped) or ballot peer match (0)
static bool upsweep_atomic() {
    const char* e = std::getenv("GSR_UPSWEEP_VARIANT");
    return e ? std::atoi(e) != 0 : true;
}

// Items per thread of the onesweep tiles: 16 (4096-key tiles) or 4 (1024-key tiles, 4x the
// blocks -- for the small candidate sets of multi-GPU bands, where a pass is latency-bound).
static int onesweep_items(long long n) {
    const char* e = std::getenv("GSR_ONESWEEP_ITEMS");
    if (e) {
        const int v = std::atoi(e);
        return v == 4 || v == 8 ? v : 16;
    }
    return n <= kOnesweepSmall ? 4 : 16;
}

// Look-back window of the onesweep passes: 8 predecessor words per probe (shipped) or 1.
static int lookback_window() {
    const char* e = std::getenv("GSR_LOOKBACK");
    const int v = e ? std::atoi(e) : 8;
    return v == 1 || v == 32 ? v : 8;
}

static int radix_sort_onesweep(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* k0, uint32_t* v0,
                               uint32_t* k1, uint32_t* v1, long long n, int nbits, uint32_t* hist, int* which,
                               hipStream_t s) {
    const int items = onesweep_items(n);
    const int lb = lookback_window();
    const int nb = div_up(n, (long long)kB * items);  // look-back tiles
    const int nbh = sort_blocks(n);                  // histogram blocks
    const int npass = (nbits + 7) / 8;
    uint32_t* ghist = hist;
    uint32_t* tickets = hist + 4 * 256;
    uint32_t* status = tickets + 16;
    const size_t words = 4 * 256 + 16 + (size_t)npass * nb * 256;
    if (hipError_t e = hipMemsetAsync(hist, 0, words * sizeof(uint32_t), s)) return (int)e;
    hipLaunchKernelGGL(radix_hist_all, dim3(nbh), dim3(kB), 0, s, keys_in, n, nbits, ghist);
    const uint32_t* kin = keys_in;
    const uint32_t* vin = vals_in;
    int dst = 0;
    for (int p = 0; p < npass; ++p) {
        const int shift = 8 * p;
        const int bits = (nbits - shift) < 8 ? (nbits - shift) : 8;
        uint32_t* ko = dst == 0 ? k0 : k1;
        uint32_t* vo = dst == 0 ? v0 : v1;
        uint32_t* st = status + (size_t)p * nb * 256;
#define GSR_ONESWEEP(KI_, LB_)                                                                          \
    hipLaunchKernelGGL((radix_onesweep<KI_, LB_>), dim3(nb), dim3(kB), 0, s, kin, vin, ko, vo, n, shift, bits, \
                       ghist + 256 * p, st, tickets + p)
        if (items == 4) {
            if (lb == 1) GSR_ONESWEEP(4, 1); else if (lb == 32) GSR_ONESWEEP(4, 32); else GSR_ONESWEEP(4, 8);
        } else if (items == 8) {
            if (lb == 1) GSR_ONESWEEP(8, 1); else if (lb == 32) GSR_ONESWEEP(8, 32); else GSR_ONESWEEP(8, 8);
        } else {
            if (lb == 1) GSR_ONESWEEP(16, 1); else if (lb == 32) GSR_ONESWEEP(16, 32); else GSR_ONESWEEP(16, 8);
        }
#undef GSR_ONESWEEP
        kin = ko;
        vin = vo;
        *which = dst;
        dst ^= 1;
    }
    return (int)hipGetLastError();
}

int radix_sort(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* k0, uint32_t* v0,
               uint32_t* k1, uint32_t* v1, long long n, int nbits, uint32_t* hist, int* which,
               hipStream_t s, bool depth_sort, const uint32_t* v2_in, uint32_t* v2_0, uint32_t* v2_1) {
    *which = -1;
    if (n <= 0) return 0;
    if (use_onesweep(depth_sort) && !v2_in)
        return radix_sort_onesweep(keys_in, vals_in, k0, v0, k1, v1, n, nbits, hist, which, s);
    const int nb = sort_blocks(n);
    uint32_t* totals = hist + (size_t)256 * (nb + 1);
    const uint32_t* kin = keys_in;
    const uint32_t* vin = vals_in;
    const uint32_t* v2in = v2_in;
    int dst = 0;
    for (int shift = 0; shift < nbits; shift += 8) {
        const int bits = (nbits - shift) < 8 ? (nbits - shift) : 8;
        uint32_t* ko = dst == 0 ? k0 : k1;
        uint32_t* vo = dst == 0 ? v0 : v1;
        uint32_t* v2o = dst == 0 ? v2_0 : v2_1;
        if (upsweep_atomic())
            hipLaunchKernelGGL(radix_upsweep_atomic, dim3(nb), dim3(kB), 0, s, kin, n, shift, bits, nb, hist);
        else
            hipLaunchKernelGGL(radix_upsweep, dim3(nb), dim3(kB), 0, s, kin, n, shift, bits, nb, hist);
        hipLaunchKernelGGL(radix_colscan, dim3(256), dim3(kB), 0, s, hist, nb, totals);
        if (v2in)
            hipLaunchKernelGGL(radix_downsweep<true>, dim3(nb), dim3(kB), 0, s, kin, vin, ko, vo, n, shift, bits, nb,
                               hist, totals, v2in, v2o);
        else
            hipLaunchKernelGGL(radix_downsweep<false>, dim3(nb), dim3(kB), 0, s, kin, vin, ko, vo, n, shift, bits, nb,
                               hist, totals, nullptr, nullptr);
        kin = ko;
        vin = vo;
        v2in = v2in ? v2o : nullptr;
        *which = dst;
        dst ^= 1;
    }
    return (int)hipGetLastError();
}

int inclusive_scan_gather(const uint32_t* in, const uint32_t* idx, uint32_t* out, int n,
                          uint32_t* partials, hipStream_t s, uint32_t* iota_out) {
    if (n <= 0) return 0;
    const int nb = sort_blocks(n);
    hipLaunchKernelGGL(scan_reduce, dim3(nb), dim3(kB), 0, s, in, idx, n, partials);
    hipLaunchKernelGGL(scan_partials, dim3(1), dim3(1024), 0, s, partials, nb);
    hipLaunchKernelGGL(scan_downsweep, dim3(nb), dim3(kB), 0, s, in, idx, n, partials, out, iota_out);
    return (int)hipGetLastError();
}

int compact_candidates(const uint32_t* tiles, const uint32_t* depth_key, int n, uint32_t* partials,
                       uint32_t* keys_out, uint32_t* gids_out, uint32_t* count_out, hipStream_t s) {
    if (n <= 0) return 0;
    const int nb = sort_blocks(n);
    hipLaunchKernelGGL(compact_count, dim3(nb), dim3(kB), 0, s, tiles, n, partials);
    hipLaunchKernelGGL(scan_partials, dim3(1), dim3(1024), 0, s, partials, nb);
    hipLaunchKernelGGL(compact_scatter, dim3(nb), dim3(kB), 0, s, tiles, depth_key, n, partials, keys_out,
                       gids_out, count_out);
    return (int)hipGetLastError();
}

int launch_duplicate(const uint32_t* gid_by_rank, const uint32_t* offsets, const uint32_t* tiles,
                     uint4* rect, int P, int grid_x, int ty0, int ty1, uint32_t* tkey, uint32_t* inst_gid,
                     hipStream_t s, uint32_t* tcount, const uint32_t* depth_key, uint32_t* inst_depth) {
    if (P <= 0) return 0;
    hipLaunchKernelGGL(duplicate_kernel, dim3(div_up(P, 256)), dim3(256), 0, s, gid_by_rank, offsets,
                       tiles, rect, P, grid_x, ty0, ty1, tkey, inst_gid, tcount, depth_key, inst_depth);
    return (int)hipGetLastError();
}

int launch_scan_duplicate(const uint32_t* gid_by_rank, const uint32_t* tiles, uint4* rect, int n,
                          int grid_x, int ty0, uint32_t* offsets, uint32_t* tkey, uint32_t* inst_gid,
                          uint32_t* scratch, hipStream_t s, uint32_t* tcount, const uint32_t* depth_key,
                          uint32_t* inst_depth) {
    if (n <= 0) return 0;
    const int nb = div_up(n, 256);
    uint32_t* ticket = scratch;
    uint32_t* status = scratch + 16;
    if (hipError_t e = hipMemsetAsync(scratch, 0, sizeof(uint32_t) * (16 + (size_t)nb), s)) return (int)e;
    hipLaunchKernelGGL(scan_duplicate_kernel, dim3(nb), dim3(256), 0, s, gid_by_rank, tiles, rect, n, grid_x, ty0,
                       offsets, tkey, inst_gid, status, ticket, tcount, depth_key, inst_depth);
    return (int)hipGetLastError();
}

// Per-tile sort form (A/B, bench/ablation only): 1 (shipped) = LDS radix when the slices are
// in gid order, 0 = bitonic network (always used for unordered slices).
static int tile_sort_variant() {
    const char* e = std::getenv("GSR_TILESORT_VARIANT");
    return e ? std::atoi(e) : 1;
}

// Digit width of the per-tile radix form (A/B): 9 (shipped) sorts the <= 27 bits in which a
// tile's depth keys differ (depths 0.2 .. 100 differ in the low 27 bits; constant high digits
// are skipped) in 3 passes, 8 needs 4.
static int tile_sort_digit_bits() {
    const char* e = std::getenv("GSR_TILESORT_BITS");
    return e && std::atoi(e) == 8 ? 8 : 9;
}

int launch_tile_depth_sort(const uint2* ranges, int tile0, int ntiles, long long K, const uint32_t* depth_key,
                           uint32_t* gid, uint32_t* ovf, uint32_t* ovf_count, uint32_t* ovf2, uint32_t* ovf2_count,
                           uint32_t* scratch_hi, uint32_t* scratch_lo, hipStream_t s, bool gid_ordered,
                           const uint32_t* sdepth) {
    if (ntiles <= 0 || K <= 0) return 0;
    // capacity of the LDS form: a power of two >= 1.5x the mean slice, 1024 .. 8192
    const long long mean = K / ntiles;
    int cap = 1024;
    while (cap < 8192 && cap < mean + mean / 2) cap <<= 1;
    if (gid_ordered && tile_sort_variant() == 1) {
#define GSR_TILE_RADIX(NT_, I_, DB_)                                                                          \
    hipLaunchKernelGGL((tile_depth_radix<NT_, I_, DB_>), dim3(ntiles), dim3(NT_), 0, s, ranges, tile0, depth_key, \
                       sdepth, gid, ovf, ovf_count)
        // one block per tile up to 4096 entries (<= 43 KB of LDS: 3 blocks per CU); longer slices
        // queue for 512-thread blocks of up to 8192 (73 KB: 2 per CU) walking the queue, and
        // beyond that for the global-memory bitonic form
        if (tile_sort_digit_bits() == 8) {
            if (cap == 1024) GSR_TILE_RADIX(256, 4, 8);
            else if (cap == 2048) GSR_TILE_RADIX(256, 8, 8);
            else GSR_TILE_RADIX(256, 16, 8);
        } else {
            if (cap == 1024) GSR_TILE_RADIX(256, 4, 9);
            else if (cap == 2048) GSR_TILE_RADIX(256, 8, 9);
            else GSR_TILE_RADIX(256, 16, 9);
        }
#undef GSR_TILE_RADIX
        const int qgrid = ntiles < 512 ? ntiles : 512;
        hipLaunchKernelGGL((tile_depth_radix_queue<512, 16, 8>), dim3(qgrid), dim3(512), 0, s, ranges, depth_key,
                           sdepth, gid, ovf, ovf_count, ovf2, ovf2_count);
        const int grid = ntiles < 64 ? ntiles : 64;
        hipLaunchKernelGGL(tile_depth_sort_large, dim3(grid), dim3(1024), sizeof(uint64_t) * kLargeLds, s, ranges,
                           depth_key, sdepth, gid, ovf2, ovf2_count, scratch_hi, scratch_lo);
        return (int)hipGetLastError();
    } else if (cap == 1024)
        hipLaunchKernelGGL((tile_depth_sort_small<1024, 256>), dim3(ntiles), dim3(256), 0, s, ranges, tile0, depth_key,
                           sdepth, gid, ovf, ovf_count);
    else if (cap == 2048)
        hipLaunchKernelGGL((tile_depth_sort_small<2048, 256>), dim3(ntiles), dim3(256), 0, s, ranges, tile0, depth_key,
                           sdepth, gid, ovf, ovf_count);
    else if (cap == 4096)
        hipLaunchKernelGGL((tile_depth_sort_small<4096, 512>), dim3(ntiles), dim3(512), 0, s, ranges, tile0, depth_key,
                           sdepth, gid, ovf, ovf_count);
    else
        hipLaunchKernelGGL((tile_depth_sort_small<8192, 1024>), dim3(ntiles), dim3(1024), 0, s, ranges, tile0,
                           depth_key, sdepth, gid, ovf, ovf_count);
    // the rare longer slices: the queue length is on the device; 64 blocks drain it (blocks
    // past the count exit at once)
    const int grid = ntiles < 64 ? ntiles : 64;
    hipLaunchKernelGGL(tile_depth_sort_large, dim3(grid), dim3(1024), sizeof(uint64_t) * kLargeLds, s, ranges,
                       depth_key, sdepth, gid, ovf, ovf_count, scratch_hi, scratch_lo);
    return (int)hipGetLastError();
}

int launch_tile_bins(const uint32_t* tkey, const uint32_t* gid, long long K, int tile0, int ntiles,
                     uint32_t* tcount, uint2* ranges, uint32_t* stile, uint32_t* sgid, hipStream_t s) {
    if (K <= 0 || ntiles <= 0) return 0;
    if (!tcount) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(tile_offsets_kernel, dim3(1), dim3(1024), 0, s, tcount, tile0, ntiles, ranges);
    hipLaunchKernelGGL(tile_scatter_kernel, dim3(div_up(K, 256)), dim3(256), 0, s, tkey, gid, K, tcount, stile, sgid);
    return (int)hipGetLastError();
}

int launch_finalize(const uint32_t* sorted_tile, long long K, uint2* ranges, hipStream_t s) {
    if (K <= 0) return 0;
    hipLaunchKernelGGL(finalize_kernel, dim3(div_up(K, 256)), dim3(256), 0, s, sorted_tile, K, ranges);
    return (int)hipGetLastError();
}

}  // namespace gsr

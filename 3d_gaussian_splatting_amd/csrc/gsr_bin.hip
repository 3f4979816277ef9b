// gsr_bin.hip -- F3 + F4 + F5 as one counting sort by tile (images of up to kBinMaxTiles tiles).
//
// The instances are grouped by tile in gid order (the order the LSD tile-key sort of the
// duplicated keys gives, gsr_sort.hip), without materialising and re-sorting the (tile, gid)
// keys.  The Gaussians are cut into nseg contiguous segments of S (a multiple of 64):
//   1. bin_count   one block per segment expands its Gaussians' band-clipped rects into
//                  instances (gid order, rect row-major = emission order) and counts them per
//                  tile in LDS; the row of T counts goes to mat[seg][0..T) (coalesced).  It
//                  also writes each Gaussian's emission base inst_start (rect.z).
//   2. bin_colscan per tile, the exclusive prefix of the counts over the segments (in place) and
//                  the tile's total.
//   3. bin_ranges  exclusive scan of the tile totals -> the tile starts and ranges[].
//   4. bin_scatter one wave per segment, counters in LDS = tile start + the segment's prefix;
//                  it expands its instances again in emission order, 64 per round, ranks the
//                  lanes of a round that hit one tile by a ballot peer match (stable: lower lane =
//                  lower gid), and stores each instance's gid at its final position.
// So every instance is written once (4 B of gid, plus 4 B of tile id for the introspection view)
// and no key array is read back, where F3 + two LSD passes + finalize move ~60 B per instance
// (DESIGN §5).  The result equals the stable tile sort of the emitted keys bit for bit; the
// instances past the binning capacity (emission index >= cap) are dropped exactly as F3 drops
// them.
//
// Expansion (per wave, 64 Gaussians per chunk): the inclusive scan `offsets` gives each
// Gaussian's emission base; per round of 64 instances each Gaussian that starts inside the
// round marks its start position in a 64-entry LDS row, and a wave prefix-max (DPP row shifts
// and row broadcasts) gives every lane the Gaussian its instance belongs to -- two LDS round
// trips per round instead of a 6-step binary search.
#include "gsr_kernels.h"

namespace gsr {
namespace {

__device__ inline uint64_t lanemask_lt_b() {
    const int lane = threadIdx.x & 63;
    return (lane == 0) ? 0ull : (~0ull >> (64 - lane));
}

__device__ __forceinline__ uint32_t udiv_small_b(uint32_t a, uint32_t b) {
    // a / b for a < 2^20, 1 <= b < 2^12 (see gsr_sort.hip udiv_small)
    return (uint32_t)(((float)a + 0.5f) * __builtin_amdgcn_rcpf((float)b));
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_u(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xF, false);
}

// inclusive prefix maximum over the wave (unsigned; 0 is the identity)
__device__ __forceinline__ uint32_t wave_prefix_max(uint32_t x) {
    x = max(x, dpp_u<0x111, 0xF>(x));  // row_shr:1
    x = max(x, dpp_u<0x112, 0xF>(x));  // row_shr:2
    x = max(x, dpp_u<0x114, 0xF>(x));  // row_shr:4
    x = max(x, dpp_u<0x118, 0xF>(x));  // row_shr:8
    x = max(x, dpp_u<0x142, 0xA>(x));  // row_bcast:15 -> rows 1, 3
    x = max(x, dpp_u<0x143, 0xC>(x));  // row_bcast:31 -> rows 2, 3
    return x;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lanes (among `active`) whose tile equals this lane's (tiles of up to 15 bits)
__device__ __forceinline__ uint64_t match_tile(uint32_t t, int nbits, uint64_t active) {
    uint64_t peers = active;
#pragma unroll
    for (int b = 0; b < 15; ++b) {
        if (b < nbits) {
            const bool bit = (t >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
    }
    return peers;
}

// inclusive prefix sum over the wave
__device__ __forceinline__ uint32_t wave_prefix_sum(uint32_t x) {
    x += dpp_u<0x111, 0xF>(x);
    x += dpp_u<0x112, 0xF>(x);
    x += dpp_u<0x114, 0xF>(x);
    x += dpp_u<0x118, 0xF>(x);
    x += dpp_u<0x142, 0xA>(x);
    x += dpp_u<0x143, 0xC>(x);
    return x;
}

struct ExpandArgs {
    const uint32_t* perm;  // expansion order: perm[r] = gid (depth order), or nullptr = gid order
    const uint4* rect;     // (minx | miny << 16, maxx | maxy << 16, inst_start, band tile count)
    int n, S, gx, ty0, T, nbits;
    long long cap;
};

// One wave expands the Gaussians of ranks [r0, r_end) (<= 64) into their instances, Gaussian by
// Gaussian in rank order and each one's band-clipped rect row-major, 64 per round, and calls
// f(ok, local tile, gid) for every lane of every round (ok: the lane holds an instance whose
// emission index inst_start + local is below the capacity).  sg / sst / mark: this wave's LDS
// rows.
template <class F>
__device__ __forceinline__ void expand_chunk(const ExpandArgs& a, int r0, int r_end, uint4* sg, uint32_t* sst,
                                             uint32_t* mark, F&& f) {
    const int lane = threadIdx.x & 63;
    const int r = r0 + lane;
    const bool valid = r < r_end;
    const uint32_t g = valid ? (a.perm ? a.perm[r] : (uint32_t)r) : 0u;
    const uint4 rr = valid ? a.rect[g] : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t nt = rr.w, minx = rr.x & 0xFFFFu, maxx = rr.y & 0xFFFFu, miny = rr.x >> 16;
    const uint32_t y0l = nt ? (miny > (uint32_t)a.ty0 ? miny : (uint32_t)a.ty0) - (uint32_t)a.ty0 : 0u;
    const uint32_t incl = wave_prefix_sum(nt);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t rel = incl - nt;
    // any instance at or past the capacity in this chunk (wave-uniform): then check per lane
    const bool capped = __ballot(nt != 0u && (long long)rr.z + nt > a.cap) != 0;
    sg[lane] = make_uint4(rel, g, maxx - minx, minx | (y0l << 16));
    sst[lane] = rr.z;
    uint32_t carry = 0;  // owner + 1 of the previous round's last instance
    for (uint32_t i = 0; i < total; i += 64) {
        mark[lane] = 0u;
        wave_sync_lds();
        if (nt && rel >= i && rel < i + 64u) mark[rel - i] = (uint32_t)lane + 1u;
        wave_sync_lds();
        uint32_t m = wave_prefix_max(mark[lane]);
        m = m > carry ? m : carry;
        carry = (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
        const uint32_t ii = i + (uint32_t)lane;
        bool ok = ii < total;
        uint32_t tl = 0, gid = 0;
        if (ok) {
            const uint32_t o = (m - 1u) & 63u;
            const uint4 e = sg[o];
            const uint32_t local = ii - e.x, wd = e.z;
            if (capped) ok = (long long)sst[o] + local < a.cap;
            const uint32_t dy = udiv_small_b(local, wd), dx = local - dy * wd;
            tl = ((e.w >> 16) + dy) * (uint32_t)a.gx + (e.w & 0xFFFFu) + dx;
            gid = e.y;
        }
        f(ok, tl, gid);
        wave_sync_lds();  // mark / sg reads done before they are rewritten
    }
}

template <int TMAX>
__global__ __launch_bounds__(256) void bin_count_kernel(const ExpandArgs a, uint32_t* __restrict__ mat) {
    __shared__ uint32_t cnt[TMAX];
    __shared__ uint4 sg[4][64];
    __shared__ uint32_t sst[4][64], mark[4][64];
    const int tid = threadIdx.x, w = tid >> 6;
    const int seg = blockIdx.x;
    const int rb = seg * a.S;
    const int re = rb + a.S < a.n ? rb + a.S : a.n;
    for (int t = tid; t < a.T; t += 256) cnt[t] = 0u;
    __syncthreads();
    for (int r0 = rb + 64 * w; r0 < re; r0 += 256)
        expand_chunk(a, r0, re, sg[w], sst[w], mark[w], [&](bool ok, uint32_t tl, uint32_t) {
            if (ok) atomicAdd(&cnt[tl], 1u);
        });
    __syncthreads();
    uint32_t* row = mat + (size_t)seg * a.T;
    for (int t = tid; t < a.T; t += 256) row[t] = cnt[t];
}

// 64 tiles per block (one per lane), 16 waves over the segments: in-place exclusive prefix of
// mat[.][t] over the segments, and the tile's total
__global__ __launch_bounds__(1024) void bin_colscan_kernel(uint32_t* __restrict__ mat, int nseg, int T,
                                                           uint32_t* __restrict__ totals) {
    __shared__ uint32_t part[16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int t = blockIdx.x * 64 + lane;
    const int per = (nseg + 15) / 16;
    const int s0 = w * per, s1 = s0 + per < nseg ? s0 + per : nseg;
    uint32_t sum = 0;
    if (t < T) {
#pragma unroll 8
        for (int s = s0; s < s1; ++s) sum += mat[(size_t)s * T + t];
    }
    part[w][lane] = sum;
    __syncthreads();
    uint32_t base = 0, total = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t v = part[k][lane];
        base += k < w ? v : 0u;
        total += v;
    }
    if (t < T) {
#pragma unroll 8
        for (int s = s0; s < s1; ++s) {
            uint32_t* p = mat + (size_t)s * T + t;
            const uint32_t v = *p;
            *p = base;
            base += v;
        }
        if (w == 0) totals[t] = total;
    }
}

// exclusive scan of the T tile totals (one 1024-thread block) -> tile starts and ranges
__global__ __launch_bounds__(1024) void bin_ranges_kernel(const uint32_t* __restrict__ totals, int T,
                                                          uint32_t* __restrict__ tstart, uint2* __restrict__ ranges) {
    __shared__ uint32_t wsum[16];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    uint32_t carry = 0;
    for (int base = 0; base < T; base += 1024) {
        const int i = base + tid;
        const uint32_t v = i < T ? totals[i] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            pre += k < w ? wsum[k] : 0u;
            tot += wsum[k];
        }
        if (i < T) {
            const uint32_t s = carry + pre + x - v;
            tstart[i] = s;
            ranges[i] = make_uint2(s, s + v);
        }
        carry += tot;
        __syncthreads();  // wsum reuse
    }
}

template <int TMAX>
__global__ __launch_bounds__(64) void bin_scatter_kernel(const ExpandArgs a, const uint32_t* __restrict__ mat,
                                                         const uint32_t* __restrict__ tstart,
                                                         uint32_t* __restrict__ out_gid,
                                                         uint32_t* __restrict__ out_tile, uint32_t tile0) {
    __shared__ uint32_t cnt[TMAX];
    __shared__ uint4 sg[64];
    __shared__ uint32_t sst[64], mark[64];
    const int lane = threadIdx.x;
    const int seg = blockIdx.x;
    const int rb = seg * a.S;
    const int re = rb + a.S < a.n ? rb + a.S : a.n;
    const uint32_t* row = mat + (size_t)seg * a.T;
    for (int t = lane; t < a.T; t += 64) cnt[t] = tstart[t] + row[t];
    wave_sync_lds();
    const uint64_t lt = lanemask_lt_b();
    for (int r0 = rb; r0 < re; r0 += 64)
        expand_chunk(a, r0, re, sg, sst, mark, [&](bool ok, uint32_t tl, uint32_t gid) {
            // Every lane takes a slot by an LDS atomic; lanes of one round that hit one tile get
            // distinct slots, but in an order the hardware picks.  A lane sees such a collision
            // when the counter moved past its own increment; then (wave-uniform, rare) the peers
            // are ranked by lane (= emission order) from the counter's final value.
            uint32_t pos = 0;
            bool clash = false;
            if (ok) {
                pos = atomicAdd(&cnt[tl], 1u);
                clash = cnt[tl] != pos + 1u;
            }
            const uint64_t act = __ballot(ok);
            if (__ballot(clash)) {
                const uint64_t peers = match_tile(tl, a.nbits, act);
                if (ok) pos = cnt[tl] - (uint32_t)__popcll(peers) + (uint32_t)__popcll(peers & lt);
            }
            if (ok) {
                out_gid[pos] = gid;
                if (out_tile) out_tile[pos] = tile0 + tl;
            }
        });
}

}  // namespace

int launch_bin(const uint4* rect, const uint32_t* perm, int n, int grid_x, int ty0, int ntiles, long long cap,
               uint32_t* mat_buf, uint32_t* out_gid, uint32_t* out_tile, uint2* ranges, hipStream_t s) {
    if (ntiles <= 0) return 0;
    if (ntiles > kBinMaxTiles) return (int)hipErrorInvalidValue;
    const int T = ntiles;
    const uint32_t tile0 = (uint32_t)ty0 * (uint32_t)grid_x;
    const BinSeg sgm(n, cap, T);
    uint32_t* mat = mat_buf;
    uint32_t* totals = mat_buf + sgm.mat_words;
    uint32_t* tstart = totals + T;
    if (n <= 0 || cap <= 0) {  // every range empty
        return (int)hipMemsetAsync(ranges + tile0, 0, sizeof(uint2) * (size_t)T, s);
    }
    ExpandArgs a{perm, rect, n, sgm.S, grid_x, ty0, T, tile_bits(T), cap};
#define GSR_BIN_LAUNCH(TM)                                                                                     \
    do {                                                                                                       \
        hipLaunchKernelGGL(bin_count_kernel<TM>, dim3(sgm.nseg), dim3(256), 0, s, a, mat);                     \
        hipLaunchKernelGGL(bin_colscan_kernel, dim3(div_up(T, 64)), dim3(1024), 0, s, mat, sgm.nseg, T, totals); \
        hipLaunchKernelGGL(bin_ranges_kernel, dim3(1), dim3(1024), 0, s, totals, T, tstart, ranges + tile0);   \
        hipLaunchKernelGGL(bin_scatter_kernel<TM>, dim3(sgm.nseg), dim3(64), 0, s, a, mat, tstart, out_gid,    \
                           out_tile, tile0);                                                                   \
    } while (0)
    if (T <= 1024) GSR_BIN_LAUNCH(1024);
    else if (T <= 2048) GSR_BIN_LAUNCH(2048);
    else if (T <= 4096) GSR_BIN_LAUNCH(4096);
    else if (T <= 8192) GSR_BIN_LAUNCH(8192);
    else GSR_BIN_LAUNCH(16384);
#undef GSR_BIN_LAUNCH
    return (int)hipGetLastError();
}

}  // namespace gsr

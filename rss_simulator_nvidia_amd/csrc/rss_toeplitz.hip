// rss_toeplitz.hip -- CDNA4 (gfx950) RSS Toeplitz engine: the IPv4 and IPv6 hash kernels, the
// many-queues passes, the counts-only register-table kernel, the synthetic-input generator and
// their launchers.  Shared device code and launch setup: rss_kernel_common.h; key search:
// rss_keysearch.hip; the C ABI and the host pipeline around them: rss_host.hip (all three
// through rss_engine.h).  The only file compiled twice (product, -DRSS_TEST_HOOKS).
//
// Hot path replaced (reference noamsto/rss_simulator_nvidia v0.0.2):
//   Toeplitz.compute_hash            rss_simulator/toeplitz.py:46-69
//   Simulator.calc_hash / entry hash rss_simulator/simulator.py:74-92
//   Simulator.calc_queue_number      rss_simulator/simulator.py:94-98
//   value_counts in write_statistics rss_simulator/simulator.py:107-113
//
// Kernel shape: one lane per tuple, 4 consecutive tuples per lane
// per iteration (3 x dwordx4 loads, nontemporal hash/queue stores), persistent
// grid-stride launch of one 1024-thread workgroup per CU.  The Toeplitz hash is
// evaluated from 8 LDS tables of 4096 entries (the XOR of the key windows each
// 12-bit slice of the input selects, 128 KiB, built per workgroup from the 96
// windows; slices cut field-LSB first so structured flows spread over the LDS
// banks): 8 ds_read_b32 + ~31 VALU per tuple instead of the reference's 96-step
// bit-serial loop (XOR trees as three-input v_bitop3).  IPv6 uses 29 word-aligned
// 11/11/10-bit and byte tables.  The per-queue histogram is privatised per lane column in
// LDS and folded into global uint64 counts once per workgroup.
// tools/kbench.hip holds the measured design space (4/6/8/12-bit tables).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rss_engine.h"
#include "rss_internal.h"
#include "rss_kernel_common.h"
#include "rss_toeplitz.h"

namespace {

template <bool kHPow2, int kQMode, int kHist, int kQWidth, bool kSmallLut>
__device__ __forceinline__ void one_tuple(const uint32_t* lut, uint32_t* bins, uint64_t i,
                                          uint32_t col, uint32_t hi, const uint32_t* reta_lds,
                                          const LaunchParams& p, char* rlist, uint32_t& rcount) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(p.tuples) + 3 * i;
    const uint32_t h = hash_of<kSmallLut>(lut, src[0], src[1], src[2], hi);
    const uint32_t q = queue_lookup<kQMode>(bucket_of<kHPow2>(h, p), p, reta_lds);
    if (p.hash_out) stream_store(p.hash_out + i, h);
    if (p.queue_out) store_queue1<kStoreWidth<kQWidth>>(p.queue_out, i, column_queue<kQWidth>(q, p));
    if constexpr (kSmallLut && kHist == HIST_RANGE8) {
        if (p.resid_out) {
            const uint32_t qq[1] = {q};
            resid_append<1>(p, rlist, rcount, qq);
        }
    }
    count_queue<kHist>(bins, q, col, p);
}

// kOff32 (with kVec4): every byte offset of the launch's streams fits 32 bits (12 n < 2^32,
// e.g. 2^28 tuples), so the loads and stores address the kernel-argument base pointers with
// a 32-bit per-lane offset (global_load ... v_off, s[base]) instead of 64-bit address pairs.
// kSmallLut: the 2.6 KiB conflict-free small tables instead of the 128 KiB 12-bit ones (many-queues
// HIST_RANGE16 launches: the rest of the LDS holds up to ~75000 u16 bins).
template <bool kHPow2, int kQMode, int kHist, int kQWidth, bool kVec4, bool kOff32 = false,
          bool kSmallLut = false>
__global__ __launch_bounds__(kBlock) void rss_toeplitz_kernel(const LaunchParams p) {
    // static: table offsets fold into ds_read; the small tables keep two more dwords for the
    // balanced tail's LDS slot (their launches' bins fill the rest of the LDS)
    __shared__ __attribute__((aligned(16))) uint32_t lut[kSmallLut ? kSmallLutDwords + 2 : kLutDwords];
    extern __shared__ uint32_t bins[];    // histogram bins, sized at launch
    const uint32_t tid = threadIdx.x;

    if constexpr (kSmallLut) {
        build_small_lut(lut, p.window, tid);
    } else {
        build_lut(lut, p.window, tid);
    }
    const uint32_t nbins = kHist == HIST_PRIVATE   ? p.Q * kBinCols
                         : kHist == HIST_SHARED    ? p.Q
                         : kHist == HIST_RANGE     ? p.q_span
                         : kHist == HIST_RANGE16   ? (p.q_span + 1) / 2
                         : kHist == HIST_RANGE8    ? (p.q_span + 3) / 4 : 0u;  // dwords
    for (uint32_t e = tid; e < nbins; e += kBlock) bins[e] = 0;
    uint32_t* reta_lds = bins + nbins;  // QM_TABLE: H entries after the bins
    if constexpr (kQMode == QM_TABLE)
        for (uint32_t e = tid; e < p.H; e += kBlock) reta_lds[e] = p.reta[e];
    __syncthreads();

    const uint32_t col = tid & (kBinCols - 1);
    uint32_t hi = 4 * kTableEntries * 4;  // byte base of tables 4..7
    asm volatile("" : "+v"(hi));          // keep it opaque (see chunk_offset)
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    uint64_t tail_begin = 0;
    // HIST_RANGE8 counts only past the LDS range: this wave's residual list and its length
    char* rlist = nullptr;
    uint32_t rcount = 0;
    if constexpr (kSmallLut && kHist == HIST_RANGE8)
        if (p.resid_out) rlist = resid_list(p);

    if constexpr (kVec4) {
        // 4 consecutive tuples per lane: 48 B = 3 x dwordx4, 16-B aligned.
        const uint4* __restrict__ src = reinterpret_cast<const uint4*>(p.tuples);
        const uint64_t ngroups = p.n >> 2;
        auto load = [&](uint64_t g, uint4& a, uint4& b, uint4& c) {
            if constexpr (kOff32) {
                const char* base = reinterpret_cast<const char*>(p.tuples);
                const uint32_t off = 48u * (uint32_t)g;
                a = *reinterpret_cast<const uint4*>(base + off);
                b = *reinterpret_cast<const uint4*>(base + off + 16u);
                c = *reinterpret_cast<const uint4*>(base + off + 32u);
            } else {
                a = src[3 * g + 0];
                b = src[3 * g + 1];
                c = src[3 * g + 2];
            }
        };
        auto body = [&](uint64_t g, const uint4 a, const uint4 b, const uint4 c) {
            const uint32_t h0 = hash_of<kSmallLut>(lut, a.x, a.y, a.z, hi);
            const uint32_t h1 = hash_of<kSmallLut>(lut, a.w, b.x, b.y, hi);
            const uint32_t h2 = hash_of<kSmallLut>(lut, b.z, b.w, c.x, hi);
            const uint32_t h3 = hash_of<kSmallLut>(lut, c.y, c.z, c.w, hi);
            const uint32_t q0 = queue_lookup<kQMode>(bucket_of<kHPow2>(h0, p), p, reta_lds);
            const uint32_t q1 = queue_lookup<kQMode>(bucket_of<kHPow2>(h1, p), p, reta_lds);
            const uint32_t q2 = queue_lookup<kQMode>(bucket_of<kHPow2>(h2, p), p, reta_lds);
            const uint32_t q3 = queue_lookup<kQMode>(bucket_of<kHPow2>(h3, p), p, reta_lds);
            if (p.hash_out) {
                uint32_t* o = kOff32 ? reinterpret_cast<uint32_t*>(
                                           reinterpret_cast<char*>(p.hash_out) + 16u * (uint32_t)g)
                                     : p.hash_out + 4 * g;
                stream_store(o, h0);
                stream_store(o + 1, h1);
                stream_store(o + 2, h2);
                stream_store(o + 3, h3);
            }
            if (p.queue_out) {
                constexpr int kW = kStoreWidth<kQWidth>;
                const uint32_t c0 = column_queue<kQWidth>(q0, p), c1 = column_queue<kQWidth>(q1, p);
                const uint32_t c2 = column_queue<kQWidth>(q2, p), c3 = column_queue<kQWidth>(q3, p);
                if constexpr (kOff32)
                    store_queue4<kW>(p.queue_out, (uint32_t)g, c0, c1, c2, c3);
                else
                    store_queue4<kW>(p.queue_out, g, c0, c1, c2, c3);
            }
            if constexpr (kSmallLut && kHist == HIST_RANGE8) {
                if (p.resid_out) {
                    const uint32_t qq[4] = {q0, q1, q2, q3};
                    resid_append<4>(p, rlist, rcount, qq);
                }
            }
            if constexpr (kHist == HIST_RANGE16) {
                const uint32_t o0 = range16_add(bins, q0, p), o1 = range16_add(bins, q1, p);
                const uint32_t o2 = range16_add(bins, q2, p), o3 = range16_add(bins, q3, p);
                range16_guard(bins, q0, o0, p);
                range16_guard(bins, q1, o1, p);
                range16_guard(bins, q2, o2, p);
                range16_guard(bins, q3, o3, p);
            } else if constexpr (kHist == HIST_RANGE8) {
                const uint32_t o0 = range8_add(bins, q0, p), o1 = range8_add(bins, q1, p);
                const uint32_t o2 = range8_add(bins, q2, p), o3 = range8_add(bins, q3, p);
                range8_guard(bins, q0, o0, p);
                range8_guard(bins, q1, o1, p);
                range8_guard(bins, q2, o2, p);
                range8_guard(bins, q3, o3, p);
            } else {
                count_queue<kHist>(bins, q0, col, p);
                count_queue<kHist>(bins, q1, col, p);
                count_queue<kHist>(bins, q2, col, p);
                count_queue<kHist>(bins, q3, col, p);
            }
        };
        auto group = [&](uint64_t g) {
            uint4 a, b, c;
            load(g, a, b, c);
            body(g, a, b, c);
        };
        bool walked = false;
        if constexpr (kSmallLut) {
            // many-queues passes (LDS-heavy: 12 table reads and a returning atomic per tuple):
            // the next group's loads are issued before this group's LDS work (p.prefetch)
            if (p.prefetch && !p.tail_rows) {
                uint64_t g = gtid;
                uint4 a, b, c;
                if (g < ngroups) load(g, a, b, c);
                while (g < ngroups) {
                    const uint64_t gn = g + gstride;
                    uint4 an = a, bn = b, cn = c;
                    if (gn < ngroups) load(gn, an, bn, cn);
                    body(g, a, b, c);
                    a = an;
                    b = bn;
                    c = cn;
                    g = gn;
                }
                walked = true;
            }
        }
        if (!walked)
            walk_rows(group, ngroups, p.tail_rows,
                      p.tail_ctr ? p.tail_ctr : ws_tail_counter(p.ws, p.Q),
                      kSmallLut ? reinterpret_cast<unsigned long long*>(lut + kSmallLutDwords)
                                : reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(bins) + p.bal_off));
        tail_begin = ngroups << 2;
    }
    for (uint64_t i = tail_begin + gtid; i < p.n; i += gstride)
        one_tuple<kHPow2, kQMode, kHist, kQWidth, kSmallLut>(lut, bins, i, col, hi, reta_lds, p, rlist,
                                                             rcount);

    // Epilogue: fold this workgroup's bins into the global uint64 counts.
    if constexpr (kHist == HIST_PRIVATE || kHist == HIST_SHARED) {
        __syncthreads();
        fold_counts([&](uint32_t q) {
            if constexpr (kHist == HIST_PRIVATE) {
                uint32_t s = 0;  // rotated column order: conflict-free
                for (uint32_t c = 0; c < kBinCols; ++c)
                    s += bins[q * kBinCols + ((c + q) & (kBinCols - 1))];
                return s;
            } else {
                return bins[q];
            }
        }, p.Q, p.counts, p.ws, p.accumulate);
    } else if constexpr (kHist == HIST_RANGE) {
        __syncthreads();
        for (uint32_t r = tid; r < p.q_span; r += kBlock)
            if (bins[r]) atomicAdd(&p.counts[p.q_lo + r], (unsigned long long)bins[r]);
    } else if constexpr (kHist == HIST_RANGE16) {
        __syncthreads();  // one row of the u16 partial matrix (rss_partial_reduce_kernel)
        uint32_t* row = p.partial + (size_t)blockIdx.x * p.partial_stride;
        for (uint32_t w = tid; w < nbins; w += kBlock) row[w] = bins[w];
    } else if constexpr (kHist == HIST_RANGE8) {
        __syncthreads();  // one row of the u8 partial matrix
        uint32_t* row = p.partial + (size_t)blockIdx.x * p.partial_stride;
        for (uint32_t w = tid; w < nbins; w += kBlock) row[w] = bins[w];
        if constexpr (kSmallLut)  // (lane 0 took part in every append of its wave)
            if (p.resid_out && (tid & 63u) == 0)
                p.resid_counts[(uint64_t)blockIdx.x * kWavesPerBlock + (tid >> 6)] = rcount;
    }
}

// HIST_RANGE passes after the first: histogram one range of queues straight from the
// queue_number array the first pass wrote (2 or 4 B/tuple instead of re-reading 12 B and
// rehashing): shared LDS bins for [q_lo, q_lo + q_span), 16-B loads when aligned.
template <typename T>
__global__ __launch_bounds__(kBlock) void rss_queue_hist_kernel(const T* __restrict__ queues,
                                                                uint64_t n, uint32_t q_lo,
                                                                uint32_t q_span,
                                                                unsigned long long* counts) {
    extern __shared__ uint32_t bins[];
    const uint32_t tid = threadIdx.x;
    for (uint32_t e = tid; e < q_span; e += kBlock) bins[e] = 0;
    __syncthreads();
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    auto add = [&](uint32_t q) {
        const uint32_t r = q - q_lo;
        if (r < q_span)
            __hip_atomic_fetch_add(&bins[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    constexpr uint32_t kPer = 16 / sizeof(T);  // queues per 16-B load
    uint64_t tail = 0;
    if (((uintptr_t)queues & 15) == 0) {
        const uint4* __restrict__ v = reinterpret_cast<const uint4*>(queues);
        const uint64_t nv = n / kPer;
        for (uint64_t i = gtid; i < nv; i += gstride) {
            const uint4 x = v[i];
            const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if constexpr (sizeof(T) == 2) {
                    add(w[k] & 0xFFFFu);
                    add(w[k] >> 16);
                } else {
                    add(w[k]);
                }
            }
        }
        tail = nv * kPer;
    }
    for (uint64_t i = tail + gtid; i < n; i += gstride) add(queues[i]);
    __syncthreads();
    for (uint32_t r = tid; r < q_span; r += kBlock)
        if (bins[r]) atomicAdd(&counts[q_lo + r], (unsigned long long)bins[r]);
}

// Queue ranges past the first pass's LDS bins, wide: ONE pass over the queue column per
// range of up to kWideSpan (u16 bins) or kWideSpan8 (u8 bins) queues instead of one per
// 16384 u32 bins.  The bins carry the hash pass's guard and poison word (range16_guard /
// range8_guard): the add that takes a field to half range moves half into ovf[r], the add
// that sees a full field (a wrap) poisons the pass, whose rows and moves the reduce then
// discards while rss_range_fallback_col_kernel recounts the range.  Each workgroup stores its
// bins as one row of a [grid][stride] matrix with plain coalesced stores -- not Q atomics per
// workgroup, which would cost more than the pass at Q = 65536 -- and
// rss_partial_reduce_kernel sums the rows and moves into the counts.
constexpr uint32_t kWideSpan = 65536;  // 128 KiB of u16 bins: one workgroup per CU
constexpr uint32_t kWideSpan8 = 163840;  // u8 bins (kBits = 8): the whole 160 KiB LDS
constexpr uint32_t kNarrowSpan = 16384;  // rss_queue_hist_kernel: u32 bins, two workgroups per CU

// regions (region_counts != NULL): the column is one list per hash-pass wave -- wave v of
// workgroup x reads the region_counts[16 x + v] entries at queues + (16 x + v) * region_cap
// (the hash pass's residual lists, resid_append) instead of grid-striding over n entries.
template <typename T, int kBits = 16>
__global__ __launch_bounds__(kBlock) void rss_queue_hist_wide_kernel(
        const T* __restrict__ queues, uint64_t n, uint32_t q_lo, uint32_t q_span,
        uint32_t* __restrict__ partial, uint32_t stride_words,
        uint32_t* __restrict__ ovf, uint32_t* __restrict__ poison,
        const uint32_t* __restrict__ region_counts, uint64_t region_cap) {
    constexpr uint32_t kPerWord = 32 / kBits, kField = (1u << kBits) - 1u;
    constexpr uint32_t kHalf = 1u << (kBits - 1);  // the guard's move
    extern __shared__ uint32_t bins[];
    const uint32_t tid = threadIdx.x;
    const uint32_t words = (q_span + kPerWord - 1) / kPerWord;
    for (uint32_t e = tid; e < words; e += kBlock) bins[e] = 0;
    __syncthreads();
    uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    if (region_counts) {  // wave v reads list 16 x + v
        const uint64_t list = (uint64_t)blockIdx.x * kWavesPerBlock + (tid >> 6);
        queues += list * region_cap;
        n = region_counts[list];
        gtid = tid & 63u;
        gstride = 64;
    }
    // the add of one queue; returns the bin's previous value (0 when q is out of range)
    auto add = [&](uint32_t q) -> uint32_t {
        const uint32_t r = q - q_lo;  // wraps for q < q_lo
        if (r >= q_span) return 0u;
        const uint32_t sh = (r % kPerWord) * kBits;
        return __hip_atomic_fetch_add(&bins[r / kPerWord], 1u << sh, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // the guard: the add that returned kHalf - 1 (its bin now holds kHalf) moves kHalf out.
    // Checked after a group's adds are all issued, so they do not wait for each other.  The
    // adds that land before its subtract are not bounded (range16_guard), so the add that sees
    // kField (a wrap) poisons the pass.
    auto guard = [&](uint32_t q, uint32_t old) {
        const uint32_t r = q - q_lo;
        if (r >= q_span) return;
        const uint32_t sh = (r % kPerWord) * kBits;
        const uint32_t f = (old >> sh) & kField;
        if (f == kHalf - 1u) {
            if constexpr (kBits == 16) RSS_GUARD_DELAY();
            const uint32_t at = __hip_atomic_fetch_sub(&bins[r / kPerWord], kHalf << sh,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            RSS_RECORD_MARGIN(kBits, kBits == 16 ? kMarginWide16 : kMarginWide8, (at >> sh) & kField);
            atomicAdd(&ovf[r], 1u);
        } else if (f == kField) {
            __hip_atomic_store(poison, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    constexpr uint32_t kPer = 16 / sizeof(T);  // queues per 16-B load
    auto add16 = [&](const uint4 x) {
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
        uint32_t q[kPer], old[kPer];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (sizeof(T) == 2) {
                q[2 * k] = w[k] & 0xFFFFu;
                q[2 * k + 1] = w[k] >> 16;
            } else {
                q[k] = w[k];
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) old[k] = add(q[k]);
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) guard(q[k], old[k]);
    };
    uint64_t tail = 0;
    if (((uintptr_t)queues & 15) == 0) {
        // four 16-B loads in flight per lane: the adds wait for their returned values (the
        // guard check), so one load per iteration would leave the stream latency-bound at
        // one workgroup per CU
        constexpr int kUnroll = 4;
        const uint4* __restrict__ v = reinterpret_cast<const uint4*>(queues);
        const uint64_t nv = n / kPer;
        uint64_t i = gtid;
        for (; i + (kUnroll - 1) * gstride < nv; i += kUnroll * gstride) {
            uint4 x[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) x[u] = v[i + u * gstride];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) add16(x[u]);
        }
        for (; i < nv; i += gstride) add16(v[i]);
        tail = nv * kPer;
    }
    for (uint64_t i = tail + gtid; i < n; i += gstride) {
        const uint32_t q = queues[i];
        guard(q, add(q));
    }
    __syncthreads();
    uint32_t* row = partial + (size_t)blockIdx.x * stride_words;
    for (uint32_t e = tid; e < words; e += kBlock) row[e] = bins[e];
}

// counts[q_lo + q] += sum over the `rows` rows of the u16 (kBits = 16) or u8 (kBits = 8)
// partial matrix (column q) + 2^(kBits - 1) x its guard moves ovf[q].  A workgroup takes a
// strip of 64 dwords (128 or 256 queues) of every row: its 256 threads are 64 columns x 4 row
// groups, each summing its rows' dword with eight loads in flight, then the 4 row groups meet
// in LDS.  (One thread per queue summing all rows ran 60 us per 65536-queue range at 2^28
// tuples -- as long as half the wide pass; profiles/r03/mqprof.)  A poisoned pass's rows and
// moves are discarded here (a bin wrapped): the recount (rss_range_fallback_kernel /
// rss_range_fallback_col_kernel, gated on the same word) takes the range instead.
constexpr uint32_t kReduceCols = 64, kReduceGroups = 4;
template <int kBits>
__global__ __launch_bounds__(kReduceCols * kReduceGroups) void rss_partial_reduce_kernel(
        const uint32_t* __restrict__ partial, uint32_t rows, uint32_t stride_words, uint32_t q_lo,
        uint32_t q_span, unsigned long long* counts, const uint32_t* __restrict__ ovf,
        const uint32_t* __restrict__ poison) {
    constexpr uint32_t kPer = 32 / kBits, kMask = (1u << kBits) - 1u;
    if (*poison) return;  // uniform: the recount takes this range
    __shared__ unsigned long long part[kReduceGroups][kReduceCols][kPer];
    const uint32_t col = threadIdx.x % kReduceCols, grp = threadIdx.x / kReduceCols;
    const uint32_t word = blockIdx.x * kReduceCols + col;  // queues kPer * word + f
    unsigned long long acc[kPer];
#pragma unroll
    for (uint32_t f = 0; f < kPer; ++f) acc[f] = 0;
    auto take = [&](uint32_t x) {
#pragma unroll
        for (uint32_t f = 0; f < kPer; ++f) acc[f] += (x >> (f * kBits)) & kMask;
    };
    if (word < stride_words) {
        constexpr uint32_t kIn = 8;
        uint32_t r = grp;
        for (; r + (kIn - 1) * kReduceGroups < rows; r += kIn * kReduceGroups) {
            uint32_t x[kIn];
#pragma unroll
            for (uint32_t k = 0; k < kIn; ++k) x[k] = partial[(size_t)(r + k * kReduceGroups) * stride_words + word];
#pragma unroll
            for (uint32_t k = 0; k < kIn; ++k) take(x[k]);
        }
        for (; r < rows; r += kReduceGroups) take(partial[(size_t)r * stride_words + word]);
    }
#pragma unroll
    for (uint32_t f = 0; f < kPer; ++f) part[grp][col][f] = acc[f];
    __syncthreads();
    if (grp == 0) {
#pragma unroll
        for (uint32_t f = 0; f < kPer; ++f) {
            for (uint32_t g = 1; g < kReduceGroups; ++g) acc[f] += part[g][col][f];
            const uint32_t q = kPer * word + f;
            if (q < q_span) {
                const unsigned long long v = acc[f] + (1ull << (kBits - 1)) * ovf[q];
                if (v) counts[q_lo + q] += v;
            }
        }
    }
}

// The recount of a guarded pass (range16_guard / range8_guard), launched after each one:
// returns at once unless the pass raised its poison word.  Then every workgroup counts the
// range in slices with u32 LDS bins (no guard needed: a bin holds one workgroup's share of
// the batch) and folds each slice with atomics into the counts.  Slow (a pass over the batch
// per slice), exact, and only ever run on inputs that pile thousands of tuples into one bin
// at once.  Two forms: this one hashes the tuples again on the small tables (a hash pass that
// writes no column holding the queues; any table partition gives the exact hash) with
// p.fb_span u32 bins per slice and, for QM_TABLE, the indirection table after them;
// rss_range_fallback_col_kernel reads a queue column (a wide pass, or a hash pass whose
// column holds the queues).
constexpr uint32_t kFallbackColSpan = 40960;  // 160 KiB of u32 bins
template <bool kHPow2, int kQMode>
__global__ __launch_bounds__(kBlock) void rss_range_fallback_kernel(const LaunchParams p) {
    if (!*p.poison) return;  // uniform across the grid: no wave is left behind
    __shared__ uint32_t lut[kSmallLutDwords];
    extern __shared__ uint32_t bins[];
    uint32_t* reta_lds = bins + p.fb_span;  // QM_TABLE: H entries after the bins
    const uint32_t tid = threadIdx.x;
    build_small_lut(lut, p.window, tid);
    if constexpr (kQMode == QM_TABLE)
        for (uint32_t e = tid; e < p.H; e += kBlock) reta_lds[e] = p.reta[e];
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    for (uint32_t lo = 0; lo < p.q_span; lo += p.fb_span) {
        const uint32_t span = min(p.fb_span, p.q_span - lo);
        for (uint32_t e = tid; e < span; e += kBlock) bins[e] = 0;
        __syncthreads();
        for (uint64_t i = gtid; i < p.n; i += gstride) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(p.tuples) + 3 * i;
            const uint32_t h = toeplitz_hash_small(lut, src[0], src[1], src[2]);
            const uint32_t r = queue_lookup<kQMode>(bucket_of<kHPow2>(h, p), p, reta_lds) - p.q_lo - lo;
            if (r < span)  // (wraps below the slice)
                __hip_atomic_fetch_add(&bins[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        for (uint32_t e = tid; e < span; e += kBlock)
            if (bins[e]) atomicAdd(&p.counts[p.q_lo + lo + e], (unsigned long long)bins[e]);
        __syncthreads();
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void rss_range_fallback_col_kernel(
        const T* __restrict__ col, uint64_t n, uint32_t q_lo, uint32_t q_span,
        unsigned long long* counts, const uint32_t* __restrict__ poison,
        const uint32_t* __restrict__ region_counts, uint64_t region_cap) {
    if (!*poison) return;  // uniform across the grid
    extern __shared__ uint32_t bins[];
    const uint32_t tid = threadIdx.x;
    uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    if (region_counts) {  // one residual list per wave (see rss_queue_hist_wide_kernel)
        const uint64_t list = (uint64_t)blockIdx.x * kWavesPerBlock + (tid >> 6);
        col += list * region_cap;
        n = region_counts[list];
        gtid = tid & 63u;
        gstride = 64;
    }
    for (uint32_t lo = 0; lo < q_span; lo += kFallbackColSpan) {
        const uint32_t span = min(kFallbackColSpan, q_span - lo);
        for (uint32_t e = tid; e < span; e += kBlock) bins[e] = 0;
        __syncthreads();
        for (uint64_t i = gtid; i < n; i += gstride) {
            const uint32_t r = (uint32_t)col[i] - q_lo - lo;  // wraps below the slice
            if (r < span)
                __hip_atomic_fetch_add(&bins[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        for (uint32_t e = tid; e < span; e += kBlock)
            if (bins[e]) atomicAdd(&counts[q_lo + lo + e], (unsigned long long)bins[e]);
        __syncthreads();
    }
}

// Counts only, power-of-two H <= 256 (histogram mode, `rss_hash_host` without per-tuple
// outputs): the queue depends on hash & (H-1) alone, at most 8 bits, so every table term
// fits a byte and the tables move from LDS into registers.  Each input byte is cut into
// 3 + 3 + 2-bit fields (36 fields, field LSBs first as above); field f's <= 8-entry byte
// table is two dwords, and v_perm_b32 looks up all four selector bytes of a dword in it at
// once.  A lane's four tuples are byte-transposed (8 v_perm per word) so that one selector
// dword holds the same field of the four tuples: one v_perm = one field of four tuples,
// and the XOR of the 36 lookups is the four tuples' buckets, one per byte.  Per four
// tuples ~170 VALU (60 v_perm) and 4 conflict-free `ds_add_u32` -- against 8 random-index
// `ds_read_b32` per tuple in the LUT kernel, whose bank conflicts bind it in this mode
// (DESIGN.md §3).  Measured 0.525-0.531 vs 0.545-0.548 ms per 2^28 tuples, read-only
// stream 0.513-0.519 (profiles/r02/perm_counts.log).
// The same kernel serves IPv6 (nine words, 108 fields, rss_hash6_device counts only).
template <int kWords>
struct PermParams {
    static constexpr int kFields = kWords * 12;  // three fields per input byte
    const uint32_t* tuples;  // kWords words per tuple
    unsigned long long* counts;
    unsigned long long* ws;  // single-pass counts workspace or NULL (fold_counts)
    uint32_t accumulate;
    uint64_t n;
    uint32_t Q;
    uint32_t q_mask;    // QM_MASK
    uint32_t q_m16;     // QM_FAST8
    uint32_t tail_rows; // balanced tail (walk_rows), with ws only
    uint32_t bal_off;   // its LDS slot's byte offset in the dynamic LDS
    uint32_t lo[kFields];  // field f: table entries 0..3 (v_perm selector 0..3)
    uint32_t hi[kFields];  //          entries 4..7 (selector 4..7)
};

__device__ __forceinline__ uint32_t vperm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}

// t_j = byte j of (x0, x1, x2, x3), tuple i in byte i
__device__ __forceinline__ void transpose_bytes(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3,
                                                uint32_t& t0, uint32_t& t1, uint32_t& t2,
                                                uint32_t& t3) {
    const uint32_t a = vperm(x1, x0, 0x05010400u), b = vperm(x1, x0, 0x07030602u);
    const uint32_t c = vperm(x3, x2, 0x05010400u), d = vperm(x3, x2, 0x07030602u);
    t0 = vperm(c, a, 0x05040100u);
    t1 = vperm(c, a, 0x07060302u);
    t2 = vperm(d, b, 0x05040100u);
    t3 = vperm(d, b, 0x07060302u);
}

// XOR of the three field terms of byte-transposed dword t (fields f .. f+2)
template <int kWords>
__device__ __forceinline__ uint32_t perm_byte_terms(const PermParams<kWords>& p, int f, uint32_t t) {
    const uint32_t f0 = vperm(p.hi[f], p.lo[f], t & 0x07070707u);
    const uint32_t f1 = vperm(p.hi[f + 1], p.lo[f + 1], (t >> 3) & 0x07070707u);
    const uint32_t f2 = vperm(p.lo[f + 2], p.lo[f + 2], (t >> 6) & 0x03030303u);
    return xor3(f0, f1, f2);
}

// buckets of four tuples (tuple i's hash & (H-1) in byte i); w = 4 x kWords words, tuple-major
template <int kWords>
__device__ __forceinline__ uint32_t perm_buckets(const PermParams<kWords>& p,
                                                 const uint32_t (&w)[4 * kWords]) {
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < kWords; ++k) {  // fully unrolled: every field index is a constant
        uint32_t t0, t1, t2, t3;
        transpose_bytes(w[k], w[kWords + k], w[2 * kWords + k], w[3 * kWords + k], t0, t1, t2, t3);
        acc = xor3(xor3(acc, perm_byte_terms(p, 12 * k + 0, t0), perm_byte_terms(p, 12 * k + 3, t1)),
                   perm_byte_terms(p, 12 * k + 6, t2), perm_byte_terms(p, 12 * k + 9, t3));
    }
    return acc;
}

template <int kQMode, int kWords>
__device__ __forceinline__ uint32_t perm_queue(uint32_t b, const PermParams<kWords>& p) {
    if constexpr (kQMode == QM_MASK) return b & p.q_mask;
    return b - __umul24(__umul24(b, p.q_m16) >> 16, p.Q);  // QM_FAST8: b, Q < 256
}

__device__ __forceinline__ void perm_count(uint32_t* bins, uint32_t q, uint32_t col) {
    __hip_atomic_fetch_add(&bins[q * kBinCols + col], 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int kQMode, int kWords>
__global__ __launch_bounds__(kBlock, 2) void rss_counts_perm_kernel(const PermParams<kWords> p) {
    extern __shared__ uint32_t bins[];  // Q x 32 private columns
    const uint32_t tid = threadIdx.x, col = tid & (kBinCols - 1);
    for (uint32_t e = tid; e < p.Q * kBinCols; e += kBlock) bins[e] = 0;
    __syncthreads();
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ngroups = p.n >> 2;
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    walk_rows([&](uint64_t g) {
        uint32_t w[4 * kWords];  // four tuples = kWords x 16 B, 16-B aligned
#pragma unroll
        for (int v = 0; v < kWords; ++v) {
            const uint4 x = src[kWords * g + v];
            w[4 * v] = x.x;
            w[4 * v + 1] = x.y;
            w[4 * v + 2] = x.z;
            w[4 * v + 3] = x.w;
        }
        const uint32_t bk = perm_buckets(p, w);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            perm_count(bins, perm_queue<kQMode>((bk >> (8 * i)) & 0xFFu, p), col);
    }, ngroups, p.tail_rows, ws_tail_counter(p.ws, p.Q),
       reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(bins) + p.bal_off));
    // the last n % 4 tuples: one per lane of the first workgroup, in byte 0
    const uint64_t i = (ngroups << 2) + gtid;
    if (i < p.n) {
        uint32_t w[4 * kWords] = {};
#pragma unroll
        for (int k = 0; k < kWords; ++k) w[k] = p.tuples[kWords * i + k];
        perm_count(bins, perm_queue<kQMode>(perm_buckets(p, w) & 0xFFu, p), col);
    }
    __syncthreads();
    fold_counts([&](uint32_t q) {  // rotated reads: conflict-free
        uint32_t s = 0;
        for (uint32_t c = 0; c < kBinCols; ++c) s += bins[q * kBinCols + ((c + q) & (kBinCols - 1))];
        return s;
    }, p.Q, p.counts, p.ws, p.accumulate);
}

// ------------------------------------------------------------- IPv6 -------
// 36-byte input: nine big-endian words, 288 bits (w0..w3 src
// address, w4..w7 dst address, w8 ports).  12-bit tables would need 384 KiB, so the
// words are cut at word-internal positions into tables that fit the 160 KiB LDS:
//   w1 w2 w3 w5 w6 w7 w8: [10:0] (2048 entries), [21:11] (2048), [31:22] (1024)
//   w0 w4 (the network prefixes, which vary least): four byte tables each
// = 14 x 8 KiB + 7 x 4 KiB + 8 x 1 KiB = 148 KiB, 29 ds_read_b32 per tuple (36 with
// byte tables only), one 1024-thread workgroup per CU.  Every table index starts at a
// word-internal bit so the host / port bits that vary between flows select the bank.
constexpr int kWords6 = RSS_INPUT6_BITS / 32;              // 9
constexpr uint32_t kLut6Bytes = 14 * 8192 + 7 * 4096 + 8 * 1024;   // 151552
constexpr uint32_t kLut6Dwords = kLut6Bytes / 4;
constexpr uint32_t kBinBytesMax6 = kLdsBytes - kLut6Bytes;          // 12 KiB
constexpr int kBlocksPerCU6 = 1;

__host__ __device__ constexpr bool byte_word6(int k) { return k == 0 || k == 4; }
// index of word k among the seven 11/11/10-split words (w1 w2 w3 w5 w6 w7 w8 -> 0..6)
__host__ __device__ constexpr int wide_rank6(int k) { return k < 4 ? k - 1 : k - 2; }
// slice j of word k: low bit in the word, width, byte offset of its table
__host__ __device__ constexpr int slice_lo6(int k, int j) {
    return byte_word6(k) ? 8 * j : (j == 0 ? 0 : (j == 1 ? 11 : 22));
}
__host__ __device__ constexpr int slice_width6(int k, int j) {
    return byte_word6(k) ? 8 : (j == 2 ? 10 : 11);
}
__host__ __device__ constexpr uint32_t slice_table6(int k, int j) {
    return byte_word6(k) ? 14 * 8192 + 7 * 4096 + ((k == 0 ? 0 : 4) + j) * 1024
         : j < 2         ? (2 * wide_rank6(k) + j) * 8192
                         : 14 * 8192 + wide_rank6(k) * 4096;
}
constexpr int slices6(int k) { return byte_word6(k) ? 4 : 3; }
static_assert(kLut6Bytes + 32 * 4 * 24 <= kLdsBytes, "IPv6 LUT + private bins for 24 queues fit");
static_assert(kBinBytesMax6 >= 4 * kRetaMax + 4096, "IPv6 bins keep >= 4 KiB beside a full RETA");

struct LaunchParams6 {
    uint32_t window[RSS_INPUT6_BITS];
    const rss_tuple6* tuples;
    uint32_t* hash_out;
    void* queue_out;
    unsigned long long* counts;
    uint64_t n;
    uint64_t h_m64;
    uint32_t h_mask, H, Q, q_mask, q_m32;
    uint32_t qwidth;  // QueueWidth of queue_out (grid-uniform runtime switch)
    uint32_t q_m16;
    uint64_t q_m64;
    uint32_t q_lo, q_span;    // HIST_RANGE, as LaunchParams
    unsigned long long* ws;   // single-pass counts workspace (rss_hash6_device_ws) or NULL
    uint32_t accumulate;      // with ws: fold mode, as LaunchParams
    uint32_t tail_rows;       // balanced tail rows (0 = static grid-stride), as LaunchParams
    uint32_t bal_off;         // balanced tail: byte offset of its LDS slot (dynamic LDS)
    uint16_t reta[kRetaMax];  // QM_TABLE: queue of bucket b, as LaunchParams::reta
};

// entry v of slice (k, j) = XOR of the windows of the set bits of v; word k bit i is
// input bit 32k + 31 - i (toeplitz.py:65-68 order extended to 36 bytes)
template <int kK, int kJ>
__device__ __forceinline__ void build_slice6(uint32_t* lut, const uint32_t* __restrict__ window,
                                             uint32_t tid) {
    constexpr int lo = slice_lo6(kK, kJ), width = slice_width6(kK, kJ);
    constexpr uint32_t entries = 1u << width;
    uint32_t* dst = lut + slice_table6(kK, kJ) / 4;
    for (uint32_t v = tid; v < entries; v += kBlock) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < width; ++b) x ^= ((v >> b) & 1u) ? window[32 * kK + 31 - lo - b] : 0u;
        dst[v] = x;
    }
}

template <int kK>
__device__ __forceinline__ void build_word6(uint32_t* lut, const uint32_t* __restrict__ window,
                                            uint32_t tid) {
    build_slice6<kK, 0>(lut, window, tid);
    build_slice6<kK, 1>(lut, window, tid);
    build_slice6<kK, 2>(lut, window, tid);
    if constexpr (slices6(kK) == 4) build_slice6<kK, 3>(lut, window, tid);
}

__device__ __forceinline__ void build_lut6(uint32_t* lut, const uint32_t* __restrict__ window,
                                           uint32_t tid) {
    build_word6<0>(lut, window, tid);
    build_word6<1>(lut, window, tid);
    build_word6<2>(lut, window, tid);
    build_word6<3>(lut, window, tid);
    build_word6<4>(lut, window, tid);
    build_word6<5>(lut, window, tid);
    build_word6<6>(lut, window, tid);
    build_word6<7>(lut, window, tid);
    build_word6<8>(lut, window, tid);
}

// One table term: the index moved to bits 2.. and masked (shift + and, or and_or with
// an opaque 64 KiB / 128 KiB base register -- the ds_read immediate holds 16 bits).
template <int kK, int kJ>
__device__ __forceinline__ uint32_t lut6_term(const char* lut, uint32_t w, uint32_t hi1,
                                              uint32_t hi2) {
    constexpr int lo = slice_lo6(kK, kJ), width = slice_width6(kK, kJ);
    constexpr uint32_t mask = ((1u << width) - 1) << 2;
    constexpr uint32_t table = slice_table6(kK, kJ);
    constexpr uint32_t imm = table & 0xFFFFu;
    uint32_t field;
    if constexpr (lo >= 2) {
        field = w >> (lo - 2);
    } else {
        field = w << (2 - lo);
    }
    uint32_t off;
    if constexpr ((table >> 16) == 0) {
        off = field & mask;
    } else if constexpr ((table >> 16) == 1) {
        off = (field & mask) | hi1;
    } else {
        off = (field & mask) | hi2;
    }
    return *reinterpret_cast<const uint32_t*>(lut + imm + off);
}

template <int kK>
__device__ __forceinline__ uint32_t word6_terms(const char* lut, uint32_t w, uint32_t hi1,
                                                uint32_t hi2) {
    uint32_t x = lut6_term<kK, 0>(lut, w, hi1, hi2) ^ lut6_term<kK, 1>(lut, w, hi1, hi2) ^
                 lut6_term<kK, 2>(lut, w, hi1, hi2);
    if constexpr (slices6(kK) == 4) x ^= lut6_term<kK, 3>(lut, w, hi1, hi2);
    return x;
}

__device__ __forceinline__ uint32_t toeplitz_hash6(const uint32_t* __restrict__ lut,
                                                   const uint32_t (&w)[kWords6], uint32_t hi1,
                                                   uint32_t hi2) {
    const char* base = reinterpret_cast<const char*>(lut);
    return (word6_terms<0>(base, w[0], hi1, hi2) ^ word6_terms<1>(base, w[1], hi1, hi2)) ^
           (word6_terms<2>(base, w[2], hi1, hi2) ^ word6_terms<3>(base, w[3], hi1, hi2)) ^
           (word6_terms<4>(base, w[4], hi1, hi2) ^ word6_terms<5>(base, w[5], hi1, hi2)) ^
           (word6_terms<6>(base, w[6], hi1, hi2) ^ word6_terms<7>(base, w[7], hi1, hi2)) ^
           word6_terms<8>(base, w[8], hi1, hi2);
}

template <bool kHPow2, int kQMode, int kHist, bool kVec4>
__global__ __launch_bounds__(kBlock) void rss_toeplitz6_kernel(const LaunchParams6 p6) {
    __shared__ uint32_t lut[kLut6Dwords];
    extern __shared__ uint32_t bins[];
    const uint32_t tid = threadIdx.x;
    build_lut6(lut, p6.window, tid);
    uint32_t hi1 = 0x10000u, hi2 = 0x20000u;  // opaque table bases (see lut6_term)
    asm volatile("" : "+v"(hi1), "+v"(hi2));
    // the modulo / histogram helpers read these LaunchParams fields only
    LaunchParams p;
    p.counts = p6.counts;
    p.h_m64 = p6.h_m64;
    p.h_mask = p6.h_mask;
    p.H = p6.H;
    p.Q = p6.Q;
    p.q_mask = p6.q_mask;
    p.q_m32 = p6.q_m32;
    p.q_m16 = p6.q_m16;
    p.q_m64 = p6.q_m64;
    p.q_lo = p6.q_lo;
    p.q_span = p6.q_span;
    const uint32_t nbins = kHist == HIST_PRIVATE ? p.Q * kBinCols
                         : kHist == HIST_SHARED  ? p.Q
                         : kHist == HIST_RANGE   ? p.q_span : 0u;
    for (uint32_t e = tid; e < nbins; e += kBlock) bins[e] = 0;
    uint32_t* reta_lds = bins + nbins;  // QM_TABLE: H entries after the bins
    if constexpr (kQMode == QM_TABLE)
        for (uint32_t e = tid; e < p6.H; e += kBlock) reta_lds[e] = p6.reta[e];
    __syncthreads();
    const uint32_t col = tid & (kBinCols - 1);
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    uint64_t tail_begin = 0;
    if constexpr (kVec4) {
        // 4 consecutive tuples per lane: 144 B = 9 x dwordx4, 16-B aligned
        const uint4* __restrict__ src = reinterpret_cast<const uint4*>(p6.tuples);
        const uint64_t ngroups = p6.n >> 2;
        auto group = [&](uint64_t g) {
            uint32_t v[4 * kWords6];
#pragma unroll
            for (int k = 0; k < kWords6; ++k) {
                const uint4 x = src[kWords6 * g + k];
                v[4 * k] = x.x;
                v[4 * k + 1] = x.y;
                v[4 * k + 2] = x.z;
                v[4 * k + 3] = x.w;
            }
            uint32_t h[4], q[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                uint32_t w[kWords6];
#pragma unroll
                for (int k = 0; k < kWords6; ++k) w[k] = v[kWords6 * t + k];
                h[t] = toeplitz_hash6(lut, w, hi1, hi2);
                q[t] = queue_lookup<kQMode>(bucket_of<kHPow2>(h[t], p), p, reta_lds);
            }
            if (p6.hash_out) {
                uint32_t* o = p6.hash_out + 4 * g;
#pragma unroll
                for (int t = 0; t < 4; ++t) stream_store(o + t, h[t]);
            }
            if (p6.queue_out) {
                if (p6.qwidth == QW_U8) {
                    store_queue4<QW_U8>(p6.queue_out, g, q[0], q[1], q[2], q[3]);
                } else if (p6.qwidth == QW_U16) {
                    store_queue4<QW_U16>(p6.queue_out, g, q[0], q[1], q[2], q[3]);
                } else {
                    store_queue4<QW_U32>(p6.queue_out, g, q[0], q[1], q[2], q[3]);
                }
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) count_queue<kHist>(bins, q[t], col, p);
        };
        // single-pass launches hand out the last rows per workgroup slot (walk_rows, the
        // balanced tail of the IPv4 kernel): the XCDs that stream faster take more of them
        walk_rows(group, ngroups, p6.tail_rows, ws_tail_counter(p6.ws, p.Q),
                  reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(bins) + p6.bal_off));
        tail_begin = ngroups << 2;
    }
    for (uint64_t i = tail_begin + gtid; i < p6.n; i += gstride) {
        const uint32_t* t = p6.tuples[i].w;
        uint32_t w[kWords6];
#pragma unroll
        for (int k = 0; k < kWords6; ++k) w[k] = t[k];
        const uint32_t h = toeplitz_hash6(lut, w, hi1, hi2);
        const uint32_t q = queue_lookup<kQMode>(bucket_of<kHPow2>(h, p), p, reta_lds);
        if (p6.hash_out) stream_store(p6.hash_out + i, h);
        if (p6.queue_out) {
            if (p6.qwidth == QW_U8) {
                store_queue1<QW_U8>(p6.queue_out, i, q);
            } else if (p6.qwidth == QW_U16) {
                store_queue1<QW_U16>(p6.queue_out, i, q);
            } else {
                store_queue1<QW_U32>(p6.queue_out, i, q);
            }
        }
        count_queue<kHist>(bins, q, col, p);
    }
    if constexpr (kHist == HIST_PRIVATE || kHist == HIST_SHARED) {
        __syncthreads();
        // atomics into the counts, or (single pass) the workspace + the last workgroup's write
        fold_counts([&](uint32_t k) {
            if constexpr (kHist == HIST_PRIVATE) {
                uint32_t s = 0;  // rotated column order: conflict-free
                for (uint32_t c = 0; c < kBinCols; ++c)
                    s += bins[k * kBinCols + ((c + k) & (kBinCols - 1))];
                return s;
            } else {
                return bins[k];
            }
        }, p.Q, p.counts, p6.ws, p6.accumulate);
    } else if constexpr (kHist == HIST_RANGE) {
        __syncthreads();
        for (uint32_t r = tid; r < p.q_span; r += kBlock)
            if (bins[r]) atomicAdd(&p.counts[p.q_lo + r], (unsigned long long)bins[r]);
    }
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void rss_generate_kernel(uint64_t seed, uint64_t first,
                                                           uint64_t n, uint32_t* out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t idx = first + i;
        const uint64_t r0 = mix64(seed + 2 * idx);
        const uint64_t r1 = mix64(seed + 2 * idx + 1);
        out[3 * i + 0] = (uint32_t)(r0 >> 32);
        out[3 * i + 1] = (uint32_t)r0;
        out[3 * i + 2] = (uint32_t)r1;
    }
}


// vec4: 0 = one tuple per lane, 1 = four per lane, 2 = four per lane with 32-bit byte offsets
// (kOff32; instantiated for the single-pass histogram modes only, the bench's step), 3 = four
// per lane on the small tables (kSmallLut; HIST_RANGE16 / HIST_RANGE8 only)
enum VecMode { VM_SCALAR = 0, VM_VEC4 = 1, VM_OFF32 = 2, VM_SMALL_LUT = 3 };
template <bool kHPow2, int kQMode, int kHist, int kQWidth>
KernelFn pick_vec_reachable(int vec4) {
    // (an else-chain: a statement after an `if constexpr` block that returns is still
    // instantiated, so every branch below is one alternative of the chain -- round 5's flat
    // form instantiated 148 unreachable kernels)
    if constexpr (kHist == HIST_RANGE8) {  // small tables, u32 / u16-residual columns only
        if constexpr ((kQWidth == QW_U32 || kQWidth == QW_U16R) && kQMode != QM_FAST8 &&
                      kQMode != QM_TABLE) {
            if (vec4 == VM_SMALL_LUT)
                return rss_toeplitz_kernel<kHPow2, kQMode, kHist, kQWidth, true, false, true>;
        }
        return nullptr;
    } else if constexpr (kQWidth == QW_U16R) {  // the small-table HIST_RANGE16 / RANGE8 bodies only
        if constexpr (kHist == HIST_RANGE16 && kQMode != QM_FAST8 && kQMode != QM_TABLE) {
            if (vec4 == VM_SMALL_LUT)
                return rss_toeplitz_kernel<kHPow2, kQMode, kHist, kQWidth, true, false, true>;
        }
        return nullptr;
    } else {
        if constexpr (kHist == HIST_PRIVATE || kHist == HIST_SHARED) {
            if (vec4 == VM_OFF32) return rss_toeplitz_kernel<kHPow2, kQMode, kHist, kQWidth, true, true>;
        }
        if constexpr (kHist == HIST_RANGE16 && kQWidth != QW_U8 && kQMode != QM_FAST8 &&
                      kQMode != QM_TABLE) {  // (H <= 1024 with those: never this many queues)
            if (vec4 == VM_SMALL_LUT)
                return rss_toeplitz_kernel<kHPow2, kQMode, kHist, kQWidth, true, false, true>;
        }
        // a small-table request with no small-table instance must not fall back to the 12-bit
        // tables: the launcher sized the dynamic LDS for the small-table span
        if (vec4 == VM_SMALL_LUT) return nullptr;
        return vec4 ? rss_toeplitz_kernel<kHPow2, kQMode, kHist, kQWidth, true>
                    : rss_toeplitz_kernel<kHPow2, kQMode, kHist, kQWidth, false>;
    }
}

// No launch reaches these combinations, so they are not instantiated: more than 7168 queues
// (the many-queues modes, setup_modes) never come with u8 queues (min(H, Q) <= 256) or
// QM_FAST8 (H <= 256, no table), and u8 bins (past 80572 queues) never with QM_FAST16
// (Q < H <= 65536)
template <bool kHPow2, int kQMode, int kHist, int kQWidth>
KernelFn pick_vec(int vec4) {
    constexpr bool kMany = kHist == HIST_GLOBAL || kHist == HIST_RANGE16 || kHist == HIST_RANGE8;
    if constexpr ((kMany && (kQWidth == QW_U8 || kQMode == QM_FAST8)) ||
                  (kHist == HIST_RANGE8 && kQMode == QM_FAST16))
        return nullptr;
    else
        return pick_vec_reachable<kHPow2, kQMode, kHist, kQWidth>(vec4);
}

template <bool kHPow2, int kQMode, int kHist>
KernelFn pick_width(int qwidth, int vec4) {
    switch (qwidth) {
        case QW_U8: return pick_vec<kHPow2, kQMode, kHist, QW_U8>(vec4);
        case QW_U16: return pick_vec<kHPow2, kQMode, kHist, QW_U16>(vec4);
        case QW_U16R: return pick_vec<kHPow2, kQMode, kHist, QW_U16R>(vec4);
        default: return pick_vec<kHPow2, kQMode, kHist, QW_U32>(vec4);
    }
}

template <bool kHPow2, int kQMode>
KernelFn pick_hist(int hist, int qwidth, int vec4) {
    switch (hist) {
        case HIST_PRIVATE: return pick_width<kHPow2, kQMode, HIST_PRIVATE>(qwidth, vec4);
        case HIST_SHARED: return pick_width<kHPow2, kQMode, HIST_SHARED>(qwidth, vec4);
        case HIST_GLOBAL: return pick_width<kHPow2, kQMode, HIST_GLOBAL>(qwidth, vec4);
        case HIST_RANGE16: return pick_width<kHPow2, kQMode, HIST_RANGE16>(qwidth, vec4);
        case HIST_RANGE8: return pick_width<kHPow2, kQMode, HIST_RANGE8>(qwidth, vec4);
        case HIST_NONE: return pick_width<kHPow2, kQMode, HIST_NONE>(qwidth, vec4);
        default: return nullptr;  // HIST_RANGE (u32 ranges): the IPv6 kernel's only
    }
}

template <bool kHPow2>
KernelFn pick_queue(int qmode, int hist, int qwidth, int vec4) {
    switch (qmode) {
        case QM_MASK: return pick_hist<kHPow2, QM_MASK>(hist, qwidth, vec4);
        case QM_FAST16: return pick_hist<kHPow2, QM_FAST16>(hist, qwidth, vec4);
        case QM_FAST8: return pick_hist<kHPow2, QM_FAST8>(hist, qwidth, vec4);
        case QM_TABLE: return pick_hist<kHPow2, QM_TABLE>(hist, qwidth, vec4);
        default: return pick_hist<kHPow2, QM_FAST32>(hist, qwidth, vec4);
    }
}

// ---------------------------------------------------------- path options ----
// A launch takes its path from its arguments and from the scratch memory it gets.  The
// tests force the other paths (the ones a launch takes when memory runs short, and the
// recount of a guarded pass) through a test-hooks build of this file (-DRSS_TEST_HOOKS:
// librss_toeplitz_hooks.so, loaded by tests/ only, rss_test_set_option in rss_test_hooks.h).
// In the product library these are constants: its hashing path reads no environment.
struct Options {
    int recount = 0;          // guarded passes: 1 poisons every pass (the recount takes it), 2 runs
                              // no gate and no recount (counts from the bins and moves alone)
    bool range8 = true;       // u8 bins past the u16 bins' reach (else u16 bins + more passes)
    bool small_lut = true;    // the small tables for many-queues hash passes (else 12-bit tables)
    int prefetch = -1;        // small-table passes' load prefetch: -1 counts only, 0 / 1 forced
    bool balance = true;      // the balanced tail (walk_rows) of single-pass and u8 launches
    bool counts_perm = true;  // the register-table counts-only kernel
    bool resid = true;        // counts only past 161144 queues: residual lists (else a column)
    bool wide = true;         // wide passes over a queue column (else u32 passes of 16384)
    int alloc_fail = 0;       // scratch kinds (AllocKind bits) whose allocation is made to fail
    int fail_launch = 0;      // k > 0: the k-th rss::launch_hash from now returns RSS_EIO
};
#ifdef RSS_TEST_HOOKS
Options g_opt;
#else
constexpr Options g_opt{};
#endif

// Small-table passes without per-tuple outputs (counts only, no scratch column) issue the
// next group's loads before this group's LDS work: 0.62 vs 0.66 ms at Q = 65536 / 131072,
// where with outputs it cost 1-2 % and the balanced tail gains 4 % instead
// (profiles/archive/r04/small_tables/prefetch_ab.jsonl).
bool prefetch_for(bool has_outputs) {
    return g_opt.prefetch >= 0 ? g_opt.prefetch == 1 : !has_outputs;
}

// Counts only, power-of-two H <= 256, 16-B aligned tuples: rss_counts_perm_kernel with the
// byte tables of (window & (H-1)) built here from the key's windows (IPv4: 96, IPv6: 288).
template <int kWords>
int launch_counts_perm(const uint32_t* window, const void* tuples, uint64_t n, unsigned long long* counts,
                       uint32_t h_mask, uint32_t Q, uint32_t q_mask, uint32_t q_m16, int qmode,
                       uint32_t bin_bytes, int cu_count, hipStream_t stream,
                       unsigned long long* ws = nullptr, uint32_t fold_mode = 0) {
    PermParams<kWords> pp;
    memset(&pp, 0, sizeof pp);
    pp.tuples = static_cast<const uint32_t*>(tuples);
    pp.counts = counts;
    pp.ws = ws;
    pp.accumulate = fold_mode;  // kFoldAccumulate
    pp.n = n;
    pp.Q = Q;
    pp.q_mask = q_mask;
    pp.q_m16 = q_m16;
    for (int k = 0; k < kWords; ++k)         // word
        for (int j = 0; j < 4; ++j)          // byte of the word, least significant first
            for (int f = 0; f < 3; ++f) {    // fields [0,3) [3,6) [6,8) of the byte
                const int id = (k * 4 + j) * 3 + f, lsb = 8 * j + 3 * f, len = f < 2 ? 3 : 2;
                uint8_t e[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                for (int v = 0; v < (1 << len); ++v)
                    for (int b = 0; b < len; ++b)  // word k bit i is input bit 32k + 31 - i
                        if ((v >> b) & 1) e[v] ^= (uint8_t)(window[32 * k + 31 - (lsb + b)] & h_mask);
                pp.lo[id] = e[0] | e[1] << 8 | e[2] << 16 | (uint32_t)e[3] << 24;
                pp.hi[id] = e[4] | e[5] << 8 | e[6] << 16 | (uint32_t)e[7] << 24;
            }
    // no LUT and <= 64 VGPRs: two 1024-lane workgroups fit a CU
    const uint64_t want = (n + 4 * kBlock - 1) / (4 * kBlock);
    const unsigned grid = (unsigned)(want < 2ull * cu_count ? want : 2ull * cu_count);
    // no balanced tail here (pp.tail_rows = 0, walk_rows' static loop): on this read-only,
    // two-workgroups-per-CU kernel it measured 5 % SLOWER (0.562 vs 0.536 ms per 2^28
    // tuples, profiles/r03/c/ab.json), where the full-output kernel gains 3 %
    const uint32_t shmem = bin_bytes;
    if (qmode == QM_MASK)
        hipLaunchKernelGGL((rss_counts_perm_kernel<QM_MASK, kWords>), dim3(grid), dim3(kBlock),
                           shmem, stream, pp);
    else
        hipLaunchKernelGGL((rss_counts_perm_kernel<QM_FAST8, kWords>), dim3(grid), dim3(kBlock),
                           shmem, stream, pp);
    RSS_HIP_CHECK(hipGetLastError());
    return RSS_OK;
}

// Whether a many-queues launch counts its queues from the queue column (launch_queue_ranges)
// rather than with one global atomic per tuple: up to 64 wide passes (4M queues).
bool ranged_histogram_ok(uint32_t q_eff) { return (uint64_t)q_eff <= 64ull * kWideSpan; }
// Without the wide passes' scratch, the most narrow passes (16384 queues each) a launch runs
// over a queue column before one global atomic per tuple is cheaper: 64 over u16 columns,
// 32 over u32 ones
uint64_t narrow_passes_max(int qw) { return qw == QW_U32 ? 32 : 64; }
// launch_hash's many-queues attempt: "count with the global-atomic kernel instead" (every
// RSS_* code is <= 0)
constexpr int kTakeAtomics = 1;

// --------------------------------------------------------- guarded passes --
// Scratch block of a guarded pass (u16 / u8 bins with guard moves and a poison word: the
// hash pass's HIST_RANGE16 / HIST_RANGE8, the wide passes over a queue column):
//   the partial matrix (a row of `words` dwords per workgroup, rounded to 16 B)
//   | ovf[q_span] | poison | zero (never written: the ungated reduce's word) | pad
//   | the balanced tail's unit counter (u64)
size_t guard_rows_bytes(unsigned grid, uint32_t words) {
    return ((size_t)grid * words * 4 + 15) & ~(size_t)15;
}
size_t guard_ctr_offset(uint32_t q_span) { return (((size_t)q_span + 2) * 4 + 7) & ~(size_t)7; }
size_t guard_tail_bytes(uint32_t q_span) { return guard_ctr_offset(q_span) + 8; }
uint32_t guard_words(int bits, uint32_t q_span) { return bits == 8 ? (q_span + 3) / 4 : (q_span + 1) / 2; }

// What a scratch block is for (the test hooks' alloc_fail bits name them)
enum AllocKind { AK_ROWS = 1, AK_WIDE = 2, AK_COLUMN = 4, AK_LISTS = 8 };

void* alloc_block(size_t bytes, hipStream_t stream, int kind) {
    if (g_opt.alloc_fail & kind) return nullptr;
    void* buf = nullptr;
    if (hipMallocAsync(&buf, bytes, stream) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return buf;
}
void* alloc_guarded(int bits, unsigned grid, uint32_t q_span, hipStream_t stream) {
    return alloc_block(guard_rows_bytes(grid, guard_words(bits, q_span)) + guard_tail_bytes(q_span),
                       stream, AK_ROWS);
}

// frees `buf` stream-ordered after its readers; the first error wins
int free_block(void* buf, int rc, hipStream_t stream) {
    if (!buf) return rc;
    const hipError_t fe = hipFreeAsync(buf, stream);
    if (fe != hipSuccess && rc == RSS_OK)
        rc = rss_set_error(RSS_EIO, "hipFreeAsync failed: %s", hipGetErrorString(fe));
    return rc;
}

// The tail of a guarded pass's block zeroed (and, under the recount hook, the poison word
// raised); returns the word the reduce is gated on.
hipError_t arm_guard(uint32_t* ovf, uint32_t q_span, const uint32_t** gate, hipStream_t stream) {
    uint32_t* poison = ovf + q_span;
    hipError_t e = hipMemsetAsync(ovf, 0, guard_tail_bytes(q_span), stream);
    if (e == hipSuccess && g_opt.recount == 1) e = hipMemsetD32Async(poison, 1, 1, stream);
    *gate = g_opt.recount == 2 ? poison + 1 : poison;
    return e;
}

template <int kBits>
void launch_reduce(const uint32_t* partial, unsigned rows, uint32_t words, uint32_t q_lo,
                   uint32_t q_span, unsigned long long* counts, const uint32_t* ovf,
                   const uint32_t* gate, hipStream_t stream) {
    hipLaunchKernelGGL(rss_partial_reduce_kernel<kBits>, dim3((words + kReduceCols - 1) / kReduceCols),
                       dim3(kReduceCols * kReduceGroups), 0, stream, partial, rows, words, q_lo,
                       q_span, counts, ovf, gate);
}

// The recount from a column of queues (or, with region_counts, residual lists), gated on
// `poison`; no-op under the "no recount" hook
template <typename T>
void launch_recount_col(const T* col, uint64_t n, uint32_t q_lo, uint32_t q_span,
                        unsigned long long* counts, const uint32_t* poison, unsigned grid,
                        hipStream_t stream, const uint32_t* region_counts = nullptr,
                        uint64_t region_cap = 0) {
    if (g_opt.recount == 2) return;
    hipLaunchKernelGGL(rss_range_fallback_col_kernel<T>, dim3(grid), dim3(kBlock),
                       std::min(kFallbackColSpan, q_span) * 4, stream, col, n, q_lo, q_span, counts,
                       poison, region_counts, region_cap);
}

// ------------------------------------------------------------ wide passes --
// Scratch of the wide passes of one launch: ONE block for all of them (the passes are
// stream-ordered, so each reuses the rows and re-zeroes the tail), allocated before the
// launch's first pass touches the counts -- a launch that cannot get it takes the narrow
// passes (or, for residual lists, the scratch column) with the counts untouched.
struct WideScratch {
    void* buf = nullptr;
    unsigned grid = 0;
    uint32_t row_words = 0;  // one row's dwords: the widest pass the launch runs
    uint32_t* partial() const { return static_cast<uint32_t*>(buf); }
    uint32_t* ovf() const {
        return reinterpret_cast<uint32_t*>(static_cast<char*>(buf) + guard_rows_bytes(grid, row_words));
    }
};
unsigned wide_grid(uint64_t n, int cu_count) {
    const uint64_t want = (n + 8ull * kBlock - 1) / (8ull * kBlock);
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, cu_count));
}
// The scratch of the wide passes over `nranged` queues: rows for u8 bins (kWideSpan8 / 4
// dwords) when launch_queue_ranges will run a u8 pass (more than kWideSpan queues left),
// else for u16 bins (kWideSpan / 2)
WideScratch alloc_wide(unsigned grid, uint32_t nranged, hipStream_t stream) {
    const bool u8 = g_opt.range8 && nranged > kWideSpan;
    const uint32_t span = u8 ? kWideSpan8 : kWideSpan;
    WideScratch s;
    s.grid = grid;
    s.row_words = guard_words(u8 ? 8 : 16, span);
    s.buf = alloc_block(guard_rows_bytes(grid, s.row_words) + guard_tail_bytes(span), stream, AK_WIDE);
    return s;
}
// a wide pass costs about two narrow ones (2^28 tuples: ~0.2 vs ~0.1 ms over a u16 column,
// profiles/r03/d/config_sweep.jsonl), so it pays from three narrow passes on
bool wide_pays(uint32_t nranged) {
    return g_opt.wide && ((uint64_t)nranged + kNarrowSpan - 1) / kNarrowSpan >= 3;
}

// One guarded wide pass over [lo, lo + sp) of a queue column (rss_queue_hist_wide_kernel):
// the pass, the reduce (gated on !poison) and the column recount (gated on poison).
template <typename T, int kBits>
hipError_t wide_pass(const T* qcol, uint64_t n, uint32_t lo, uint32_t sp, unsigned long long* counts,
                     const WideScratch& sc, int cu_count, hipStream_t stream,
                     const uint32_t* region_counts, uint64_t region_cap) {
    const uint32_t words = guard_words(kBits, sp);
    uint32_t* ovf = sc.ovf();
    const uint32_t* gate = nullptr;
    hipError_t e = arm_guard(ovf, sp, &gate, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((rss_queue_hist_wide_kernel<T, kBits>), dim3(sc.grid), dim3(kBlock), words * 4,
                       stream, qcol, n, lo, sp, sc.partial(), words, ovf, ovf + sp, region_counts,
                       region_cap);
    launch_reduce<kBits>(sc.partial(), sc.grid, words, lo, sp, counts, ovf, gate, stream);
    launch_recount_col(qcol, n, lo, sp, counts, ovf + sp, region_counts ? sc.grid : (unsigned)cu_count,
                       stream, region_counts, region_cap);
    return hipGetLastError();
}

// Queue ranges [first, nqueues) of a many-queues launch, histogrammed from the queue column
// (u16 or u32) the first pass wrote.  With a wide scratch block: one wide pass per 163840
// queues in u8 bins while more than 65536 are left, then one in u16 bins -- 2.5 times the
// queues per read of the column.  Without: one rss_queue_hist_kernel pass (u32 bins, no
// guard) per 16384 queues.  Regions (region_counts != NULL, wide only): the "column" is one
// residual list per hash-pass wave (resid_append), 16 per workgroup of wsc->grid, read one
// wave per list.
int launch_queue_ranges(const void* qcol, int qw, uint64_t n, uint32_t first, uint32_t nqueues,
                        unsigned long long* counts, int cu_count, hipStream_t stream,
                        const WideScratch* wsc, const uint32_t* region_counts = nullptr,
                        uint64_t region_cap = 0) {
    if (first >= nqueues) return RSS_OK;
    if (wsc && wsc->buf) {
        const uint16_t* c16 = static_cast<const uint16_t*>(qcol);
        const uint32_t* c32 = static_cast<const uint32_t*>(qcol);
        for (uint32_t lo = first; lo < nqueues;) {
            hipError_t e;
            uint32_t sp;
            if (g_opt.range8 && nqueues - lo > kWideSpan) {
                sp = std::min<uint32_t>(kWideSpan8, nqueues - lo);
                e = qw == QW_U16 ? wide_pass<uint16_t, 8>(c16, n, lo, sp, counts, *wsc, cu_count, stream,
                                                          region_counts, region_cap)
                                 : wide_pass<uint32_t, 8>(c32, n, lo, sp, counts, *wsc, cu_count, stream,
                                                          region_counts, region_cap);
            } else {
                sp = std::min<uint32_t>(kWideSpan, nqueues - lo);
                e = qw == QW_U16 ? wide_pass<uint16_t, 16>(c16, n, lo, sp, counts, *wsc, cu_count, stream,
                                                           region_counts, region_cap)
                                 : wide_pass<uint32_t, 16>(c32, n, lo, sp, counts, *wsc, cu_count, stream,
                                                           region_counts, region_cap);
            }
            if (e != hipSuccess)
                return rss_set_error(RSS_EIO, "wide queue histogram launch failed: %s", hipGetErrorString(e));
            lo += sp;
        }
        return RSS_OK;
    }
    if (region_counts)
        return rss_set_error(RSS_EIO, "rss_hash_device: residual lists without the wide passes' scratch");
    const uint32_t span = kNarrowSpan;
    const uint64_t qwant = (n + 8ull * kBlock - 1) / (8ull * kBlock);
    const unsigned qgrid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(qwant, (uint64_t)cu_count * 2));
    for (uint32_t lo = first; lo < nqueues; lo += span) {
        const uint32_t sp = std::min<uint32_t>(span, nqueues - lo);
        if (qw == QW_U16)
            hipLaunchKernelGGL(rss_queue_hist_kernel<uint16_t>, dim3(qgrid), dim3(kBlock), sp * 4,
                               stream, static_cast<const uint16_t*>(qcol), n, lo, sp, counts);
        else
            hipLaunchKernelGGL(rss_queue_hist_kernel<uint32_t>, dim3(qgrid), dim3(kBlock), sp * 4,
                               stream, static_cast<const uint32_t*>(qcol), n, lo, sp, counts);
        RSS_HIP_CHECK(hipGetLastError());
    }
    return RSS_OK;
}

// ------------------------------------------------------ guarded hash pass --
using FallbackFn = void (*)(const LaunchParams);
template <bool kHPow2>
FallbackFn pick_fallback_q(int qmode) {
    switch (qmode) {
        case QM_MASK: return rss_range_fallback_kernel<kHPow2, QM_MASK>;
        case QM_FAST16: return rss_range_fallback_kernel<kHPow2, QM_FAST16>;
        case QM_FAST32: return rss_range_fallback_kernel<kHPow2, QM_FAST32>;
        case QM_TABLE: return rss_range_fallback_kernel<kHPow2, QM_TABLE>;
        default: return nullptr;  // (QM_FAST8: H <= 256 and no table, never this many queues)
    }
}
FallbackFn pick_fallback(bool h_pow2, int qmode) {
    return h_pow2 ? pick_fallback_q<true>(qmode) : pick_fallback_q<false>(qmode);
}

// A guarded hash pass (HIST_RANGE16 when bits = 16, HIST_RANGE8 when 8) over [p.q_lo, p.q_lo
// + p.q_span) on the block `buf` (alloc_guarded, freed here on every path): the tail zeroed,
// the pass (a row of bins per workgroup, guard moves, poison), the reduce (gated on
// !poison) and the recount (gated on poison) -- from `qcol` when the launch writes a column
// holding the queues themselves (QW_U32 / QW_U16 `qw`), else by rehashing the tuples.
int launch_guarded(KernelFn fn, FallbackFn fallback, int bits, unsigned grid, int cu_count,
                   uint32_t shmem, LaunchParams& p, const void* qcol, int qw, void* buf,
                   uint32_t reta_bytes, hipStream_t stream) {
    const bool col = qcol && (qw == QW_U32 || qw == QW_U16);
    if (!fn || (!col && !fallback)) {
        (void)hipFreeAsync(buf, stream);
        return rss_set_error(RSS_EIO, "rss_hash_device: no kernel instance for this launch");
    }
    const uint32_t words = guard_words(bits, p.q_span);
    uint32_t* tail = reinterpret_cast<uint32_t*>(static_cast<char*>(buf) + guard_rows_bytes(grid, words));
    p.partial = static_cast<uint32_t*>(buf);
    p.partial_stride = words;
    p.ovf = tail;
    p.poison = tail + p.q_span;
    // balanced tail (walk_rows, u8 passes on the small tables): its unit counter in the zeroed
    // tail, its LDS slot past the small tables; the last tenth of the rows goes out per
    // workgroup slot
    const uint32_t tail_rows = balanced_tail_rows(p.n / 4, grid);
    if (bits == 8 && tail_rows && g_opt.balance && !p.prefetch && !p.resid_out) {  // (lists: static walk)
        p.tail_rows = tail_rows;
        p.tail_ctr = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(tail) +
                                                           guard_ctr_offset(p.q_span));
    }
    const uint32_t* gate = nullptr;
    hipError_t e = arm_guard(tail, p.q_span, &gate, stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), shmem, stream, p);
        if (bits == 8)
            launch_reduce<8>(p.partial, grid, words, p.q_lo, p.q_span, p.counts, p.ovf, gate, stream);
        else
            launch_reduce<16>(p.partial, grid, words, p.q_lo, p.q_span, p.counts, p.ovf, gate, stream);
        if (col && qw == QW_U32)
            launch_recount_col(static_cast<const uint32_t*>(qcol), p.n, p.q_lo, p.q_span, p.counts,
                               p.poison, (unsigned)cu_count, stream);
        else if (col)
            launch_recount_col(static_cast<const uint16_t*>(qcol), p.n, p.q_lo, p.q_span, p.counts,
                               p.poison, (unsigned)cu_count, stream);
        else if (g_opt.recount != 2) {
            p.fb_span = std::min<uint32_t>(p.q_span, (kLdsBytes - kSmallLutBytes - reta_bytes) / 4);
            hipLaunchKernelGGL(fallback, dim3(cu_count), dim3(kBlock), p.fb_span * 4 + reta_bytes,
                               stream, p);
        }
        e = hipGetLastError();
    }
    int rc = e == hipSuccess ? RSS_OK
                             : rss_set_error(RSS_EIO, "rss_hash_device: launch failed: %s", hipGetErrorString(e));
    rc = free_block(buf, rc, stream);
    p.partial = nullptr;
    p.ovf = p.poison = nullptr;
    p.tail_ctr = nullptr;
    p.tail_rows = 0;
    return rc;
}

// ws: rss_hash_device_ws's single-pass counts workspace, or NULL (counts zeroed by a
// hipMemsetAsync unless RSS_FLAG_ACCUMULATE).  Used when the launch histograms in LDS bins
// (private or shared); the many-queues range passes ignore it and zero the counts as before.
int launch_hash(const rss_key* key, const rss_tuple4* d_tuples, size_t n, uint32_t htable,
                uint32_t nqueues, uint32_t* d_hash, void* d_queue, uint64_t* d_counts,
                uint32_t flags, hipStream_t stream, const uint32_t* reta = nullptr,
                uint64_t* ws = nullptr) {
    if (!key) return rss_set_error(RSS_EINVAL, "rss_hash_device: key is NULL");
    if (key->len < RSS_KEY_MIN_BYTES)
        return rss_set_error(RSS_EINVAL, "rss_hash_device: key not prepared (len=%u)", key->len);
    if (htable < 1 || nqueues < 1)
        return rss_set_error(RSS_EINVAL, "rss_hash_device: htable (%u) and nqueues (%u) must be >= 1",
                             htable, nqueues);
    if (n && !d_tuples) return rss_set_error(RSS_EINVAL, "rss_hash_device: tuples is NULL");
    if (reta) {
        const int rc = check_reta(reta, htable, nqueues, "rss_hash_device_reta");
        if (rc) return rc;
    }
    // every queue is < q_eff = min(H, Q) (or max(reta) + 1): bins and widths by q_eff
    const uint32_t q_eff = effective_queues(htable, nqueues, reta);
    int qwidth = QW_U32;
    if (flags & RSS_FLAG_QUEUE_U8) {
        if (q_eff > 256)
            return rss_set_error(RSS_EINVAL, "rss_hash_device: RSS_FLAG_QUEUE_U8 needs min(htable, nqueues) <= 256 "
                                         "(got %u)", q_eff);
        qwidth = QW_U8;
    } else if (flags & RSS_FLAG_QUEUE_U16) {
        if (q_eff > 65536)
            return rss_set_error(RSS_EINVAL, "rss_hash_device: RSS_FLAG_QUEUE_U16 needs min(htable, nqueues) <= 65536 "
                                         "(got %u)", q_eff);
        qwidth = QW_U16;
    }
    LaunchParams p;
    memset(&p, 0, sizeof p);
    int qmode, hist;
    uint32_t bin_bytes;
    const uint32_t reta_bytes = reta ? htable * 4 : 0;
    const bool h_pow2 = setup_modes(&p, htable, q_eff, d_counts != nullptr, &qmode, &hist,
                                    &bin_bytes, kBinBytesMax - reta_bytes);
    // single pass: the kernel's last workgroup writes the counts (fold_counts)
    const bool single_pass = ws && d_counts && n > 0 && (hist == HIST_PRIVATE || hist == HIST_SHARED);
    if (d_counts && !(flags & RSS_FLAG_ACCUMULATE) && !single_pass)
        RSS_HIP_CHECK(hipMemsetAsync(d_counts, 0, sizeof(uint64_t) * nqueues, stream));
    else if (single_pass) {
        const int trc = zero_counts_tail(d_counts, q_eff, nqueues, flags, stream);
        if (trc) return trc;
    }
    if (n == 0) return RSS_OK;

    memcpy(p.window, key->window, sizeof p.window);
    p.tuples = d_tuples;
    p.hash_out = d_hash;
    p.queue_out = d_queue;
    p.prefetch = prefetch_for(d_hash || d_queue);

    p.counts = reinterpret_cast<unsigned long long*>(d_counts);
    p.n = n;
    if (single_pass) {
        p.ws = reinterpret_cast<unsigned long long*>(ws);
        p.accumulate = (flags & RSS_FLAG_ACCUMULATE) ? kFoldAccumulate : 0u;
    }
    if (reta) {
        qmode = QM_TABLE;
        for (uint32_t b = 0; b < htable; ++b) p.reta[b] = (uint16_t)reta[b];
    }
    // the 4-tuples-per-lane body needs 16-B aligned tuples / hashes and a queue
    // pointer aligned to the 4 queues it stores at once
    const uintptr_t qalign = qwidth == QW_U8 ? 4 : (qwidth == QW_U16 ? 8 : 16);
    const bool vec4 = aligned16(d_tuples) && (!d_hash || aligned16(d_hash)) &&
                      (!d_queue || ((uintptr_t)d_queue % qalign) == 0);
    DeviceInfo info;
    int rc = device_info(&info);
    if (rc) return rc;
    if (!d_hash && !d_queue && d_counts && !reta && h_pow2 && htable <= 256u &&
        hist == HIST_PRIVATE && (qmode == QM_MASK || qmode == QM_FAST8) && aligned16(d_tuples) &&
        g_opt.counts_perm)
        return launch_counts_perm<3>(key->window, d_tuples, n, p.counts, p.h_mask, p.Q, p.q_mask,
                                     p.q_m16, qmode, bin_bytes, info.cu_count, stream, p.ws,
                                     p.accumulate);
    const uint64_t per_lane = vec4 ? 4 : 1;
    const uint64_t want = (n + per_lane * kBlock - 1) / (per_lane * kBlock);
    const uint64_t cap = (uint64_t)info.cu_count * kBlocksPerCU;
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    // many queues: the guarded passes, or kTakeAtomics when the launch counts with one
    // global atomic per tuple instead (no scratch memory for them, or a column would need
    // more narrow passes than the atomics cost)
    if (hist == HIST_GLOBAL && d_counts) {
        const int mq = [&]() -> int {
            // More queues than u32 LDS bins (DESIGN.md §3 "Many queues").  Guarded u16 bins
            // (HIST_RANGE16): twice the queues of u32 bins in the LDS the tables leave -- 16384
            // beside the 12-bit tables and, on the small tables (4-tuple body, no indirection
            // table), up to 80572 in one pass.  Up to 16384 the 12-bit tables stay: 8 lookups and
            // 3 VALU per lookup fewer than the small tables' 21 when the bins fit beside them.
            const uint32_t span12 = ((kBinBytesMax - reta_bytes) / 4) * 2;
            const bool small_lut = q_eff > span12 && vec4 && !reta && qwidth != QW_U8 && g_opt.small_lut;
            const uint32_t lut_bytes = small_lut ? kSmallStaticBytes : kLutBytes;
            const uint32_t span = ((kLdsBytes - lut_bytes - reta_bytes) / 4) * 2;
            const int vm = small_lut ? VM_SMALL_LUT : (vec4 ? VM_VEC4 : VM_SCALAR);
            const uint32_t qbytes = q_eff <= 65536u ? 2 : 4;
            FallbackFn fb = pick_fallback(h_pow2, qmode);
            if (q_eff <= span) {
                p.q_lo = 0;
                p.q_span = q_eff;
                KernelFn fn = h_pow2 ? pick_queue<true>(qmode, HIST_RANGE16, qwidth, vm)
                                     : pick_queue<false>(qmode, HIST_RANGE16, qwidth, vm);
                void* buf = alloc_guarded(16, grid, q_eff, stream);
                if (!buf) return kTakeAtomics;  // no memory for the u16 bins' rows
                return launch_guarded(fn, fb, 16, grid, info.cu_count, ((q_eff + 1) / 2) * 4 + reta_bytes, p,
                                      d_queue, qwidth, buf, reta_bytes, stream);
            }
            // Past the u16 bins' reach: guarded u8 bins (HIST_RANGE8) hold span8 = 161144 queues
            // beside the small tables -- one pass up to there, and the first range of a
            // queue-column launch beyond.
            const uint32_t span8 = kLdsBytes - kSmallStaticBytes;
            void* r8buf = nullptr;  // the u8 pass's scratch block, when it runs
            if (small_lut && g_opt.range8 && fb)
                r8buf = alloc_guarded(8, grid, std::min(q_eff, span8), stream);
            if (r8buf && q_eff <= span8) {
                p.q_lo = 0;
                p.q_span = q_eff;
                KernelFn fn = h_pow2 ? pick_queue<true>(qmode, HIST_RANGE8, qwidth, VM_SMALL_LUT)
                                     : pick_queue<false>(qmode, HIST_RANGE8, qwidth, VM_SMALL_LUT);
                return launch_guarded(fn, fb, 8, grid, info.cu_count, guard_words(8, q_eff) * 4, p, d_queue,
                                      qwidth, r8buf, 0, stream);
            }
            // Counts only past span8 (u8 hash pass + wide passes): the queues past the pass's LDS
            // range go to per-wave residual lists (resid_append) instead of a queue column --
            // only those tuples' queues are written and read again, not every tuple's.
            if (r8buf && !d_queue && q_eff > span8 && g_opt.resid) {
                // the static walk gives a wave at most `rows` groups of 4 tuples per lane, plus the
                // < 4 tail tuples (wave 0 of workgroup 0); 8 entries more keep every list 16-B aligned
                const uint64_t per_row = (uint64_t)grid * kBlock;
                const uint64_t rows = (n / 4 + per_row - 1) / per_row;
                const uint64_t lcap = (rows * 4 * 64 + 4 + 7) & ~7ull;
                const uint32_t nres = q_eff - span8;
                const size_t esize = nres <= 65536u ? 2 : 4;
                const size_t nlists = (size_t)grid * kWavesPerBlock;
                const size_t list_bytes = nlists * lcap * esize;
                void* lists = alloc_block(list_bytes + nlists * 4, stream, AK_LISTS);
                WideScratch wsc = lists ? alloc_wide(grid, nres, stream) : WideScratch{};
                if (lists && wsc.buf) {
                    uint32_t* list_counts = reinterpret_cast<uint32_t*>(static_cast<char*>(lists) + list_bytes);
                    p.queue_out = nullptr;
                    p.resid_out = lists;
                    p.resid_counts = list_counts;
                    p.resid_cap = lcap;
                    p.resid_u16 = esize == 2;
                    p.prefetch = prefetch_for(false);
                    p.q_lo = 0;
                    p.q_span = span8;
                    KernelFn fn = h_pow2 ? pick_queue<true>(qmode, HIST_RANGE8, QW_U32, VM_SMALL_LUT)
                                         : pick_queue<false>(qmode, HIST_RANGE8, QW_U32, VM_SMALL_LUT);
                    rc = launch_guarded(fn, fb, 8, grid, info.cu_count, guard_words(8, span8) * 4, p, nullptr,
                                        QW_U32, r8buf, 0, stream);
                    p.resid_out = nullptr;
                    if (rc == RSS_OK)
                        rc = launch_queue_ranges(lists, esize == 2 ? QW_U16 : QW_U32, n, 0, nres,
                                                 p.counts + span8, info.cu_count, stream, &wsc, list_counts,
                                                 lcap);
                    rc = free_block(wsc.buf, rc, stream);
                    return free_block(lists, rc, stream);
                }
                (void)free_block(wsc.buf, RSS_OK, stream);  // no room for the lists: the scratch
                (void)free_block(lists, RSS_OK, stream);    // column below
            }
            if (ranged_histogram_ok(q_eff)) {
                void* qcol = d_queue;
                int qw = qwidth;
                bool scratch = false, ranged = true;
                // counts only past the small tables' range: a u16 column of q - span (QW_U16R) when
                // the rest of the queues fit 16 bits, else the queues themselves
                const uint32_t first_span = r8buf ? span8 : span;
                const bool resid = !d_queue && small_lut && q_eff - first_span <= 0xFFFFu;
                const uint32_t sbytes = resid ? 2 : qbytes;
                if (!qcol || qwidth == QW_U8) {  // (u8 queues always fit the bins: q_eff <= 256)
                    qcol = alloc_block((size_t)n * sbytes, stream, AK_COLUMN);
                    if (qcol) {
                        scratch = true;
                        qw = resid ? QW_U16R : (qbytes == 2 ? QW_U16 : QW_U32);
                    } else {
                        ranged = false;  // no room for a scratch column: one global atomic per tuple
                    }
                }
                if (ranged) {
                    p.queue_out = qcol;
                    p.prefetch = prefetch_for(true);  // the pass writes a column
                    p.q_lo = 0;
                    const bool v4 = vec4 && ((uintptr_t)qcol % (qw == QW_U32 ? 16 : 8)) == 0;
                    // the first range: the bins the first pass's tables leave (small tables: 4-tuple
                    // body only; the caller's queue buffer may not be aligned for it)
                    const bool b1 = small_lut && v4 && qw != QW_U8;
                    const bool r8 = b1 && r8buf;  // (a caller's u32 column: b1 == small_lut)
                    if (!r8 && r8buf) {
                        (void)free_block(r8buf, RSS_OK, stream);
                        r8buf = nullptr;
                    }
                    const uint32_t span1 = b1 ? (r8 ? span8 : span) : span12;
                    p.q_span = span1;  // < q_eff here
                    const int vm1 = b1 ? VM_SMALL_LUT : (v4 ? VM_VEC4 : VM_SCALAR);
                    const int bits1 = r8 ? 8 : 16;
                    KernelFn fn = h_pow2 ? pick_queue<true>(qmode, r8 ? HIST_RANGE8 : HIST_RANGE16, qw, vm1)
                                         : pick_queue<false>(qmode, r8 ? HIST_RANGE8 : HIST_RANGE16, qw, vm1);
                    const unsigned g1 = v4 ? grid : (unsigned)std::min<uint64_t>((n + kBlock - 1) / kBlock, cap);
                    // every scratch block before the first pass touches the counts
                    void* buf1 = r8 ? r8buf : alloc_guarded(16, g1, span1, stream);
                    r8buf = nullptr;
                    const uint32_t nranged = q_eff - span1;
                    WideScratch wsc = buf1 && wide_pays(nranged)
                                          ? alloc_wide(wide_grid(n, info.cu_count), nranged, stream)
                                          : WideScratch{};
                    // no rows for the first range, or no wide scratch and more narrow passes
                    // over the column than one atomic per tuple costs: the atomics (the counts
                    // are untouched so far)
                    const uint64_t narrow = ((uint64_t)nranged + kNarrowSpan - 1) / kNarrowSpan;
                    if (!buf1 || (!wsc.buf && narrow > narrow_passes_max(qw))) {
                        (void)free_block(buf1, RSS_OK, stream);
                        (void)free_block(wsc.buf, RSS_OK, stream);
                        (void)free_block(scratch ? qcol : nullptr, RSS_OK, stream);
                        return kTakeAtomics;
                    }
                    const uint32_t shmem1 = guard_words(bits1, span1) * 4 + (bits1 == 16 ? reta_bytes : 0);
                    rc = launch_guarded(fn, fb, bits1, g1, info.cu_count, shmem1, p, qcol, qw, buf1,
                                        reta_bytes, stream);
                    if (rc == RSS_OK && qw == QW_U16R)  // queues [span1, q_eff) as [0, q_eff - span1)
                        rc = launch_queue_ranges(qcol, QW_U16, n, 0, nranged, p.counts + span1,
                                                 info.cu_count, stream, &wsc);
                    else if (rc == RSS_OK)
                        rc = launch_queue_ranges(qcol, qw, n, span1, q_eff, p.counts, info.cu_count,
                                                 stream, &wsc);
                    rc = free_block(wsc.buf, rc, stream);
                    // the scratch column goes back on every path (stream-ordered after its readers)
                    return free_block(scratch ? qcol : nullptr, rc, stream);
                }
            }
            (void)free_block(r8buf, RSS_OK, stream);  // unused: global atomics below
            return kTakeAtomics;
        }();
        if (mq != kTakeAtomics) return mq;
        p.queue_out = d_queue;  // (a ranged attempt may have pointed them elsewhere)
        p.prefetch = prefetch_for(d_hash || d_queue);
        p.q_lo = p.q_span = 0;
    }
    // 32-bit byte offsets when every stream's bytes fit them (input 12 n B is the largest)
    const int vmode = vec4 ? (12ull * n < (1ull << 32) && !(flags & RSS_FLAG_ADDR64) ? 2 : 1) : 0;
    KernelFn fn = h_pow2 ? pick_queue<true>(qmode, hist, qwidth, vmode)
                         : pick_queue<false>(qmode, hist, qwidth, vmode);
    if (!fn) return rss_set_error(RSS_EIO, "rss_hash_device: no kernel instance for this launch");
    uint32_t shmem = bin_bytes + reta_bytes;  // dynamic part; the 128 KiB LUT is static
    // Balanced tail (single-pass launches: the workspace holds its unit counter and is used
    // by one launch at a time): the last ~1/10 of the grid-stride rows handed out per
    // workgroup slot, so the XCDs finish together.  Needs 8 bytes of LDS beside the bins.
    const uint32_t bal_off = (shmem + 7u) & ~7u;
    const uint32_t tail = balanced_tail_rows(n / 4, grid);
    if (single_pass && vec4 && tail && bal_off + 8 <= kBinBytesMax && g_opt.balance) {
        p.tail_rows = tail;
        p.bal_off = bal_off;
        shmem = bal_off + 8;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), shmem, stream, p);
    RSS_HIP_CHECK(hipGetLastError());
    return RSS_OK;
}

using KernelFn6 = void (*)(const LaunchParams6);

template <bool kHPow2, int kQMode, int kHist>
KernelFn6 pick6_vec(bool vec4) {
    if constexpr (kQMode == QM_FAST8 && (kHist == HIST_GLOBAL || kHist == HIST_RANGE))
        return nullptr;  // (H <= 256: never more queues than the LDS bins hold)
    else
        return vec4 ? rss_toeplitz6_kernel<kHPow2, kQMode, kHist, true>
                    : rss_toeplitz6_kernel<kHPow2, kQMode, kHist, false>;
}

template <bool kHPow2, int kQMode>
KernelFn6 pick6_hist(int hist, bool vec4) {
    switch (hist) {
        case HIST_PRIVATE: return pick6_vec<kHPow2, kQMode, HIST_PRIVATE>(vec4);
        case HIST_SHARED: return pick6_vec<kHPow2, kQMode, HIST_SHARED>(vec4);
        case HIST_GLOBAL: return pick6_vec<kHPow2, kQMode, HIST_GLOBAL>(vec4);
        case HIST_RANGE: return pick6_vec<kHPow2, kQMode, HIST_RANGE>(vec4);
        default: return pick6_vec<kHPow2, kQMode, HIST_NONE>(vec4);
    }
}

template <bool kHPow2>
KernelFn6 pick6(int qmode, int hist, bool vec4) {
    switch (qmode) {
        case QM_MASK: return pick6_hist<kHPow2, QM_MASK>(hist, vec4);
        case QM_FAST16: return pick6_hist<kHPow2, QM_FAST16>(hist, vec4);
        case QM_FAST8: return pick6_hist<kHPow2, QM_FAST8>(hist, vec4);
        case QM_TABLE: return pick6_hist<kHPow2, QM_TABLE>(hist, vec4);
        default: return pick6_hist<kHPow2, QM_FAST32>(hist, vec4);
    }
}

int launch_hash6(const rss_key6* key, const rss_tuple6* d_tuples, size_t n, uint32_t htable,
                 uint32_t nqueues, uint32_t* d_hash, void* d_queue, uint64_t* d_counts,
                 uint32_t flags, hipStream_t stream, const uint32_t* reta = nullptr,
                 uint64_t* ws = nullptr) {
    if (!key || key->len < RSS_KEY_MIN_BYTES)
        return rss_set_error(RSS_EINVAL, "rss_hash6_device: key NULL or not prepared");
    if (htable < 1 || nqueues < 1)
        return rss_set_error(RSS_EINVAL, "rss_hash6_device: htable (%u) and nqueues (%u) must be >= 1",
                             htable, nqueues);
    if (n && !d_tuples) return rss_set_error(RSS_EINVAL, "rss_hash6_device: tuples is NULL");
    if (reta) {
        const int rc = check_reta(reta, htable, nqueues, "rss_hash6_device_reta");
        if (rc) return rc;
    }
    const uint32_t q_eff = effective_queues(htable, nqueues, reta);  // as launch_hash
    uint32_t qwidth = QW_U32;
    if (flags & RSS_FLAG_QUEUE_U8) {
        if (q_eff > 256)
            return rss_set_error(RSS_EINVAL, "rss_hash6_device: RSS_FLAG_QUEUE_U8 needs min(htable, nqueues) <= 256 "
                                         "(got %u)", q_eff);
        qwidth = QW_U8;
    } else if (flags & RSS_FLAG_QUEUE_U16) {
        if (q_eff > 65536)
            return rss_set_error(RSS_EINVAL, "rss_hash6_device: RSS_FLAG_QUEUE_U16 needs min(htable, nqueues) <= 65536 "
                                         "(got %u)", q_eff);
        qwidth = QW_U16;
    }
    LaunchParams tmp;  // reuse the IPv4 mode selection
    memset(&tmp, 0, sizeof tmp);
    int qmode, hist;
    uint32_t bin_bytes;
    const uint32_t reta_bytes = reta ? htable * 4 : 0;  // the table in LDS after the bins
    const uint32_t budget = kBinBytesMax6 - reta_bytes;   // bins share the LDS with the LUT
    const bool h_pow2 = setup_modes(&tmp, htable, q_eff, d_counts != nullptr, &qmode, &hist,
                                    &bin_bytes, budget);
    if (reta) qmode = QM_TABLE;
    // single pass (rss_hash6_device_ws): the kernel's last workgroup writes the counts, as
    // launch_hash; otherwise zero them first unless accumulating
    const bool single_pass = ws && d_counts && n > 0 && (hist == HIST_PRIVATE || hist == HIST_SHARED);
    if (d_counts && !(flags & RSS_FLAG_ACCUMULATE) && !single_pass)
        RSS_HIP_CHECK(hipMemsetAsync(d_counts, 0, sizeof(uint64_t) * nqueues, stream));
    else if (single_pass) {
        const int trc = zero_counts_tail(d_counts, q_eff, nqueues, flags, stream);
        if (trc) return trc;
    }
    if (n == 0) return RSS_OK;
    LaunchParams6 p;
    memset(&p, 0, sizeof p);
    memcpy(p.window, key->window, sizeof p.window);
    p.tuples = d_tuples;
    p.hash_out = d_hash;
    p.queue_out = d_queue;
    p.counts = reinterpret_cast<unsigned long long*>(d_counts);
    p.n = n;
    p.h_m64 = tmp.h_m64;
    p.h_mask = tmp.h_mask;
    p.H = tmp.H;
    p.Q = tmp.Q;
    p.q_mask = tmp.q_mask;
    p.q_m32 = tmp.q_m32;
    p.q_m16 = tmp.q_m16;
    p.q_m64 = tmp.q_m64;
    p.qwidth = qwidth;
    if (single_pass) {
        p.ws = reinterpret_cast<unsigned long long*>(ws);
        p.accumulate = (flags & RSS_FLAG_ACCUMULATE) ? kFoldAccumulate : 0u;
    }
    if (reta)
        for (uint32_t b = 0; b < htable; ++b) p.reta[b] = (uint16_t)reta[b];
    const uintptr_t qalign = qwidth == QW_U8 ? 4 : (qwidth == QW_U16 ? 8 : 16);
    const bool vec4 = aligned16(d_tuples) && (!d_hash || aligned16(d_hash)) &&
                      (!d_queue || ((uintptr_t)d_queue % qalign) == 0);
    DeviceInfo info;
    int rc = device_info(&info);
    if (rc) return rc;
    // counts only, power-of-two H <= 256: the register-table kernel (no LUT, so private bins
    // up to Q = 256 fit beside it)
    if (!d_hash && !d_queue && d_counts && !reta && h_pow2 && htable <= 256u && q_eff <= 256u &&
        (qmode == QM_MASK || qmode == QM_FAST8) && aligned16(d_tuples) && g_opt.counts_perm)
        return launch_counts_perm<9>(key->window, d_tuples, n, p.counts, p.h_mask, p.Q, p.q_mask,
                                     p.q_m16, qmode, q_eff * kBinCols * 4, info.cu_count, stream,
                                     p.ws, p.accumulate);
    const uint64_t per_lane = vec4 ? 4 : 1;
    const uint64_t want = (n + per_lane * kBlock - 1) / (per_lane * kBlock);
    const uint64_t cap = (uint64_t)info.cu_count * kBlocksPerCU6;
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    // many queues: as launch_hash (first range in LDS + the queue column, then the column)
    if (hist == HIST_GLOBAL && d_counts) {
        const uint32_t span = budget / 4;
        const uint32_t qbytes = q_eff <= 65536u ? 2 : 4;
        if (ranged_histogram_ok(q_eff)) {
            void* qcol = d_queue;
            bool scratch = false, ranged = true;
            if (!qcol || qwidth == QW_U8) {
                qcol = alloc_block((size_t)n * qbytes, stream, AK_COLUMN);
                if (qcol) {
                    scratch = true;
                    p.qwidth = qbytes == 2 ? QW_U16 : QW_U32;
                } else {
                    ranged = false;  // as launch_hash: global atomics below instead
                }
            }
            if (ranged) {
                p.queue_out = qcol;
                p.q_lo = 0;
                p.q_span = std::min<uint32_t>(span, q_eff);
                const uint32_t qw = p.qwidth;
                const bool v4 = vec4 && ((uintptr_t)qcol % (qw == QW_U32 ? 16 : 8)) == 0;
                KernelFn6 fn = h_pow2 ? pick6<true>(qmode, HIST_RANGE, v4) : pick6<false>(qmode, HIST_RANGE, v4);
                const unsigned g1 = v4 ? grid : (unsigned)std::min<uint64_t>((n + kBlock - 1) / kBlock, cap);
                // the wide passes' scratch before the first pass touches the counts; without
                // it, more narrow passes than the atomics cost take the atomics (as launch_hash)
                const uint32_t nranged = q_eff - p.q_span;
                WideScratch wsc = wide_pays(nranged) ? alloc_wide(wide_grid(n, info.cu_count), nranged, stream)
                                                     : WideScratch{};
                const uint64_t narrow = ((uint64_t)nranged + kNarrowSpan - 1) / kNarrowSpan;
                if (!wsc.buf && narrow > narrow_passes_max((int)qw)) {
                    (void)free_block(scratch ? qcol : nullptr, RSS_OK, stream);
                    p.queue_out = d_queue;
                    p.qwidth = qwidth;
                    p.q_lo = p.q_span = 0;
                } else {
                    hipLaunchKernelGGL(fn, dim3(g1), dim3(kBlock), span * 4 + reta_bytes, stream, p);
                    const hipError_t le = hipGetLastError();
                    rc = le == hipSuccess
                             ? launch_queue_ranges(qcol, (int)qw, n, span, q_eff, p.counts, info.cu_count, stream,
                                                   &wsc)
                             : rss_set_error(RSS_EIO, "rss_hash6_device: range launch failed: %s",
                                             hipGetErrorString(le));
                    rc = free_block(wsc.buf, rc, stream);
                    return free_block(scratch ? qcol : nullptr, rc, stream);
                }
            }
        }
    }
    KernelFn6 fn = h_pow2 ? pick6<true>(qmode, hist, vec4) : pick6<false>(qmode, hist, vec4);
    uint32_t shmem = bin_bytes + reta_bytes;
    // the balanced tail of single-pass launches (as launch_hash: 8 bytes of LDS beside the bins)
    const uint32_t bal_off = (shmem + 7u) & ~7u;
    const uint32_t tail = balanced_tail_rows(n / 4, grid);
    if (single_pass && vec4 && tail && bal_off + 8 <= kBinBytesMax6 && g_opt.balance) {
        p.tail_rows = tail;
        p.bal_off = bal_off;
        shmem = bal_off + 8;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), shmem, stream, p);
    RSS_HIP_CHECK(hipGetLastError());
    return RSS_OK;
}

}  // namespace

// ---------------------------------------------------- launchers (rss_engine.h) --
// What the C ABI (rss_host.hip) calls; the launch logic above stays internal to this file.
namespace rss {

int launch_hash(const rss_key* key, const rss_tuple4* d_tuples, size_t n, uint32_t htable,
                uint32_t nqueues, uint32_t* d_hash, void* d_queue, uint64_t* d_counts,
                uint32_t flags, hipStream_t stream, const uint32_t* reta, uint64_t* ws) {
#ifdef RSS_TEST_HOOKS
    if (g_opt.fail_launch > 0 && --g_opt.fail_launch == 0)
        return rss_set_error(RSS_EIO, "rss_hash_device: launch failed (test hook fail_launch)");
#endif
    return ::launch_hash(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, flags,
                         stream, reta, ws);
}

int launch_hash6(const rss_key6* key, const rss_tuple6* d_tuples, size_t n, uint32_t htable,
                 uint32_t nqueues, uint32_t* d_hash, void* d_queue, uint64_t* d_counts,
                 uint32_t flags, hipStream_t stream, const uint32_t* reta, uint64_t* ws) {
    return ::launch_hash6(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, flags,
                          stream, reta, ws);
}

int launch_generate(uint64_t seed, uint64_t first_index, size_t n, rss_tuple4* d_tuples,
                    hipStream_t stream) {
    DeviceInfo info;
    int rc = device_info(&info);
    if (rc) return rc;
    const uint64_t want = (n + 255) / 256;
    const uint64_t cap = (uint64_t)info.cu_count * 8;
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    hipLaunchKernelGGL(rss_generate_kernel, dim3(grid), dim3(256), 0, stream, seed, first_index,
                       (uint64_t)n, reinterpret_cast<uint32_t*>(d_tuples));
    RSS_HIP_CHECK(hipGetLastError());
    return RSS_OK;
}

}  // namespace rss

#ifdef RSS_TEST_HOOKS
// ------------------------------------------------- test hooks (tests only) --
// Exported by librss_toeplitz_hooks.so alone (rss_test_hooks.h): the product library has
// neither these symbols nor the options they set.
namespace {
uint32_t g_guard_sleep_host = 0;  // the value last copied to g_guard_sleep
}  // namespace

extern "C" {

int rss_test_set_option(const char* name, int value) {
    if (!name) return rss_set_error(RSS_EINVAL, "rss_test_set_option: NULL name");
    const std::string n(name);
    if (n == "recount") g_opt.recount = value;
    else if (n == "range8") g_opt.range8 = value != 0;
    else if (n == "small_lut") g_opt.small_lut = value != 0;
    else if (n == "prefetch") g_opt.prefetch = value;
    else if (n == "balance") g_opt.balance = value != 0;
    else if (n == "counts_perm") g_opt.counts_perm = value != 0;
    else if (n == "resid") g_opt.resid = value != 0;
    else if (n == "wide") g_opt.wide = value != 0;
    else if (n == "alloc_fail") g_opt.alloc_fail = value;  // AllocKind bits
    else if (n == "fail_launch") g_opt.fail_launch = value;
    else if (n == "guard_sleep") {
        const uint32_t v = value > 0 ? (uint32_t)value : 0u;
        RSS_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_guard_sleep), &v, sizeof v));
        g_guard_sleep_host = v;
    } else return rss_set_error(RSS_EINVAL, "rss_test_set_option: unknown option '%s'", name);
    return RSS_OK;
}

// (the device word only when it was set: a process without a GPU never touches HIP here)
void rss_test_reset_options(void) {
    g_opt = Options{};
    if (g_guard_sleep_host) {
        const uint32_t zero = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_guard_sleep), &zero, sizeof zero);
        g_guard_sleep_host = 0;
    }
}

int rss_test_guard_margin(uint32_t* out, int reset) {
    if (!out) return rss_set_error(RSS_EINVAL, "rss_test_guard_margin: NULL out");
    RSS_HIP_CHECK(hipDeviceSynchronize());
    RSS_HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_guard_margin), sizeof(uint32_t) * kMargins));
    if (reset) {
        const uint32_t zero[kMargins] = {};
        RSS_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_guard_margin), zero, sizeof zero));
    }
    return RSS_OK;
}

}  // extern "C"
#endif  // RSS_TEST_HOOKS

// rss_keysearch.hip -- key search: the per-queue counts of the same
// device-resident tuples under many keys in one launch -- the scale-up of the reference's
// HashKey.random_hash_key() candidates (hash_key.py:53-60) each run through
// Simulator.calc_hash / calc_queue_number / value_counts (simulator.py:74-113).  Two table
// sets (packed buckets of 8 / 4 keys, pairs of full hashes), described below.  No test hooks:
// compiled once for both libraries.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <algorithm>

#include "rss_engine.h"
#include "rss_kernel_common.h"

namespace {

// Key search: per-queue counts of the same tuples under many
// keys.  A table index depends only on the tuple, so one table can serve two keys: entry
// v holds (key A's XOR of windows, key B's) as 8 bytes and ONE ds_read_b64 -- 64 banks,
// 256 B/clk (twice ds_read_b32's rate) -- fetches both keys' terms.  Two table sets:
// * the packed kernel (power-of-two H, several keys' low bits per entry) reads the small
//   tables' 21 fields (5, 5, 5, 5, 5, 5, 2 bits of each word, LSB first; kSmallLut) with
//   8-byte entries: 32 entries x 8 B = 256 B cover the 64 banks exactly once, so every entry
//   sits on its own bank pair and a random index never conflicts -- 21 conflict-free reads
//   (2 LDS cycles each) per tuple against 9 random reads at ~7 cycles each on the wide
//   tables below (PMC: 0 against 44 of 80 LDS cycles per 64 tuples x 8 keys in bank
//   conflicts, profiles/r04/pmc_keysearch*/); at Q = 24 the two run equal (the small tables'
//   extra address VALU makes it VALU-bound instead), but 5.25 KiB of tables leave ~155 KiB to
//   the bins: 8 keys per workgroup up to Q = 154 (wide tables: 40) and 4 up to 309 (80);
// * the pair kernel (any H: two full 32-bit hashes, their Lemire remainders and two adds per
//   tuple) keeps the nine wide tables of 2048 / 1024 entries (11 / 10 input bits, field LSBs
//   first as in the hash kernel's partition), whose 9 lookups cost less VALU than 21:
//     t0 w0[10:0]  t1 w0[21:11]  t2 w1[10:0]  t3 w2[15:11] | w2[31:27] << 5  t4 w0[31:22]
//     t5 w1[21:11] t6 w2[10:0]   t7 w2[26:16] t8 w1[31:22]
//   = 6 x 16 + 3 x 8 KiB = 120 KiB; on the small tables it ran 0.77 against 0.97 T
//   evaluations/s at H = 100, Q = 24 (profiles/archive/r04/small_tables/keysearch_configs.jsonl).
// blockIdx.y selects the pair; each workgroup histograms its grid-stride share of the
// tuples into counts rows 2y, 2y+1.  With the tuples resident in the 256 MiB Infinity Cache
// the re-reads stay on die.
constexpr uint32_t kPairLutBytes = kSmallTables * 256;            // 5376 (packed kernel)
constexpr uint32_t kPackedBinBytesMax = kLdsBytes - kPairLutBytes;  // 154.75 KiB for the bins
constexpr uint32_t kWidePairLutBytes = 6 * 16384 + 3 * 8192;     // 122880 (pair kernel)
constexpr uint32_t kWidePairBinBytesMax = kLdsBytes - kWidePairLutBytes;  // 40 KiB, 2 x Q bins

__host__ __device__ constexpr int wide_pair_width(int t) {
    return (t == 3 || t == 4 || t == 8) ? 10 : 11;
}
__host__ __device__ constexpr uint32_t wide_pair_table(int t) {  // byte offset
    return t == 0 ? 0u : t == 1 ? 16384u : t == 2 ? 32768u : t == 3 ? 49152u : t == 4 ? 57344u
         : t == 5 ? 65536u : t == 6 ? 81920u : t == 7 ? 98304u : 114688u;
}
// input bit (0 = MSB of the source ip) feeding bit b of table t's index
__host__ __device__ constexpr int wide_pair_bit(int t, int b) {
    return t == 0 ? 31 - b : t == 1 ? 20 - b : t == 2 ? 63 - b
         : t == 3 ? (b < 5 ? 84 - b : 73 - b)
         : t == 4 ? 9 - b : t == 5 ? 52 - b : t == 6 ? 95 - b : t == 7 ? 79 - b : 41 - b;
}

template <int kT>
__device__ __forceinline__ void build_wide_pair_table(uint2* lut, const uint32_t* __restrict__ wa,
                                                      const uint32_t* __restrict__ wb, uint32_t tid) {
    uint32_t a = 0, b = 0;
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        const bool set = (tid >> j) & 1u;
        a ^= set ? wa[wide_pair_bit(kT, j)] : 0u;
        b ^= set ? wb[wide_pair_bit(kT, j)] : 0u;
    }
    uint2* dst = lut + wide_pair_table(kT) / 8;
    dst[tid] = make_uint2(a, b);
    if constexpr (wide_pair_width(kT) == 11)
        dst[tid + 1024] = make_uint2(a ^ wa[wide_pair_bit(kT, 10)], b ^ wb[wide_pair_bit(kT, 10)]);
}

// byte address of wide table t's entry: 2 VALU (4 for the two-field t3); tables 5..8 take
// their 64 KiB base from the opaque register `hi`
template <int kT>
__device__ __forceinline__ uint32_t wide_pair_offset(uint32_t w0, uint32_t w1, uint32_t w2,
                                                     uint32_t hi) {
    if constexpr (kT == 0) return (w0 << 3) & 0x3FF8u;
    if constexpr (kT == 1) return (w0 >> 8) & 0x3FF8u;
    if constexpr (kT == 2) return (w1 << 3) & 0x3FF8u;
    if constexpr (kT == 3) return ((w2 >> 8) & 0xF8u) | ((w2 >> 19) & 0x1F00u);
    if constexpr (kT == 4) return (w0 >> 19) & 0x1FF8u;
    if constexpr (kT == 5) return ((w1 >> 8) & 0x3FF8u) | hi;
    if constexpr (kT == 6) return ((w2 << 3) & 0x3FF8u) | hi;
    if constexpr (kT == 7) return ((w2 >> 13) & 0x3FF8u) | hi;
    return ((w1 >> 19) & 0x1FF8u) | hi;
}

template <int kT>
__device__ __forceinline__ uint2 wide_pair_term(const char* lut, uint32_t w0, uint32_t w1,
                                                uint32_t w2, uint32_t hi) {
    constexpr uint32_t kImm = wide_pair_table(kT) & 0xFFFFu;
    return *reinterpret_cast<const uint2*>(lut + kImm + wide_pair_offset<kT>(w0, w1, w2, hi));
}

// (hash under key A, hash under key B) of one tuple on the wide tables
__device__ __forceinline__ uint2 toeplitz_hash_wide_pair(const uint2* __restrict__ lut, uint32_t w0,
                                                         uint32_t w1, uint32_t w2, uint32_t hi) {
    const char* base = reinterpret_cast<const char*>(lut);
    const uint2 t0 = wide_pair_term<0>(base, w0, w1, w2, hi), t1 = wide_pair_term<1>(base, w0, w1, w2, hi);
    const uint2 t2 = wide_pair_term<2>(base, w0, w1, w2, hi), t3 = wide_pair_term<3>(base, w0, w1, w2, hi);
    const uint2 t4 = wide_pair_term<4>(base, w0, w1, w2, hi), t5 = wide_pair_term<5>(base, w0, w1, w2, hi);
    const uint2 t6 = wide_pair_term<6>(base, w0, w1, w2, hi), t7 = wide_pair_term<7>(base, w0, w1, w2, hi);
    const uint2 t8 = wide_pair_term<8>(base, w0, w1, w2, hi);
    return make_uint2(xor3(xor3(t0.x, t1.x, t2.x), xor3(t3.x, t4.x, t5.x), xor3(t6.x, t7.x, t8.x)),
                      xor3(xor3(t0.y, t1.y, t2.y), xor3(t3.y, t4.y, t5.y), xor3(t6.y, t7.y, t8.y)));
}

// entry e = 32 t + v of the 21 pair tables: (XOR of key A's windows, of key B's) over the
// input bits set in v; `win(i)` gives the two keys' window i as a uint2
template <typename Win>
__device__ __forceinline__ void build_small_pair_lut(uint2* lut, Win win, uint32_t tid) {
    for (uint32_t e = tid; e < kSmallLutDwords; e += kBlock) {
        const int t = (int)(e >> 5);
        const uint32_t v = e & 31u;
        const int width = small_width(t % kSmallFields);
        uint32_t a = 0, b = 0;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            if (j < width && ((v >> j) & 1u)) {
                const uint2 w = win(small_slice_bit(t, j));
                a ^= w.x;
                b ^= w.y;
            }
        }
        lut[e] = (v >> width) ? make_uint2(0u, 0u) : make_uint2(a, b);
    }
}

// table 7k + j's 8-byte term for word w (= word k): the field moved to byte offset 8 * field
template <int kT>
__device__ __forceinline__ uint2 small_pair_term(const char* lut, uint32_t w) {
    constexpr int j = kT % kSmallFields, o = 5 * j;
    uint32_t off;
    if constexpr (j == 0)
        off = (w << 3) & 0xF8u;
    else if constexpr (j == 6)
        off = (w >> 27) & 0x18u;
    else
        off = (w >> (o - 3)) & 0xF8u;
    return *reinterpret_cast<const uint2*>(lut + kT * 256 + off);
}

template <int kBase>
__device__ __forceinline__ uint2 small_pair_word(const char* lut, uint32_t w) {  // 7 terms
    const uint2 t0 = small_pair_term<kBase + 0>(lut, w), t1 = small_pair_term<kBase + 1>(lut, w);
    const uint2 t2 = small_pair_term<kBase + 2>(lut, w), t3 = small_pair_term<kBase + 3>(lut, w);
    const uint2 t4 = small_pair_term<kBase + 4>(lut, w), t5 = small_pair_term<kBase + 5>(lut, w);
    const uint2 t6 = small_pair_term<kBase + 6>(lut, w);
    return make_uint2(xor3(xor3(t0.x, t1.x, t2.x), xor3(t3.x, t4.x, t5.x), t6.x),
                      xor3(xor3(t0.y, t1.y, t2.y), xor3(t3.y, t4.y, t5.y), t6.y));
}

// (hash under key A, hash under key B) of one tuple (packed kernel: 8 / 4 keys' low bits)
__device__ __forceinline__ uint2 toeplitz_hash_pair(const uint2* __restrict__ lut, uint32_t w0,
                                                    uint32_t w1, uint32_t w2) {
    const char* base = reinterpret_cast<const char*>(lut);
    const uint2 a = small_pair_word<0>(base, w0), b = small_pair_word<7>(base, w1);
    const uint2 c = small_pair_word<14>(base, w2);
    return make_uint2(xor3(a.x, b.x, c.x), xor3(a.y, b.y, c.y));
}

template <bool kHPow2, int kQMode, int kHist>
__device__ __forceinline__ void count_pair(uint32_t* bins_a, uint32_t* bins_b, uint2 h,
                                           uint32_t col, const LaunchParams& qa,
                                           const LaunchParams& qb) {
    count_queue<kHist>(bins_a, queue_of<kQMode>(bucket_of<kHPow2>(h.x, qa), qa), col, qa);
    count_queue<kHist>(bins_b, queue_of<kQMode>(bucket_of<kHPow2>(h.y, qb), qb), col, qb);
}

template <int kHist>
__device__ __forceinline__ void flush_bins(const uint32_t* bins, unsigned long long* counts,
                                           uint32_t Q, uint32_t tid) {
    for (uint32_t k = tid; k < Q; k += kBlock) {
        uint32_t s;
        if constexpr (kHist == HIST_PRIVATE) {
            s = 0;
            for (uint32_t c = 0; c < kBinCols; ++c) s += bins[k * kBinCols + ((c + k) & (kBinCols - 1))];
        } else {
            s = bins[k];
        }
        if (s) atomicAdd(&counts[k], (unsigned long long)s);
    }
}

template <bool kHPow2, int kQMode, int kHist, bool kVec4>
__global__ __launch_bounds__(kBlock) void rss_key_search_kernel(const LaunchParams p) {
    __shared__ uint2 lut[kWidePairLutBytes / 8];
    extern __shared__ uint32_t bins[];
    const uint32_t tid = threadIdx.x;
    // keys 2y and 2y+1; an odd last key is paired with itself and its copy discarded
    const uint32_t key_a = 2 * blockIdx.y;
    const bool has_b = key_a + 1 < p.nkeys;
    const uint32_t key_b = has_b ? key_a + 1 : key_a;
    const uint32_t* wa = p.key_windows + (size_t)RSS_INPUT_BITS * key_a;
    const uint32_t* wb = p.key_windows + (size_t)RSS_INPUT_BITS * key_b;
    build_wide_pair_table<0>(lut, wa, wb, tid);
    build_wide_pair_table<1>(lut, wa, wb, tid);
    build_wide_pair_table<2>(lut, wa, wb, tid);
    build_wide_pair_table<3>(lut, wa, wb, tid);
    build_wide_pair_table<4>(lut, wa, wb, tid);
    build_wide_pair_table<5>(lut, wa, wb, tid);
    build_wide_pair_table<6>(lut, wa, wb, tid);
    build_wide_pair_table<7>(lut, wa, wb, tid);
    build_wide_pair_table<8>(lut, wa, wb, tid);
    const uint32_t per_key =
        kHist == HIST_PRIVATE ? p.Q * kBinCols : (kHist == HIST_SHARED ? p.Q : 0u);
    for (uint32_t e = tid; e < 2 * per_key; e += kBlock) bins[e] = 0;
    __syncthreads();

    LaunchParams qa = p, qb = p;  // per-key counts rows
    qa.counts = p.counts + (size_t)key_a * p.q_stride;
    qb.counts = p.counts + (size_t)key_b * p.q_stride;
    uint32_t* bins_a = bins;
    uint32_t* bins_b = bins + per_key;
    const uint32_t col = tid & (kBinCols - 1);
    uint32_t hi = 65536u;
    asm volatile("" : "+v"(hi));
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    uint64_t tail_begin = 0;
    if constexpr (kVec4) {
        const uint4* __restrict__ src = reinterpret_cast<const uint4*>(p.tuples);
        const uint64_t ngroups = p.n >> 2;
        for (uint64_t g = gtid; g < ngroups; g += gstride) {
            const uint4 a = src[3 * g + 0];
            const uint4 b = src[3 * g + 1];
            const uint4 c = src[3 * g + 2];
            count_pair<kHPow2, kQMode, kHist>(bins_a, bins_b, toeplitz_hash_wide_pair(lut, a.x, a.y, a.z, hi), col, qa, qb);
            count_pair<kHPow2, kQMode, kHist>(bins_a, bins_b, toeplitz_hash_wide_pair(lut, a.w, b.x, b.y, hi), col, qa, qb);
            count_pair<kHPow2, kQMode, kHist>(bins_a, bins_b, toeplitz_hash_wide_pair(lut, b.z, b.w, c.x, hi), col, qa, qb);
            count_pair<kHPow2, kQMode, kHist>(bins_a, bins_b, toeplitz_hash_wide_pair(lut, c.y, c.z, c.w, hi), col, qa, qb);
        }
        tail_begin = ngroups << 2;
    }
    for (uint64_t i = tail_begin + gtid; i < p.n; i += gstride) {
        const uint32_t* t = reinterpret_cast<const uint32_t*>(p.tuples) + 3 * i;
        count_pair<kHPow2, kQMode, kHist>(bins_a, bins_b, toeplitz_hash_wide_pair(lut, t[0], t[1], t[2], hi), col, qa, qb);
    }
    if constexpr (kHist == HIST_PRIVATE || kHist == HIST_SHARED) {
        __syncthreads();
        flush_bins<kHist>(bins_a, qa.counts, p.Q, tid);
        if (has_b) flush_bins<kHist>(bins_b, qb.counts, p.Q, tid);
    }
}

// Packed-bucket key search.  For a power-of-two H the bucket (simulator.py:97,
// `hash % htable`) is the low log2(H) bits of the hash, and the low bits of a XOR are
// the XOR of the low bits: a table term needs only those bits of each key.  With
// H <= 256 an 8-byte entry holds the low BYTE of 8 keys' terms (H <= 65536: the low
// half-word of 4 keys'), so the same 21 conflict-free ds_read_b64 of the pair kernel
// serve 8 (4) keys and the per-key work is a bit-field extract, the queue step and one
// LDS add.
// Bins are [q][key][lane column]: the key's offset is a ds_add immediate and every
// half-wave's adds stay conflict-free.
constexpr uint32_t kPackedPrepBytes = RSS_INPUT_BITS * 8;  // packed windows, before the bins

template <int kLaneBits, int kQMode, bool kVec4>
__global__ __launch_bounds__(kBlock) void rss_key_search_packed_kernel(const LaunchParams p) {
    constexpr uint32_t kKeys = 64 / kLaneBits;
    __shared__ uint2 lut[kPairLutBytes / 8];
    extern __shared__ uint32_t bins[];
    const uint32_t tid = threadIdx.x;
    const uint32_t key0 = kKeys * blockIdx.y;

    // 1. pack: lane k of packed[i] = low kLaneBits of key (key0 + k)'s window i (a key
    //    past the end repeats the last key; its counts are discarded)
    uint2* packed = reinterpret_cast<uint2*>(bins);
    if (tid < RSS_INPUT_BITS) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (uint32_t k = 0; k < kKeys; ++k) {
            const uint32_t key = min(key0 + k, p.nkeys - 1);
            const uint32_t w = p.key_windows[(size_t)RSS_INPUT_BITS * key + tid] &
                               ((1u << kLaneBits) - 1);
            const uint32_t shift = k * kLaneBits;
            if (shift < 32) lo |= w << shift;
            else hi |= w << (shift - 32);
        }
        packed[tid] = make_uint2(lo, hi);
    }
    __syncthreads();
    build_small_pair_lut(lut, [&](int i) { return packed[i]; }, tid);
    __syncthreads();  // packed windows are dead: the region becomes bins
    const uint32_t nbins = p.Q * kKeys * kBinCols;
    for (uint32_t e = tid; e < nbins; e += kBlock) bins[e] = 0;
    __syncthreads();

    uint32_t* bins_col = bins + (tid & (kBinCols - 1));
    char* bins_colb = reinterpret_cast<char*>(bins_col);
    const uint32_t hbits = 31 - __clz(p.H);  // log2(H)
    constexpr uint32_t kRowShift = kLaneBits == 8 ? 10 : 9;  // log2(kKeys * kBinCols * 4)
    // byte-lane queue step folded into the bin address: q * 2^kRowShift =
    // (b << kRowShift) - d * (Q << kRowShift), d = floor(b / Q) (as QM_FAST8): two
    // full-rate 24-bit multiplies, the second a v_mad_i32_i24
    const int neg_q_row = -(int)(p.Q << kRowShift);
    // byte lanes: mask every lane to the bucket bits at once, then each key's bucket is
    // a plain byte select (which the multiplies and shifts take as an SDWA operand)
    const uint32_t lane_mask4 = (p.H - 1) * 0x01010101u;
    auto count = [&](uint2 x) {
        if constexpr (kLaneBits == 8) {
            x.x &= lane_mask4;
            x.y &= lane_mask4;
        }
#pragma unroll
        for (uint32_t k = 0; k < kKeys; ++k) {
            const uint32_t word = (k * kLaneBits) < 32 ? x.x : x.y;
            const uint32_t b = kLaneBits == 8 ? (word >> ((k * 8) & 31)) & 0xFFu
                                              : __builtin_amdgcn_ubfe(word, (k * kLaneBits) & 31, hbits);
            uint32_t row;
            if constexpr (kLaneBits == 8 && kQMode == QM_FAST16) {
                const uint32_t d = __umul24(b, p.q_m16) >> 16;
                row = (uint32_t)__mul24((int)d, neg_q_row) + (b << kRowShift);
            } else {
                row = queue_of<kQMode>(b, p) << kRowShift;
            }
            __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(bins_colb + row) + k * kBinCols, 1u,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    uint64_t tail_begin = 0;
    if constexpr (kVec4) {
        const uint4* __restrict__ src = reinterpret_cast<const uint4*>(p.tuples);
        const uint64_t ngroups = p.n >> 2;
        for (uint64_t g = gtid; g < ngroups; g += gstride) {
            const uint4 a = src[3 * g + 0];
            const uint4 b = src[3 * g + 1];
            const uint4 c = src[3 * g + 2];
            count(toeplitz_hash_pair(lut, a.x, a.y, a.z));
            count(toeplitz_hash_pair(lut, a.w, b.x, b.y));
            count(toeplitz_hash_pair(lut, b.z, b.w, c.x));
            count(toeplitz_hash_pair(lut, c.y, c.z, c.w));
        }
        tail_begin = ngroups << 2;
    }
    for (uint64_t i = tail_begin + gtid; i < p.n; i += gstride) {
        const uint32_t* t = reinterpret_cast<const uint32_t*>(p.tuples) + 3 * i;
        count(toeplitz_hash_pair(lut, t[0], t[1], t[2]));
    }
    __syncthreads();
    for (uint32_t e = tid; e < p.Q * kKeys; e += kBlock) {
        const uint32_t q = e / kKeys, k = e % kKeys;
        if (key0 + k >= p.nkeys) continue;
        uint32_t s = 0;
        for (uint32_t c = 0; c < kBinCols; ++c) s += bins[e * kBinCols + ((c + e) & (kBinCols - 1))];
        if (s) atomicAdd(&p.counts[(size_t)(key0 + k) * p.q_stride + q], (unsigned long long)s);
    }
}

template <bool kHPow2, int kQMode, int kHist>
KernelFn pick_search_vec(bool vec4) {
    return vec4 ? rss_key_search_kernel<kHPow2, kQMode, kHist, true>
                : rss_key_search_kernel<kHPow2, kQMode, kHist, false>;
}

template <bool kHPow2, int kQMode>
KernelFn pick_search_hist(int hist, bool vec4) {
    switch (hist) {
        case HIST_PRIVATE: return pick_search_vec<kHPow2, kQMode, HIST_PRIVATE>(vec4);
        case HIST_SHARED: return pick_search_vec<kHPow2, kQMode, HIST_SHARED>(vec4);
        default: return pick_search_vec<kHPow2, kQMode, HIST_GLOBAL>(vec4);
    }
}

template <bool kHPow2>
KernelFn pick_search(int qmode, int hist, bool vec4) {
    switch (qmode) {
        case QM_MASK: return pick_search_hist<kHPow2, QM_MASK>(hist, vec4);
        case QM_FAST16: return pick_search_hist<kHPow2, QM_FAST16>(hist, vec4);
        default: return pick_search_hist<kHPow2, QM_FAST32>(hist, vec4);
    }
}

// ~256K tuples per workgroup amortise its 120 KiB table build
inline unsigned search_grid_x(size_t n, int cu_count) {
    const uint64_t slices = (n + (1u << 18) - 1) >> 18;
    return (unsigned)(slices < (uint64_t)cu_count ? slices : cu_count);
}

template <int kLaneBits, int kQMode>
KernelFn pick_packed_vec(bool vec4) {
    return vec4 ? rss_key_search_packed_kernel<kLaneBits, kQMode, true>
                : rss_key_search_packed_kernel<kLaneBits, kQMode, false>;
}

KernelFn pick_packed(int lane_bits, int qmode, bool vec4) {
    if (lane_bits == 8)
        return qmode == QM_MASK ? pick_packed_vec<8, QM_MASK>(vec4) : pick_packed_vec<8, QM_FAST16>(vec4);
    return qmode == QM_MASK ? pick_packed_vec<16, QM_MASK>(vec4) : pick_packed_vec<16, QM_FAST16>(vec4);
}

int launch_search(const uint32_t* d_windows, size_t nkeys, const rss_tuple4* d_tuples, size_t n,
                  uint32_t htable, uint32_t nqueues, uint64_t* d_counts, hipStream_t stream) {
    if (!d_windows || !d_counts || nkeys == 0)
        return rss_set_error(RSS_EINVAL, "rss_key_search_device: windows/counts NULL or no keys");
    if (htable < 1 || nqueues < 1)
        return rss_set_error(RSS_EINVAL,
                             "rss_key_search_device: htable (%u) and nqueues (%u) must be >= 1",
                             htable, nqueues);
    if (n && !d_tuples) return rss_set_error(RSS_EINVAL, "rss_key_search_device: tuples is NULL");
    RSS_HIP_CHECK(hipMemsetAsync(d_counts, 0, sizeof(uint64_t) * nqueues * nkeys, stream));
    if (n == 0) return RSS_OK;
    LaunchParams p;
    memset(&p, 0, sizeof p);
    p.tuples = d_tuples;
    p.n = n;
    p.q_stride = nqueues;  // rows keep the caller's nqueues; queues >= min(H, Q) stay zero
    const uint32_t q_eff = effective_queues(htable, nqueues, nullptr);
    int qmode, hist;
    uint32_t bin_bytes;  // per key; a workgroup holds the bins of its two keys
    const bool h_pow2 = setup_modes(&p, htable, q_eff, true, &qmode, &hist, &bin_bytes,
                                    kWidePairBinBytesMax / 2, false);
    const bool vec4 = aligned16(d_tuples);
    DeviceInfo info;
    int rc = device_info(&info);
    if (rc) return rc;
    // packed buckets (8 keys per table entry for H <= 256, 4 for H <= 65536) whenever
    // their private bins fit (8 keys: Q <= 154, 4 keys: Q <= 309); else pairs of full hashes
    const bool bytes_fit = (uint64_t)q_eff * 8 * kBinCols * 4 <= kPackedBinBytesMax;
    const int lane_bits = htable <= 256u && bytes_fit ? 8 : 16;
    const uint32_t keys_per_wg = 64 / lane_bits;
    const uint64_t packed_bins = (uint64_t)q_eff * keys_per_wg * kBinCols * 4;
    if (h_pow2 && htable <= 65536u && packed_bins <= kPackedBinBytesMax) {
        p.q_m16 = 65536u / q_eff + (65536u % q_eff != 0);
        KernelFn fn = pick_packed(lane_bits, qmode, vec4);
        const unsigned gx = search_grid_x(n, info.cu_count);
        const uint32_t shmem = (uint32_t)std::max<uint64_t>(packed_bins, kPackedPrepBytes);
        const size_t max_keys = (size_t)keys_per_wg * 65535;  // grid.y limit
        for (size_t k0 = 0; k0 < nkeys; k0 += max_keys) {
            const size_t kn = nkeys - k0 < max_keys ? nkeys - k0 : max_keys;
            p.key_windows = d_windows + k0 * RSS_INPUT_BITS;
            p.counts = reinterpret_cast<unsigned long long*>(d_counts + k0 * nqueues);
            p.nkeys = (uint32_t)kn;
            hipLaunchKernelGGL(fn, dim3(gx, (unsigned)((kn + keys_per_wg - 1) / keys_per_wg)),
                               dim3(kBlock), shmem, stream, p);
            RSS_HIP_CHECK(hipGetLastError());
        }
        return RSS_OK;
    }
    KernelFn fn = h_pow2 ? pick_search<true>(qmode, hist, vec4) : pick_search<false>(qmode, hist, vec4);
    const unsigned gx = search_grid_x(n, info.cu_count);
    constexpr size_t kMaxKeysPerLaunch = 2 * 65535;  // grid.y (key pairs) limit
    for (size_t k0 = 0; k0 < nkeys; k0 += kMaxKeysPerLaunch) {
        const size_t kn = nkeys - k0 < kMaxKeysPerLaunch ? nkeys - k0 : kMaxKeysPerLaunch;
        p.key_windows = d_windows + k0 * RSS_INPUT_BITS;
        p.counts = reinterpret_cast<unsigned long long*>(d_counts + k0 * nqueues);
        p.nkeys = (uint32_t)kn;
        hipLaunchKernelGGL(fn, dim3(gx, (unsigned)((kn + 1) / 2)), dim3(kBlock), 2 * bin_bytes,
                           stream, p);
        RSS_HIP_CHECK(hipGetLastError());
    }
    return RSS_OK;
}

}  // namespace

// ------------------------------------------------------ launcher (rss_engine.h) --
namespace rss {

int launch_search(const uint32_t* d_windows, size_t nkeys, const rss_tuple4* d_tuples, size_t n,
                  uint32_t htable, uint32_t nqueues, uint64_t* d_counts, hipStream_t stream) {
    return ::launch_search(d_windows, nkeys, d_tuples, n, htable, nqueues, d_counts, stream);
}

}  // namespace rss

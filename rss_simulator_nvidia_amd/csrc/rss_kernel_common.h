// rss_kernel_common.h -- what the engine's kernel files share (internal, not ABI): the
// constants, LaunchParams, the 12-bit and small Toeplitz tables, bucket / queue steps, the
// histogram bins (private, shared, guarded u16 / u8), the output stores, the single-pass
// fold, the balanced walk and the residual lists; and the host-side launch setup (device
// info, modulo strategy, histogram placement, indirection-table checks).  Everything is in
// an anonymous namespace: each kernel file (rss_toeplitz.hip, rss_keysearch.hip) instantiates
// what it uses.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <vector>

#include "rss_engine.h"
#include "rss_internal.h"
#include "rss_toeplitz.h"

namespace {

// ------------------------------------------------------------ constants -----
constexpr int kBlock = 1024;            // threads per workgroup (16 waves)
constexpr int kBlocksPerCU = 1;         // the 128 KiB LUT admits one workgroup per CU
constexpr int kChunkBits = 12;          // input bits per table lookup
constexpr int kTables = RSS_INPUT_BITS / kChunkBits;        // 8
constexpr uint32_t kTableEntries = 1u << kChunkBits;        // 4096
constexpr uint32_t kLutDwords = kTables * kTableEntries;    // 32768
constexpr uint32_t kLutBytes = kLutDwords * 4;              // 128 KiB
constexpr uint32_t kLdsBytes = 160 * 1024;                  // gfx950 LDS per CU
constexpr uint32_t kBinBytesMax = kLdsBytes - kLutBytes;    // 32 KiB for histogram bins
constexpr int kBinCols = 32;            // private histogram columns (one per bank)
static_assert(kLutBytes == 128 * 1024, "LUT layout: 8 tables x 4096 x u32");
static_assert(kBlock * 4 == (int)kTableEntries, "LUT build maps 4 entries per thread per table");

enum QueueMode { QM_MASK = 0, QM_FAST16 = 1, QM_FAST32 = 2, QM_TABLE = 3, QM_FAST8 = 4 };
constexpr uint32_t kRetaMax = 1024;  // indirection-table entries carried in the kernarg
enum HistMode { HIST_PRIVATE = 0, HIST_SHARED = 1, HIST_GLOBAL = 2, HIST_NONE = 3, HIST_RANGE = 4,
                HIST_RANGE16 = 5, HIST_RANGE8 = 6 };
// HIST_RANGE8 (IPv4 small-table kernel, past the u16 bins' reach): u8 bins, four per dword, a
// guard at 0x80 and a poison word for a bin that wraps (range8_guard) -- 161144 queues in the
// LDS beside the small tables, one pass.
// HIST_RANGE16 (IPv4 kernel): HIST_RANGE with u16 bins, two per dword, twice the queues in the
// same LDS -- a guard at 0x8000 and a poison word like HIST_RANGE8's (range16_guard).
// HIST_RANGE: shared u32 LDS bins for queues [q_lo, q_lo + q_span) only -- the IPv6 kernel's
// first range of a multi-pass launch for nqueues whose bins do not fit the LDS beside its
// tables (launch_hash6), instead of one global atomic per tuple (13x slower).
enum QueueWidth { QW_U32 = 0, QW_U16 = 1, QW_U8 = 2, QW_U16R = 3 };
// QW_U16R: a counts-only many-queues launch's scratch column (launch_hash): u16 q - q_span for
// the queues past the hash pass's LDS range [0, q_span), 0xFFFF (never counted) for the rest --
// half the bytes of a u32 column for the wide pass that counts [q_span, q_eff).

// Everything a launch needs, passed by value in the kernarg segment.
struct LaunchParams {
    uint32_t window[RSS_INPUT_BITS];  // rss_key::window
    const rss_tuple4* tuples;
    uint32_t* hash_out;
    void* queue_out;
    unsigned long long* counts;
    unsigned long long* ws;       // single-pass counts workspace (rss_hash_device_ws) or NULL
    uint32_t accumulate;          // with ws: fold mode (kFoldAccumulate)
    uint64_t n;
    uint64_t h_m64;     // ceil(2^64 / H) for the non-power-of-two htable path
    uint32_t h_mask;    // H - 1 when H is a power of two
    uint32_t H;
    uint32_t Q;
    uint32_t q_mask;    // Q - 1 (power of two) or ~0u when Q >= H (identity)
    uint32_t q_m32;     // ceil(2^32 / Q): exact b % Q for b, Q < 2^16
    uint32_t nkeys;     // key search: keys in this launch
    uint64_t q_m64;     // ceil(2^64 / Q): exact b % Q for any 32-bit b, Q
    uint32_t q_m16;     // ceil(2^16 / Q): exact b % Q for b < 256 (QM_FAST8, packed search)
    const uint32_t* key_windows;  // key search: nkeys x 96 windows in device memory
    uint32_t q_lo, q_span;        // HIST_RANGE: the queues this pass counts
    uint32_t* partial;            // HIST_RANGE16 / RANGE8: u16 / u8 [grid][partial_stride] rows;
    uint32_t partial_stride;      //   dwords per row
    uint32_t q_stride;            // key search: row stride of the [keys, nqueues] counts (>= Q)
    uint32_t tail_rows;           // balanced tail: rows handed out as units (0 = static grid-stride)
    uint32_t bal_off;             // balanced tail: byte offset of its LDS slot (dynamic LDS)
    uint32_t* ovf;                // HIST_RANGE16 / RANGE8: u32 [q_span] guard moves (2^15 / 128)
    uint32_t* poison;             //   set when a bin wrapped (rows and moves discarded)
    uint32_t fb_span;             // the recount's queues per slice (its u32 bins in the LDS)
    uint32_t prefetch;            // small-table passes: next group's loads before this group's LDS work
    unsigned long long* tail_ctr; // balanced tail's unit counter when the launch has no ws (HIST_RANGE8)
    void* resid_out;              // HIST_RANGE8 counts only: per-wave lists of q - q_span for the
    uint32_t* resid_counts;       //   tuples past the LDS range (u16 when resid_u16, else u32), wave
    uint64_t resid_cap;           //   v of workgroup x's at resid_out + (16 x + v) * resid_cap entries,
    uint32_t resid_u16;           //   its length in resid_counts[16 x + v] (no queue column)
    uint16_t reta[kRetaMax];      // QM_TABLE: queue of bucket b (ethtool -X indirection)
};

// ------------------------------------------------------------- device -------
// LUT: eight tables, each indexed by 12 of the 96 input bits; entry v of table t
// holds the XOR of the key windows of the input bits set in v -- the reference's
// inner loop (toeplitz.py:65-68) pre-summed over 12 bits.  Toeplitz is linear in
// the input bits, so any partition of the 96 bits into tables gives the exact hash.
// Entry (t, v) lives at LDS byte t*16384 + v*4.  One hash = 8 ds_read_b32 + 7 XOR.
//
// Partition (words w0 = src ip, w1 = dst ip, w2 = sport << 16 | dport, bit 0 = LSB):
//   t0: w0[31:24] | w2[15:12] << 8     t1: w1[31:24] | w2[31:28] << 8
//   t2: w0[11:0]   t3: w1[11:0]   t4: w0[23:12]   t5: w1[23:12]
//   t6: w2[11:0] (dport)          t7: w2[27:16] (sport)
// Every field's least significant bits -- the ones that vary from flow to flow in
// real traffic (sequential ports, neighbouring hosts) -- are the LOW bits of a table
// index, i.e. they select the LDS bank ((addr/4) mod 32 for ds_read_b32).  Slicing
// the MSB-first bit string in order instead puts e.g. sport[7:0] at index bits 4..11:
// on flow-like input (one IP pair, sequential source ports) every lane of a wave
// then reads a different entry of ONE bank, a 32-way conflict (measured: 55 % more
// SQ_LDS_BANK_CONFLICT cycles and 16 % longer counts-only launches than uniform input).

// Input bit (toeplitz.py:65-68 order: 0 = MSB of the source ip) that feeds bit b of
// table t's index.  Word k bit i is input bit 32k + 31 - i.
__host__ __device__ constexpr int slice_bit(int t, int b) {
    return t == 0 ? (b < 8 ? 7 - b : 91 - b)      // w0[24+b] ; w2[4+b]
         : t == 1 ? (b < 8 ? 39 - b : 75 - b)     // w1[24+b] ; w2[20+b]
         : t == 2 ? 31 - b                        // w0[b]
         : t == 3 ? 63 - b                        // w1[b]
         : t == 4 ? 19 - b                        // w0[12+b]
         : t == 5 ? 51 - b                        // w1[12+b]
         : t == 6 ? 95 - b                        // w2[b]
                  : 79 - b;                       // w2[16+b]
}

// Build: thread `tid` owns v = hi*1024 + tid (hi = 0..3) of every table: the low
// ten bits of v are its thread id, so it XORs their windows once per table and
// derives the four entries from the two top-bit windows.
__device__ __forceinline__ void build_lut(uint32_t* lut, const uint32_t* __restrict__ window,
                                          uint32_t tid) {
#pragma unroll
    for (int t = 0; t < kTables; ++t) {
        uint32_t base = 0;
#pragma unroll
        for (int b = 0; b < 10; ++b) base ^= ((tid >> b) & 1u) ? window[slice_bit(t, b)] : 0u;
        const uint32_t w10 = window[slice_bit(t, 10)], w11 = window[slice_bit(t, 11)];
        uint32_t* dst = lut + t * kTableEntries + tid;
        dst[0 * kBlock] = base;
        dst[1 * kBlock] = base ^ w10;
        dst[2 * kBlock] = base ^ w11;
        dst[3 * kBlock] = base ^ w10 ^ w11;
    }
}

// Byte address of table t's entry for (w0, w1, w2): the index moved to bits 2..13 and
// masked -- 2 VALU ops for the one-field tables 2..7, 4 for the two-field tables 0..1.
// Tables 4..7 sit above the 16-bit ds_read immediate, so their base 0x10000 is ORed
// in by the same v_and_or_b32 from `hi` -- an opaque register holding 0x10000 (a
// literal would cost a separate v_or).
template <int kT>
__device__ __forceinline__ uint32_t chunk_offset(uint32_t w0, uint32_t w1, uint32_t w2,
                                                 uint32_t hi) {
    constexpr uint32_t kMask = (kTableEntries - 1) << 2;  // 0x3FFC
    if constexpr (kT == 0) return ((w0 >> 22) & 0x3FCu) | ((w2 >> 2) & 0x3C00u);
    if constexpr (kT == 1) return ((w1 >> 22) & 0x3FCu) | ((w2 >> 18) & 0x3C00u);
    if constexpr (kT == 2) return (w0 << 2) & kMask;
    if constexpr (kT == 3) return (w1 << 2) & kMask;
    if constexpr (kT == 4) return ((w0 >> 10) & kMask) | hi;
    if constexpr (kT == 5) return ((w1 >> 10) & kMask) | hi;
    if constexpr (kT == 6) return ((w2 << 2) & kMask) | hi;
    return ((w2 >> 14) & kMask) | hi;
}

template <int kT>
__device__ __forceinline__ uint32_t lut_term(const char* lut, uint32_t w0, uint32_t w1, uint32_t w2,
                                             uint32_t hi) {
    constexpr uint32_t kImm = (kT & 3) * (kTableEntries * 4);  // fits the 16-bit offset
    return *reinterpret_cast<const uint32_t*>(lut + kImm + chunk_offset<kT>(w0, w1, w2, hi));
}

// a ^ b ^ c in one VALU op (v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Toeplitz hash of one 96-bit input (toeplitz.py:46-69 over the bytes of :113-142).
__device__ __forceinline__ uint32_t toeplitz_hash(const uint32_t* __restrict__ lut, uint32_t w0,
                                                  uint32_t w1, uint32_t w2, uint32_t hi) {
    const char* base = reinterpret_cast<const char*>(lut);
    return xor3(xor3(lut_term<0>(base, w0, w1, w2, hi), lut_term<1>(base, w0, w1, w2, hi),
                     lut_term<2>(base, w0, w1, w2, hi)),
                xor3(lut_term<3>(base, w0, w1, w2, hi), lut_term<4>(base, w0, w1, w2, hi),
                     lut_term<5>(base, w0, w1, w2, hi)),
                lut_term<6>(base, w0, w1, w2, hi) ^ lut_term<7>(base, w0, w1, w2, hi));
}

// Small tables (many-queues launches, DESIGN.md §3 "Many queues"): 21 tables of at most 32
// entries -- word k (w0, w1, w2) cut LSB first into fields of 5, 5, 5, 5, 5, 5 and 2 bits,
// table 7k + j indexed by field j -- 2688 bytes instead of the 12-bit tables' 128 KiB, so the
// LDS left for histogram bins grows from 16384 u16 queues to 80572 u16 / 161144 u8 queues.
// Each table starts on a 128-byte (32-bank) boundary and has at most 32 entries, so entry v
// is alone on bank v: lanes that hit one bank read one address and broadcast -- a random
// index can never conflict.  21 conflict-free ds_read_b32 (2 LDS cycles each) per tuple
// replace 8 random 12-bit reads (2 + ~4.5 conflict cycles each on uniform input) or 12
// random byte-table reads (the round-3 form, ~7 cycles each).  Entry (t, v) lives at LDS
// byte t*128 + v*4.
constexpr int kSmallFields = 7;                                  // per 32-bit word
constexpr int kSmallTables = 3 * kSmallFields;                   // 21
constexpr uint32_t kSmallLutDwords = kSmallTables * 32;          // 672
constexpr uint32_t kSmallLutBytes = kSmallLutDwords * 4;         // 2688
constexpr uint32_t kSmallStaticBytes = kSmallLutBytes + 8;      // + the balanced tail's LDS slot
__host__ __device__ constexpr int small_width(int j) { return j < 6 ? 5 : 2; }
// input bit (toeplitz.py:65-68 order) of bit b of table t's index: word t/7, bit 5 (t%7) + b
__host__ __device__ constexpr int small_slice_bit(int t, int b) {
    return 32 * (t / kSmallFields) + 31 - 5 * (t % kSmallFields) - b;
}

__device__ __forceinline__ void build_small_lut(uint32_t* lut, const uint32_t* __restrict__ window,
                                                uint32_t tid) {
    for (uint32_t e = tid; e < kSmallLutDwords; e += kBlock) {
        const int t = (int)(e >> 5);
        const uint32_t v = e & 31u;
        const int width = small_width(t % kSmallFields);
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 5; ++b)
            x ^= (b < width && ((v >> b) & 1u)) ? window[small_slice_bit(t, b)] : 0u;
        lut[e] = (v >> width) ? 0u : x;  // entries past a 2-bit table's 4 are never read
    }
}

// table 7k + j's term for word w (= word k): the field moved to byte offset 4 * field
template <int kT>
__device__ __forceinline__ uint32_t small_term(const char* lut, uint32_t w) {
    constexpr int j = kT % kSmallFields, o = 5 * j;
    uint32_t off;
    if constexpr (j == 0)
        off = (w << 2) & 0x7Cu;
    else if constexpr (j == 6)
        off = (w >> 28) & 0x0Cu;
    else
        off = (w >> (o - 2)) & 0x7Cu;
    return *reinterpret_cast<const uint32_t*>(lut + kT * 128 + off);
}

template <int kBase>
__device__ __forceinline__ uint32_t small_word(const char* lut, uint32_t w) {  // 7 terms
    return xor3(xor3(small_term<kBase + 0>(lut, w), small_term<kBase + 1>(lut, w),
                     small_term<kBase + 2>(lut, w)),
                xor3(small_term<kBase + 3>(lut, w), small_term<kBase + 4>(lut, w),
                     small_term<kBase + 5>(lut, w)),
                small_term<kBase + 6>(lut, w));
}

__device__ __forceinline__ uint32_t toeplitz_hash_small(const uint32_t* __restrict__ lut, uint32_t w0,
                                                        uint32_t w1, uint32_t w2) {
    const char* b = reinterpret_cast<const char*>(lut);
    return xor3(small_word<0>(b, w0), small_word<7>(b, w1), small_word<14>(b, w2));
}

template <bool kSmallLut>
__device__ __forceinline__ uint32_t hash_of(const uint32_t* lut, uint32_t w0, uint32_t w1,
                                            uint32_t w2, uint32_t hi) {
    if constexpr (kSmallLut) return toeplitz_hash_small(lut, w0, w1, w2);
    return toeplitz_hash(lut, w0, w1, w2, hi);
}

// hash % htable  (simulator.py:97, first modulo)
template <bool kHPow2>
__device__ __forceinline__ uint32_t bucket_of(uint32_t h, const LaunchParams& p) {
    if constexpr (kHPow2) {
        return h & p.h_mask;
    } else {
        // Lemire-Kaser-Kurz direct remainder, exact for all 32-bit h and H.
        const uint64_t low = p.h_m64 * (uint64_t)h;
        return (uint32_t)__umul64hi(low, (uint64_t)p.H);
    }
}

// bucket % nqueues  (simulator.py:97, second modulo)
template <int kQMode>
__device__ __forceinline__ uint32_t queue_of(uint32_t b, const LaunchParams& p) {
    if constexpr (kQMode == QM_MASK) {
        return b & p.q_mask;
    } else if constexpr (kQMode == QM_FAST8) {
        // b < 256, Q < 256: b - Q * ((b * ceil(2^16 / Q)) >> 16), exact (checked for every
        // b, Q), with full-rate 24-bit multiplies instead of FAST16's two quarter-rate ones
        const uint32_t d = __umul24(b, p.q_m16) >> 16;
        return b - __umul24(d, p.Q);
    } else if constexpr (kQMode == QM_FAST16) {
        return __umulhi(p.q_m32 * b, p.Q);  // b < 2^16, Q < 2^16
    } else {
        const uint64_t low = p.q_m64 * (uint64_t)b;
        return (uint32_t)__umul64hi(low, (uint64_t)p.Q);
    }
}

// queue of a bucket: the modulo modes above, or the indirection table copied to LDS
template <int kQMode>
__device__ __forceinline__ uint32_t queue_lookup(uint32_t b, const LaunchParams& p,
                                                 const uint32_t* reta_lds) {
    if constexpr (kQMode == QM_TABLE) {
        return reta_lds[b];
    } else {
        return queue_of<kQMode>(b, p);
    }
}

#ifdef RSS_TEST_HOOKS
// Test-hooks build only: the largest number of adds that landed on a guarded bin between the
// add that took it to half range and the guard's subtract, per guard kind (kMarginHash16: the
// hash pass's u16 bins, kMarginWide16: the u16 wide passes, kMarginHash8 / kMarginWide8: the
// u8 ones, modulo 256) -- read by rss_test_guard_margin.
enum { kMarginHash16 = 0, kMarginWide16 = 1, kMarginHash8 = 2, kMarginWide8 = 3, kMargins = 4 };
__device__ uint32_t g_guard_margin[kMargins];
// `at`: the field's value when the subtract landed = half + the adds in between (mod 2^bits)
template <int kBits>
__device__ __forceinline__ void record_margin(int kind, uint32_t at) {
    constexpr uint32_t kHalf = 1u << (kBits - 1), kField = (1u << kBits) - 1u;
    __hip_atomic_fetch_max(&g_guard_margin[kind], (at - kHalf) & kField, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
#define RSS_RECORD_MARGIN(bits, kind, at) record_margin<bits>(kind, at)
// Test-hooks build only: before its subtract a u16 guard's wave sleeps g_guard_sleep times
// s_sleep 127 (~3 us each), so that the workgroup's other waves carry the bin past 0xFFFF --
// a real wrap, which the poison word must catch (rss_test_set_option "guard_sleep").
__device__ uint32_t g_guard_sleep;
__device__ __forceinline__ void guard_delay() {
    const uint32_t n = *reinterpret_cast<volatile uint32_t*>(&g_guard_sleep);
    for (uint32_t i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
}
#define RSS_GUARD_DELAY() guard_delay()
#else
#define RSS_RECORD_MARGIN(bits, kind, at) ((void)(at))
#define RSS_GUARD_DELAY() ((void)0)
#endif

// HIST_RANGE16's two halves: the add (returns the dword's previous value, 0 out of range)
// and the guard (the add that returned 0x7FFF, so that its bin now holds 0x8000, subtracts
// 0x8000 from the bin and counts one move of 2^15 in p.ovf[r]).  The 4-tuple body issues its
// four adds before the four guards, so they do not wait for each other.
// Nothing bounds the adds that land on the bin between that add and the subtract: the
// workgroup's other waves keep adding while the guard's wave waits for its returns, and wave
// issue is not fair.  So a bin can pass 0xFFFF and carry into its neighbour (observed once in
// a u16 wide pass, profiles/archive/r04/u16_guard/).  Exactly the add that takes a field past 0xFFFF
// returns 0xFFFF, and it raises *p.poison: the launch's rows and moves are then discarded (the
// reduce is gated on !poison) and rss_range_fallback_kernel / rss_range_fallback_col_kernel
// recount the range with u32 bins (gated on poison) -- exact whatever the timing.
__device__ __forceinline__ uint32_t range16_add(uint32_t* bins, uint32_t q, const LaunchParams& p) {
    const uint32_t r = q - p.q_lo;  // wraps for q < q_lo
    if (r >= p.q_span) return 0u;
    return __hip_atomic_fetch_add(&bins[r >> 1], 1u << ((r & 1u) * 16u), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void range16_guard(uint32_t* bins, uint32_t q, uint32_t old,
                                              const LaunchParams& p) {
    const uint32_t r = q - p.q_lo;
    if (r >= p.q_span) return;
    const uint32_t sh = (r & 1u) * 16u;
    const uint32_t f = (old >> sh) & 0xFFFFu;
    if (f == 0x7FFFu) {
        RSS_GUARD_DELAY();
        const uint32_t at = __hip_atomic_fetch_sub(&bins[r >> 1], 0x8000u << sh, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        RSS_RECORD_MARGIN(16, kMarginHash16, (at >> sh) & 0xFFFFu);
        atomicAdd(&p.ovf[r], 1u);
    } else if (f == 0xFFFFu) {
        __hip_atomic_store(p.poison, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// HIST_RANGE8's halves.  u8 bins, four per dword: the add that returns 0x7F (its bin now
// holds 0x80) subtracts 0x80 from the bin and counts one move of 128 in p.ovf (a u32 per
// queue, summed by the partial reduce).  Unlike u16 bins, the adds in flight while that
// subtract is pending are not bounded below the field's headroom: a workgroup can hold 4096
// adds on one bin (every lane's four tuples in one queue), and a field that passes 0xFF
// carries into its neighbour.  Exactly the add that takes a field past 0xFF sees 0xFF, so
// that add raises *p.poison: the launch's bins are then discarded -- the partial reduce is
// gated on !poison and rss_range8_fallback_kernel (gated on poison) recounts the range with
// u32 bins.  Uniform and flow-like input stay far from it (a bin meets ~8 adds per workgroup
// at 131072 queues); a batch of one repeated tuple takes the fallback.
__device__ __forceinline__ uint32_t range8_add(uint32_t* bins, uint32_t q, const LaunchParams& p) {
    const uint32_t r = q - p.q_lo;  // wraps for q < q_lo
    if (r >= p.q_span) return 0u;
    return __hip_atomic_fetch_add(&bins[r >> 2], 1u << ((r & 3u) * 8u), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void range8_guard(uint32_t* bins, uint32_t q, uint32_t old,
                                             const LaunchParams& p) {
    const uint32_t r = q - p.q_lo;
    if (r >= p.q_span) return;
    const uint32_t sh = (r & 3u) * 8u;
    const uint32_t f = (old >> sh) & 0xFFu;
    if (f == 0x7Fu) {
        const uint32_t at = __hip_atomic_fetch_sub(&bins[r >> 2], 0x80u << sh, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        RSS_RECORD_MARGIN(8, kMarginHash8, (at >> sh) & 0xFFu);
        atomicAdd(&p.ovf[r], 1u);
    } else if (f == 0xFFu) {
        __hip_atomic_store(p.poison, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int kHist>
__device__ __forceinline__ void count_queue(uint32_t* bins, uint32_t q, uint32_t col,
                                            const LaunchParams& p) {
    if constexpr (kHist == HIST_PRIVATE) {
        __hip_atomic_fetch_add(&bins[q * kBinCols + col], 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (kHist == HIST_SHARED) {
        __hip_atomic_fetch_add(&bins[q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (kHist == HIST_GLOBAL) {
        atomicAdd(&p.counts[q], 1ull);
    } else if constexpr (kHist == HIST_RANGE) {
        const uint32_t r = q - p.q_lo;  // wraps for q < q_lo
        if (r < p.q_span)
            __hip_atomic_fetch_add(&bins[r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (kHist == HIST_RANGE16) {
        range16_guard(bins, q, range16_add(bins, q, p), p);
    } else if constexpr (kHist == HIST_RANGE8) {
        range8_guard(bins, q, range8_add(bins, q, p), p);
    }
}



// Streaming outputs are written once and never re-read by this kernel: use
// nontemporal stores so they do not displace the input stream in L2.
template <typename T>
__device__ __forceinline__ void stream_store(T* dst, T v) {
    __builtin_nontemporal_store(v, dst);
}

// the value a queue column of width kQWidth holds for queue q (QW_U16R: see QueueWidth)
template <int kQWidth>
__device__ __forceinline__ uint32_t column_queue(uint32_t q, const LaunchParams& p) {
    if constexpr (kQWidth == QW_U16R) return min(q - p.q_span, 0xFFFFu);  // q < q_span wraps
    return q;
}
template <int kQWidth>
constexpr int kStoreWidth = kQWidth == QW_U16R ? QW_U16 : kQWidth;

template <int kQWidth>
__device__ __forceinline__ void store_queue1(void* out, uint64_t i, uint32_t q) {
    if constexpr (kQWidth == QW_U8) {
        stream_store(static_cast<uint8_t*>(out) + i, (uint8_t)q);
    } else if constexpr (kQWidth == QW_U16) {
        stream_store(static_cast<uint16_t*>(out) + i, (uint16_t)q);
    } else {
        stream_store(static_cast<uint32_t*>(out) + i, q);
    }
}

// four consecutive queues of group g (tuples 4g .. 4g+3) as one 4/8/16-byte store
template <int kQWidth, typename Idx>
__device__ __forceinline__ void store_queue4(void* out, Idx g, uint32_t q0, uint32_t q1,
                                             uint32_t q2, uint32_t q3) {
    if constexpr (kQWidth == QW_U8) {
        stream_store(static_cast<uint32_t*>(out) + g, q0 | q1 << 8 | q2 << 16 | q3 << 24);
    } else if constexpr (kQWidth == QW_U16) {
        uint32_t* o = static_cast<uint32_t*>(out) + 2 * g;
        stream_store(o, q0 | q1 << 16);
        stream_store(o + 1, q2 | q3 << 16);
    } else {
        uint32_t* o = static_cast<uint32_t*>(out) + 4 * g;
        stream_store(o, q0);
        stream_store(o + 1, q1);
        stream_store(o + 2, q2);
        stream_store(o + 3, q3);
    }
}

// Fold a workgroup's per-queue totals (`sum_of(q)`, q < Q) into the global uint64 counts.
// Without a workspace: one atomicAdd per non-zero total (counts zeroed by the caller or by
// a hipMemsetAsync before the launch).  With one (rss_hash_device_ws, single-pass counts) the
// launch writes the batch's counts itself (overwriting, or adding when `mode &
// kFoldAccumulate`) and leaves the workspace zero for the next launch -- so a batch's counts
// need no zeroing launch before it.  Arrival fold: each workgroup adds (1 << kArrivalShift) |
// total into ws[1 + q] for every queue; the add whose returned arrival count is gridDim.x - 1
// is the queue's last, so its workgroup writes counts[q] = old sum + its own and resets
// ws[1 + q].  Every queue is finalised by one atomic round trip and needs no release/acquire:
// its count travels in the atomics on one location (the balanced tail's unit counter is
// reset in walk_rows by the launch's final claim, also one location).  Stress-tested in
// tests/test_gpu_single_pass.py.  (Rounds 2-3 used a ticket fold -- totals, a ticket, the
// last workgroup's exchanges: three serialised round trips on the last workgroup's path.)
constexpr uint32_t kFoldAccumulate = 1u;
// ws[1 + q] = (arrivals << kArrivalShift) | sum.  Sums stay below 2^44 (a launch is < 2^44
// tuples) and arrivals below 2^20 workgroups.
constexpr uint32_t kArrivalShift = 44;
constexpr unsigned long long kArrivalOne = 1ull << kArrivalShift;
constexpr unsigned long long kSumMask = kArrivalOne - 1;
// the balanced tail's unit counter: ws[Q + 1]
__host__ __device__ __forceinline__ unsigned long long* ws_tail_counter(unsigned long long* ws,
                                                                        uint32_t Q) {
    return ws + Q + 1;
}

template <typename SumOf>
__device__ __forceinline__ void fold_counts(SumOf sum_of, uint32_t Q, unsigned long long* counts,
                                            unsigned long long* ws, uint32_t mode) {
    const uint32_t tid = threadIdx.x;
    if (!ws) {
        for (uint32_t q = tid; q < Q; q += blockDim.x) {
            const uint32_t s = sum_of(q);
            if (s) atomicAdd(&counts[q], (unsigned long long)s);
        }
        return;
    }
    const bool accumulate = (mode & kFoldAccumulate) != 0;
    const unsigned long long last = (unsigned long long)gridDim.x - 1;
    for (uint32_t q = tid; q < Q; q += blockDim.x) {
        const unsigned long long add = kArrivalOne | sum_of(q);
        // the sums travel in the atomics on one word each: no fence is needed
        const unsigned long long old = atomicAdd(&ws[1 + q], add);
        if ((old >> kArrivalShift) == last) {  // every other workgroup's add is in `old`
            const unsigned long long total = (old & kSumMask) + (add & kSumMask);
            counts[q] = accumulate ? counts[q] + total : total;
            atomicExch(&ws[1 + q], 0ull);  // after every add of this launch to it
        }
    }
}

// The grid's walk over `ngroups` groups of 4 tuples (`group(g)`), one grid-stride row at a
// time: row r = groups [r * gstride, (r + 1) * gstride), workgroup w takes slot w of it.
// With `tail_rows` (single-pass launches, DESIGN.md §3 "Balanced tail") rows [0, srows) go
// statically and the last tail_rows rows are handed out in order as units of one workgroup
// slot (kBlock groups) through the workspace counter `next`, one claim per workgroup in
// flight (issued one unit ahead, broadcast through the LDS word `slot`), so the workgroups
// -- the XCDs -- that stream faster (measured: even XCDs finish ~4 % before odd ones) take
// more of the tail and every XCD ends together, while the whole grid still sweeps one
// window of the arrays at a time.  `next` is reset by the launch's final claim (below).
template <typename Group>
__device__ __forceinline__ void walk_rows(Group group, uint64_t ngroups, uint32_t tail_rows,
                                          unsigned long long* next, unsigned long long* slot) {
    const uint32_t tid = threadIdx.x;
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    if (!tail_rows) {
        for (uint64_t g = gtid; g < ngroups; g += gstride) group(g);
        return;
    }
    const uint64_t nrows = (ngroups + gstride - 1) / gstride;
    const uint64_t srows = nrows - tail_rows;  // the launcher keeps tail_rows < nrows
    // Every workgroup claims until a claim fails (returns >= the tail's units), so a launch
    // makes exactly tail units + gridDim.x claims; the one that returns the last of them is the
    // final RMW of the launch on `next` and resets it -- one location, so no fence is needed.
    const unsigned long long last_claim = (unsigned long long)tail_rows * gridDim.x + gridDim.x - 1;
    auto publish = [&](unsigned long long c) {  // tid 0
        if (c == last_claim) atomicExch(next, 0ull);
        *slot = c;
    };
    unsigned long long claim = 0;
    if (tid == 0) claim = atomicAdd(next, 1ull);  // the first tail unit, in flight meanwhile
    for (uint64_t row = 0; row < srows; ++row) group(row * gstride + gtid);  // full rows
    if (tid == 0) publish(claim);
    __syncthreads();
    const uint64_t first = srows * gridDim.x, nunits = nrows * gridDim.x;
    uint64_t u = first + *slot;
    while (u < nunits) {
        __syncthreads();  // every lane has read the slot
        if (tid == 0) claim = atomicAdd(next, 1ull);  // the next unit, during this one
        const uint64_t g = (u / gridDim.x) * gstride + (u % gridDim.x) * kBlock + tid;
        if (g < ngroups) group(g);
        if (tid == 0) publish(claim);
        __syncthreads();
        u = first + *slot;
    }
}

// Rows of a launch of `ngroups` groups on `grid` workgroups, and the tail a single-pass
// launch hands out (about a tenth; none below 16 rows, where the spread is a few us)
inline uint32_t balanced_tail_rows(uint64_t ngroups, unsigned grid) {
    const uint64_t per_row = (uint64_t)grid * kBlock;
    const uint64_t rows = (ngroups + per_row - 1) / per_row;
    return rows >= 16 ? (uint32_t)std::max<uint64_t>(1, rows / 10) : 0u;
}

// HIST_RANGE8 counts only, queues past the pass's LDS range (q >= q_span): instead of a queue
// column with every tuple's queue, each wave appends r = q - q_span to a list of its own (K
// queues per lane): a ballot per slot, the entries at the wave's running length `count` plus
// the lanes below (mbcnt), stored at 32-bit offsets from the wave's list (`list`, uniform).
// No atomic: the length is the same in every lane (sums of ballot popcounts), and a wave's
// list never exceeds its tuples (the launcher sizes resid_cap for the static walk's share of a
// wave).  The entries are exact whether or not the bins are poisoned.
constexpr uint32_t kWavesPerBlock = kBlock / 64;
__device__ __forceinline__ char* resid_list(const LaunchParams& p) {
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    return static_cast<char*>(p.resid_out) +
           ((uint64_t)blockIdx.x * kWavesPerBlock + wave) * p.resid_cap * (p.resid_u16 ? 2 : 4);
}
template <int K>
__device__ __forceinline__ void resid_append(const LaunchParams& p, char* list, uint32_t& count,
                                             const uint32_t* q) {
    // The first active lane took part in every earlier append of its wave (lanes leave the
    // walk from the top, and the < 4 tail tuples are lanes 0..2): its length is the wave's.
    // Per slot: the ballot's compare, two mbcnt and one shift-add for the address (the
    // length's byte offset stays scalar), one subtract for the entry.
    const uint32_t sh = p.resid_u16 ? 1u : 2u;
    uint32_t at = __builtin_amdgcn_readfirstlane(count) << sh;  // byte offset of the next entry
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t m = __ballot(q[k] >= p.q_span);
        if (q[k] >= p.q_span) {
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            char* dst = list + (at + (below << sh));
            if (p.resid_u16)
                *reinterpret_cast<uint16_t*>(dst) = (uint16_t)(q[k] - p.q_span);
            else
                *reinterpret_cast<uint32_t*>(dst) = q[k] - p.q_span;
        }
        at += (uint32_t)__popcll(m) << sh;
    }
    count = at >> sh;
}

// --------------------------------------------------------------- host -------
struct DeviceInfo {
    int cu_count = 0;
};

std::mutex g_dev_mutex;
std::vector<DeviceInfo> g_devices;

inline int device_info(DeviceInfo* out) {
    int dev = 0;
    RSS_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(g_dev_mutex);
    if ((int)g_devices.size() <= dev) g_devices.resize(dev + 1);
    if (g_devices[dev].cu_count == 0) {
        int cus = 0;
        RSS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        g_devices[dev].cu_count = cus > 0 ? cus : 1;
    }
    *out = g_devices[dev];
    return RSS_OK;
}

using KernelFn = void (*)(const LaunchParams);

inline bool is_pow2(uint32_t x) { return x && !(x & (x - 1)); }
inline bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

// ceil(2^64 / d) as Lemire's M = floor((2^64 - 1) / d) + 1 (wraps to 0 for d = 1,
// which still yields the correct remainder 0).
inline uint64_t magic64(uint32_t d) { return UINT64_MAX / d + 1; }
inline uint32_t magic32(uint32_t d) { return UINT32_MAX / d + 1; }

// The queues a launch can produce.  Without an indirection table queue = bucket % Q with
// bucket < H (simulator.py:96-98), so every queue is < min(H, Q); with one, < max(reta) + 1.
// Bins, the queue-width check and the counts the kernels write are sized by this; counts
// [q_eff, nqueues) of the caller's vector are always zero (zero_counts_tail).
inline uint32_t effective_queues(uint32_t htable, uint32_t nqueues, const uint32_t* reta) {
    if (reta) {
        uint32_t m = 0;
        for (uint32_t b = 0; b < htable; ++b) m = std::max(m, reta[b]);
        return m + 1;  // <= nqueues (check_reta)
    }
    return nqueues < htable ? nqueues : htable;
}

// counts[q_eff, nqueues) of a non-accumulating launch: queues no tuple can have
inline int zero_counts_tail(uint64_t* d_counts, uint32_t q_eff, uint32_t nqueues, uint32_t flags,
                     hipStream_t stream) {
    if (d_counts && q_eff < nqueues && !(flags & RSS_FLAG_ACCUMULATE))
        RSS_HIP_CHECK(hipMemsetAsync(d_counts + q_eff, 0, sizeof(uint64_t) * (nqueues - q_eff),
                                     stream));
    return RSS_OK;
}

// Modulo strategy (mask / exact 16-bit magic / exact 64-bit magic) and histogram
// placement (private LDS columns / shared LDS bins / global atomics) for H and Q.
// Returns whether H is a power of two.
inline bool setup_modes(LaunchParams* p, uint32_t htable, uint32_t nqueues, bool want_counts, int* qmode,
                 int* hist, uint32_t* bin_bytes, uint32_t bin_budget = kBinBytesMax,
                 bool allow_fast8 = true) {
    p->H = htable;
    p->Q = nqueues;
    p->h_mask = htable - 1;
    p->h_m64 = magic64(htable);
    if (nqueues >= htable) {  // bucket < htable <= nqueues: remainder is the bucket itself
        *qmode = QM_MASK;
        p->q_mask = 0xFFFFFFFFu;
    } else if (is_pow2(nqueues)) {
        *qmode = QM_MASK;
        p->q_mask = nqueues - 1;
    } else if (htable <= 65536u) {  // bucket < 2^16 and nqueues < htable <= 2^16
        *qmode = htable <= 256u && allow_fast8 ? QM_FAST8 : QM_FAST16;
        p->q_m32 = magic32(nqueues);
        p->q_m16 = 65536u / nqueues + (65536u % nqueues != 0);
    } else {
        *qmode = QM_FAST32;
        p->q_m64 = magic64(nqueues);
    }
    *bin_bytes = 0;
    if (!want_counts) {
        *hist = HIST_NONE;
    } else if ((uint64_t)nqueues * kBinCols * 4 <= bin_budget) {
        *hist = HIST_PRIVATE;
        *bin_bytes = nqueues * kBinCols * 4;
    } else if ((uint64_t)nqueues * 4 <= bin_budget) {
        *hist = HIST_SHARED;
        *bin_bytes = nqueues * 4;
    } else {
        *hist = HIST_GLOBAL;
    }
    return is_pow2(htable);
}

// An indirection table travels in the kernel arguments as u16[htable <= kRetaMax].
inline int check_reta(const uint32_t* reta, uint32_t htable, uint32_t nqueues, const char* who) {
    if (htable > kRetaMax)
        return rss_set_error(RSS_EINVAL, "%s: htable %u exceeds %u entries", who, htable, kRetaMax);
    for (uint32_t b = 0; b < htable; ++b) {
        if (reta[b] >= nqueues)
            return rss_set_error(RSS_EINVAL, "%s: reta[%u] = %u >= nqueues %u", who, b, reta[b],
                                 nqueues);
        if (reta[b] > 0xFFFFu)
            return rss_set_error(RSS_EINVAL, "%s: reta[%u] = %u exceeds 65535", who, b, reta[b]);
    }
    return RSS_OK;
}

}  // namespace

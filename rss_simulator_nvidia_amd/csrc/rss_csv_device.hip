// rss_csv_device.hip -- CSV ingest/egress on the GPU.
//
// rss_csv_hash_text runs the whole `--csv` job of the reference CLI for a CANONICAL
// file image (the rules of rss_csv.cpp, include/rss_toeplitz.h) on the device:
//
//   pd.read_csv                        rss_simulator/simulator.py:55
//   calc_hash / calc_queue_number      rss_simulator/simulator.py:74-98
//   write_statistics (both to_csv)     rss_simulator/simulator.py:100-115
//
// Only the file bytes cross PCIe: the text goes up once, the statistics file comes
// down once.  On the device (all byte work, HBM-bound, no MFMA):
//   1. newline index   -- 64 B per thread, SWAR newline count, exclusive scan, emit
//   2. row parse       -- one thread per line, the canonical scanner of rss_csv.cpp
//                         (any violation -> RSS_ENOTSUP, the caller falls back)
//   3. empty-line drop -- flag scan + scatter, only when the file has empty lines
//   4. hash            -- rss_hash_device / rss_hash_device_reta (rss_toeplitz.hip)
//   5. format          -- row lengths, exclusive scan, every thread writes its row
// The header and the per-queue count lines are built on the host (a few hundred bytes).
// rss_csv_hash_file streams a file through pinned staging and runs the same steps per
// line-aligned segment below 4 GiB (newline positions are 32-bit), so any file size works.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <type_traits>
#include <vector>

#include "rss_internal.h"
#include "rss_toeplitz.h"

namespace {

#define CSV_HIP_CHECK(expr)                                                            \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return rss_set_error(e_ == hipErrorOutOfMemory ? RSS_ENOMEM : RSS_EIO,     \
                                 "%s failed: %s", #expr, hipGetErrorString(e_));       \
    } while (0)

constexpr int kThreads = 256;        // text kernels: 4 waves per workgroup
constexpr int kChunk = 64;           // bytes of text per thread in the newline passes
constexpr int kScanItems = 16;       // elements per thread in the scan passes
constexpr int kScanTile = kThreads * kScanItems;

// --------------------------------------------------------------- scan --------
// Exclusive scan of uint32 in[n] into uint64 out[n] (three passes: tile sums, one
// workgroup over the tile sums, tile-local scan + tile offset).  *total = sum.

__device__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* lds_waves, uint64_t* block_total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) lds_waves[wave] = x;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
        const uint64_t t = lds_waves[w];
        if (w < wave) before += t;
        all += t;
    }
    __syncthreads();  // lds_waves may be reused by the caller
    if (block_total) *block_total = all;
    return before + x - v;
}

__global__ __launch_bounds__(kThreads) void scan_tile_sums(const uint32_t* __restrict__ in,
                                                           uint64_t n, uint64_t* tile_sum) {
    __shared__ uint64_t waves[kThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint64_t s = 0;
    for (int k = 0; k < kScanItems; ++k)
        if (base + k < n) s += in[base + k];
    uint64_t total;
    block_exclusive_scan(s, waves, &total);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

// one workgroup: tile_sum[0..ntiles) -> exclusive offsets in place, total at [ntiles]
__global__ __launch_bounds__(kThreads) void scan_tile_offsets(uint64_t* tile_sum, uint64_t ntiles) {
    __shared__ uint64_t waves[kThreads / 64];
    const uint64_t per = (ntiles + kThreads - 1) / kThreads;
    const uint64_t a = (uint64_t)threadIdx.x * per;
    uint64_t s = 0;
    for (uint64_t i = a; i < a + per && i < ntiles; ++i) s += tile_sum[i];
    uint64_t total;
    uint64_t run = block_exclusive_scan(s, waves, &total);
    for (uint64_t i = a; i < a + per && i < ntiles; ++i) {
        const uint64_t v = tile_sum[i];
        tile_sum[i] = run;
        run += v;
    }
    if (threadIdx.x == 0) tile_sum[ntiles] = total;
}

__global__ __launch_bounds__(kThreads) void scan_tiles(const uint32_t* __restrict__ in, uint64_t n,
                                                       const uint64_t* __restrict__ tile_off,
                                                       uint64_t* out) {
    __shared__ uint64_t waves[kThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = base + k < n ? in[base + k] : 0u;
        s += v[k];
    }
    uint64_t run = tile_off[blockIdx.x] + block_exclusive_scan(s, waves, nullptr);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        if (base + k < n) out[base + k] = run;
        run += v[k];
    }
}

// ------------------------------------------------------- newline index -------
// exact count of 0x0A bytes in a word (no false positives: the classic zero-byte
// test on x ^ 0x0A0A0A0A with the carry-free form)
__device__ __forceinline__ uint32_t newlines_in(uint32_t x) {
    const uint32_t y = x ^ 0x0A0A0A0Au;
    const uint32_t t = ((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y;
    return __popc(~t & 0x80808080u);
}

__global__ __launch_bounds__(kThreads) void count_newlines(const uint8_t* __restrict__ text,
                                                           uint64_t len, uint32_t* cnt) {
    const uint64_t t = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    const uint64_t a = t * kChunk;
    if (a >= len) return;
    uint32_t c = 0;
    if (a + kChunk <= len) {
        const uint4* p = reinterpret_cast<const uint4*>(text + a);
#pragma unroll
        for (int k = 0; k < kChunk / 16; ++k) {
            const uint4 x = p[k];
            c += newlines_in(x.x) + newlines_in(x.y) + newlines_in(x.z) + newlines_in(x.w);
        }
    } else {
        for (uint64_t i = a; i < len; ++i) c += text[i] == '\n';
    }
    cnt[t] = c;
}

__global__ __launch_bounds__(kThreads) void emit_newlines(const uint8_t* __restrict__ text,
                                                          uint64_t len,
                                                          const uint64_t* __restrict__ off,
                                                          uint32_t* pos) {
    const uint64_t t = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    const uint64_t a = t * kChunk;
    if (a >= len) return;
    uint64_t o = off[t];
    const uint64_t e = a + kChunk < len ? a + kChunk : len;
    if (e - a == kChunk) {
        const uint4* p = reinterpret_cast<const uint4*>(text + a);
#pragma unroll
        for (int k = 0; k < kChunk / 16; ++k) {
            const uint4 x = p[k];
            const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (!newlines_in(w[j])) continue;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (((w[j] >> (8 * b)) & 0xFFu) == '\n') pos[o++] = (uint32_t)(a + 16 * k + 4 * j + b);
            }
        }
    } else {
        for (uint64_t i = a; i < e; ++i)
            if (text[i] == '\n') pos[o++] = (uint32_t)i;
    }
}

// ------------------------------------------------------------ row parse ------
// Port of rss_csv.cpp's scan_uint / scan_ip / scan_row over one line [p, e) whose
// line end (and one '\r' before it) is already cut off.
__device__ __forceinline__ bool d_digit(const uint8_t* p, const uint8_t* e) {
    return p < e && (uint32_t)(*p - '0') <= 9u;
}

template <int kMaxDigits, uint32_t kMax>
__device__ __forceinline__ bool d_scan_uint(const uint8_t*& p, const uint8_t* e, uint32_t& v) {
    if (!d_digit(p, e)) return false;
    uint32_t x = (uint32_t)(*p++ - '0');
    if (x == 0) {
        v = 0;
        return !d_digit(p, e);
    }
    for (int k = 1; k < kMaxDigits && d_digit(p, e); ++k) x = x * 10 + (uint32_t)(*p++ - '0');
    if (d_digit(p, e) || x > kMax) return false;
    v = x;
    return true;
}

__device__ __forceinline__ bool d_scan_ip(const uint8_t*& p, const uint8_t* e, uint32_t& out) {
    uint32_t ip = 0;
    for (int k = 0; k < 4; ++k) {
        uint32_t octet;
        if (!d_scan_uint<3, 255>(p, e, octet)) return false;
        ip = ip << 8 | octet;
        if (k < 3) {
            if (p >= e || *p != '.') return false;
            ++p;
        }
    }
    out = ip;
    return true;
}

struct Layout {
    uint8_t col[4];
};

// one canonical row in [p, end) (line end and one '\r' already cut off)
__device__ __forceinline__ bool parse_row(const uint8_t* p, const uint8_t* end, const Layout& layout,
                                          uint32_t (&v)[4]) {
    bool ok = true;
    for (int f = 0; f < 4 && ok; ++f) {
        const int c = layout.col[f];
        ok = c < 2 ? d_scan_ip(p, end, v[c]) : d_scan_uint<5, 65535>(p, end, v[c]);
        if (ok && f < 3) {
            ok = p < end && *p == ',';
            ++p;
        }
    }
    return ok && p == end;
}

// ---- IPv6 rows: the scanner of rss_csv.cpp (scan_ip6 / scan_row6) on one line ----
// character classes of rss_csv.cpp's Hex6Table: 0..15 hex digit, kColon6, kEnd6 (',' '\r'
// '\n' or the line end), -1 anything else
constexpr int kColon6 = 16, kEnd6 = 17;

__device__ __forceinline__ int d_class6(const uint8_t* p, const uint8_t* e) {
    if (p >= e) return kEnd6;
    const uint32_t c = *p, l = c | 0x20u;
    if (c - '0' <= 9u) return (int)(c - '0');
    if (l - 'a' <= 5u) return (int)(l - 'a' + 10);
    if (c == ':') return kColon6;
    return (c == ',' || c == '\r' || c == '\n') ? kEnd6 : -1;
}

// Groups are shifted into a 128-bit accumulator; at '::' the head moves aside and the
// tail starts from zero, so the address is head << 16 * (8 - gap) | tail (no group array).
__device__ __forceinline__ bool d_scan_ip6(const uint8_t*& p, const uint8_t* e, uint32_t (&out)[4]) {
    unsigned __int128 acc = 0, head = 0;
    int ng = 0, gap = -1;
    if (p + 1 < e && p[0] == ':' && p[1] == ':') {
        gap = 0;
        p += 2;
    }
    while (!(gap >= 0 && d_class6(p, e) == kEnd6)) {
        uint32_t v = 0;
        int digits = 0, h;
        while ((h = d_class6(p, e)) >= 0 && h < 16 && digits < 4) {
            v = v << 4 | (uint32_t)h;
            ++digits;
            ++p;
        }
        if (digits == 0 || (h >= 0 && h < 16) || ng == 8) return false;
        acc = acc << 16 | v;
        ++ng;
        if (h == kEnd6) break;
        if (h != kColon6) return false;
        if (p + 1 < e && p[1] == ':') {
            if (gap >= 0) return false;
            gap = ng;
            head = acc;
            acc = 0;
            p += 2;
        } else {
            ++p;  // a single ':' must be followed by another group
        }
    }
    if (gap < 0 ? ng != 8 : ng > 7) return false;
    if (gap > 0) acc |= head << (16 * (8 - gap));
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = (uint32_t)(acc >> (96 - 32 * k));
    return true;
}

// one canonical IPv6 row in [p, end) (line end and one '\r' already cut off)
__device__ __forceinline__ bool parse_row6(const uint8_t* p, const uint8_t* end, const Layout& layout,
                                           rss_tuple6& t) {
    uint32_t a0[4] = {0, 0, 0, 0}, a1[4] = {0, 0, 0, 0}, port0 = 0, port1 = 0;
    for (int f = 0; f < 4; ++f) {
        const int c = layout.col[f];
        if (c < 2) {
            uint32_t a[4];
            if (!d_scan_ip6(p, end, a)) return false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // selects, not a dynamically indexed array
                a0[k] = c == 0 ? a[k] : a0[k];
                a1[k] = c == 1 ? a[k] : a1[k];
            }
        } else {
            uint32_t v;
            if (!d_scan_uint<5, 65535>(p, end, v)) return false;
            port0 = c == 2 ? v : port0;
            port1 = c == 3 ? v : port1;
        }
        if (f < 3) {
            if (p >= end || *p != ',') return false;
            ++p;
        }
    }
    if (p != end) return false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        t.w[k] = a0[k];
        t.w[4 + k] = a1[k];
    }
    t.w[8] = port0 << 16 | port1;
    return true;
}

// The two row families of the device path: IPv4 rows are parsed into packed 4-tuples
// and formatted from them; IPv6 rows keep the byte span of their text, which pandas
// writes back verbatim (rss_csv.cpp), plus the 36-byte tuple of rss_hash6_device.
struct Span {
    uint32_t start, len;  // line text in the segment, without its line end
};

struct RowsV4 {
    using Tuple = rss_tuple4;
    static constexpr uint32_t kParseSpan = 16384;  // 256 canonical lines <= 11.5 KiB
    __device__ static int classify(const uint8_t* p, const uint8_t* e, const Layout& layout,
                                   Tuple& t, uint32_t& len) {
        if (e > p && e[-1] == '\r') --e;
        if (e == p) return 0;
        uint32_t v[4];
        if (!parse_row(p, e, layout, v)) return 2;
        t.sip = v[0];
        t.dip = v[1];
        t.ports = v[2] << 16 | v[3];
        len = (uint32_t)(e - p);
        return 1;
    }
};

struct RowsV6 {
    using Tuple = rss_tuple6;
    static constexpr uint32_t kParseSpan = 24576;  // 256 canonical lines <= 23.3 KiB
    __device__ static int classify(const uint8_t* p, const uint8_t* e, const Layout& layout,
                                   Tuple& t, uint32_t& len) {
        if (e > p && e[-1] == '\r') --e;
        if (e == p) return 0;
        if (!parse_row6(p, e, layout, t)) return 2;
        len = (uint32_t)(e - p);
        return 1;
    }
};

// One workgroup parses 256 consecutive lines.  Their text is one contiguous span: it is
// staged into LDS with coalesced 16-byte loads and parsed from there (canonical lines fit
// Rows::kParseSpan); a longer span (only possible for non-canonical text) is parsed
// straight from global memory.  spans (IPv6 only) gets each row's text span.
template <class Rows>
__global__ __launch_bounds__(kThreads) void parse_lines(
    const uint8_t* __restrict__ text, uint64_t len, const uint32_t* __restrict__ pos,
    uint64_t nnl, uint64_t nlines, Layout layout, typename Rows::Tuple* tuples, Span* spans,
    uint32_t* is_row, unsigned long long* n_empty, unsigned long long* n_bad) {
    constexpr uint32_t kParseSpan = Rows::kParseSpan;
    __shared__ __attribute__((aligned(16))) uint8_t span[kParseSpan + 32];
    const uint64_t i0 = (uint64_t)blockIdx.x * kThreads;
    const uint64_t i = i0 + threadIdx.x;
    const uint64_t last = (i0 + kThreads < nlines ? i0 + kThreads : nlines) - 1;
    const uint64_t span_s = i0 ? (uint64_t)pos[i0 - 1] + 1 : 0;
    const uint64_t span_e = last < nnl ? (uint64_t)pos[last] : len;
    const uint64_t base = span_s & ~15ull;  // 16-B aligned copy window [base, span_e)
    const bool staged = span_e - base <= kParseSpan;
    if (staged) {
        const uint64_t chunks = (span_e - base + 15) / 16;
        for (uint64_t c = threadIdx.x; c < chunks; c += kThreads) {
            const uint64_t g = base + 16 * c;
            if (g + 16 <= len) {
                *reinterpret_cast<uint4*>(span + 16 * c) = *reinterpret_cast<const uint4*>(text + g);
            } else {
                for (uint64_t k = g; k < len; ++k) span[16 * c + (k - g)] = text[k];
            }
        }
    }
    __syncthreads();
    if (i >= nlines) return;
    const uint64_t s = i ? (uint64_t)pos[i - 1] + 1 : 0;
    const uint64_t e = i < nnl ? pos[i] : len;
    typename Rows::Tuple t;
    uint32_t row_len = 0;
    // 0 = empty line, 1 = row, 2 = not canonical; the two branches keep LDS and global
    // addressing apart (ds_read vs global_load, no flat loads)
    const int kind = staged ? Rows::classify(span + (s - base), span + (e - base), layout, t, row_len)
                            : Rows::classify(text + s, text + e, layout, t, row_len);
    if (kind == 0) {  // "\n", "\r\n" or a final "\r": skipped like skip_empty_line
        is_row[i] = 0;
        atomicAdd(n_empty, 1ull);
        return;
    }
    if (kind == 2) {
        atomicAdd(n_bad, 1ull);
        is_row[i] = 0;
        return;
    }
    is_row[i] = 1;
    tuples[i] = t;
    if (spans) spans[i] = Span{(uint32_t)s, row_len};
}

template <class Tuple>
__global__ __launch_bounds__(kThreads) void compact_rows(const Tuple* __restrict__ in,
                                                         const Span* __restrict__ in_spans,
                                                         const uint32_t* __restrict__ is_row,
                                                         const uint64_t* __restrict__ slot,
                                                         uint64_t nlines, Tuple* out,
                                                         Span* out_spans) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= nlines || !is_row[i]) return;
    out[slot[i]] = in[i];
    if (in_spans) out_spans[slot[i]] = in_spans[i];
}

// --------------------------------------------------------------- format ------
__device__ __forceinline__ uint32_t d_uint_len(uint32_t v) {
    return 1 + (v >= 10u) + (v >= 100u) + (v >= 1000u) + (v >= 10000u) + (v >= 100000u) +
           (v >= 1000000u) + (v >= 10000000u) + (v >= 100000000u) + (v >= 1000000000u);
}

__device__ __forceinline__ uint32_t d_ip_len(uint32_t ip) {
    return d_uint_len(ip >> 24) + d_uint_len((ip >> 16) & 0xFFu) + d_uint_len((ip >> 8) & 0xFFu) +
           d_uint_len(ip & 0xFFu) + 3;
}

__device__ __forceinline__ uint8_t* d_put_uint(uint8_t* p, uint32_t v) {
    const uint32_t n = d_uint_len(v);
    for (uint32_t k = n; k > 0; --k) {
        p[k - 1] = (uint8_t)('0' + v % 10u);
        v /= 10u;
    }
    return p + n;
}

__device__ __forceinline__ uint8_t* d_put_ip(uint8_t* p, uint32_t ip) {
    for (int k = 3; k >= 0; --k) {
        p = d_put_uint(p, (ip >> (8 * k)) & 0xFFu);
        if (k) *p++ = '.';
    }
    return p;
}

__global__ __launch_bounds__(kThreads) void row_lengths(const rss_tuple4* __restrict__ t,
                                                        const uint32_t* __restrict__ hash,
                                                        const uint32_t* __restrict__ queue,
                                                        uint64_t n, uint32_t* len) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const rss_tuple4 r = t[i];
    len[i] = d_ip_len(r.sip) + d_ip_len(r.dip) + d_uint_len(r.ports >> 16) +
             d_uint_len(r.ports & 0xFFFFu) + d_uint_len(hash[i]) + d_uint_len(queue[i]) + 6;
}

// One workgroup formats 256 consecutive rows.  Their output is one contiguous span
// [g0, g1): each thread writes its row into an LDS image of the span laid out on the
// global 16-byte grid, then the workgroup stores the whole 16-byte chunks with coalesced
// 16-byte stores and the (at most two) partial chunks at the span's ends byte by byte,
// so neighbouring workgroups never write the same bytes.
constexpr uint32_t kMaxRowBytes = 15 + 1 + 15 + 1 + 5 + 1 + 5 + 1 + 10 + 1 + 10 + 1;  // 66

__global__ __launch_bounds__(kThreads) void write_rows(const rss_tuple4* __restrict__ t,
                                                       const uint32_t* __restrict__ hash,
                                                       const uint32_t* __restrict__ queue,
                                                       uint64_t n, Layout layout,
                                                       const uint64_t* __restrict__ off,
                                                       uint64_t total, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t img[kThreads * kMaxRowBytes + 32];
    const uint64_t r0 = (uint64_t)blockIdx.x * kThreads;
    const uint64_t i = r0 + threadIdx.x;
    const uint64_t g0 = off[r0];
    const uint64_t g1 = r0 + kThreads < n ? off[r0 + kThreads] : total;
    const uint64_t base = g0 & ~15ull;
    if (i < n) {
        const rss_tuple4 r = t[i];
        const uint32_t col[4] = {r.sip, r.dip, r.ports >> 16, r.ports & 0xFFFFu};
        uint8_t* w = img + (off[i] - base);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const int c = layout.col[f];
            w = c < 2 ? d_put_ip(w, col[c]) : d_put_uint(w, col[c]);
            *w++ = ',';
        }
        w = d_put_uint(w, hash[i]);
        *w++ = ',';
        w = d_put_uint(w, queue[i]);
        *w = '\n';
    }
    __syncthreads();
    const uint64_t a16 = (g0 + 15) & ~15ull, b16 = g1 & ~15ull;
    if (a16 >= b16) {  // the span lies inside one or two 16-B chunks
        for (uint64_t p = g0 + threadIdx.x; p < g1; p += kThreads) out[p] = img[p - base];
        return;
    }
    if (threadIdx.x < a16 - g0) out[g0 + threadIdx.x] = img[g0 + threadIdx.x - base];
    if (threadIdx.x < g1 - b16) out[b16 + threadIdx.x] = img[b16 + threadIdx.x - base];
    const uint4* src = reinterpret_cast<const uint4*>(img + (a16 - base));
    uint4* dst = reinterpret_cast<uint4*>(out + a16);
    for (uint64_t c = threadIdx.x; c < (b16 - a16) / 16; c += kThreads) dst[c] = src[c];
}

// IPv6 rows: the row's own text (pandas writes the address strings back verbatim),
// then ",hash,queue\n".  Same LDS-image scheme as write_rows.
constexpr uint32_t kMaxRow6Bytes = 39 + 1 + 39 + 1 + 5 + 1 + 5 + 1 + 10 + 1 + 10 + 1;  // 114

__global__ __launch_bounds__(kThreads) void row_lengths6(const Span* __restrict__ spans,
                                                         const uint32_t* __restrict__ hash,
                                                         const uint32_t* __restrict__ queue,
                                                         uint64_t n, uint32_t* len) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    len[i] = spans[i].len + d_uint_len(hash[i]) + d_uint_len(queue[i]) + 3;
}

__global__ __launch_bounds__(kThreads) void write_rows6(const uint8_t* __restrict__ text,
                                                        const Span* __restrict__ spans,
                                                        const uint32_t* __restrict__ hash,
                                                        const uint32_t* __restrict__ queue,
                                                        uint64_t n, const uint64_t* __restrict__ off,
                                                        uint64_t total, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t img[kThreads * kMaxRow6Bytes + 32];
    const uint64_t r0 = (uint64_t)blockIdx.x * kThreads;
    const uint64_t i = r0 + threadIdx.x;
    const uint64_t g0 = off[r0];
    const uint64_t g1 = r0 + kThreads < n ? off[r0 + kThreads] : total;
    const uint64_t base = g0 & ~15ull;
    if (i < n) {
        const Span sp = spans[i];
        uint8_t* w = img + (off[i] - base);
        const uint8_t* src = text + sp.start;
        for (uint32_t k = 0; k < sp.len; ++k) w[k] = src[k];
        w += sp.len;
        *w++ = ',';
        w = d_put_uint(w, hash[i]);
        *w++ = ',';
        w = d_put_uint(w, queue[i]);
        *w = '\n';
    }
    __syncthreads();
    const uint64_t a16 = (g0 + 15) & ~15ull, b16 = g1 & ~15ull;
    if (a16 >= b16) {
        for (uint64_t p = g0 + threadIdx.x; p < g1; p += kThreads) out[p] = img[p - base];
        return;
    }
    if (threadIdx.x < a16 - g0) out[g0 + threadIdx.x] = img[g0 + threadIdx.x - base];
    if (threadIdx.x < g1 - b16) out[b16 + threadIdx.x] = img[b16 + threadIdx.x - base];
    const uint4* src = reinterpret_cast<const uint4*>(img + (a16 - base));
    uint4* dst = reinterpret_cast<uint4*>(out + a16);
    for (uint64_t c = threadIdx.x; c < (b16 - a16) / 16; c += kThreads) dst[c] = src[c];
}

// ---------------------------------------------------------------- host -------
inline unsigned blocks_for(uint64_t n, uint64_t per_block) {
    return (unsigned)((n + per_block - 1) / per_block);
}

// Device allocations of one call, released on every exit path: back to the context's pool
// (rss_ctx::csv_pool), where the next call finds them, rather than to hipFree.  A fresh
// multi-GB hipMalloc maps new pages -- 10-25 ms of a 120 ms file job (RSS_CSV_TIMING) --
// while a pooled block costs nothing.  The pool is trimmed to kPoolBytes after every call
// (largest blocks first) and emptied when an allocation runs out of memory.  Reuse is
// stream-ordered: every call on a context runs on its stream[0].
constexpr size_t kPoolBytes = 8ull << 30;

void trim_pool(rss_ctx* ctx, size_t cap) {
    auto& pool = ctx->csv_pool;
    size_t total = 0;
    for (const auto& b : pool) total += b.second;
    while (total > cap && !pool.empty()) {
        size_t big = 0;
        for (size_t k = 1; k < pool.size(); ++k)
            if (pool[k].second > pool[big].second) big = k;
        (void)hipFree(pool[big].first);
        total -= pool[big].second;
        pool.erase(pool.begin() + big);
    }
}

struct DeviceBuffers {
    explicit DeviceBuffers(rss_ctx* ctx) : ctx_(ctx) {}
    DeviceBuffers(const DeviceBuffers&) = delete;
    DeviceBuffers& operator=(const DeviceBuffers&) = delete;
    ~DeviceBuffers() {
        for (const auto& b : blocks_) ctx_->csv_pool.push_back(b);
        trim_pool(ctx_, kPoolBytes);
    }
    template <typename T>
    int alloc(T** out, uint64_t count) {
        const size_t bytes = count ? count * sizeof(T) : 1;
        // best fit among pooled blocks no more than twice (+1 MiB) the request
        auto& pool = ctx_->csv_pool;
        size_t pick = pool.size();
        for (size_t k = 0; k < pool.size(); ++k)
            if (pool[k].second >= bytes && pool[k].second <= 2 * bytes + (1u << 20) &&
                (pick == pool.size() || pool[k].second < pool[pick].second))
                pick = k;
        if (pick < pool.size()) {
            blocks_.push_back(pool[pick]);
            pool.erase(pool.begin() + pick);
            *out = static_cast<T*>(blocks_.back().first);
            return RSS_OK;
        }
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipErrorOutOfMemory && !pool.empty()) {
            (void)hipGetLastError();
            trim_pool(ctx_, 0);
            e = hipMalloc(&p, bytes);
        }
        if (e != hipSuccess)
            return rss_set_error(e == hipErrorOutOfMemory ? RSS_ENOMEM : RSS_EIO,
                                 "rss_csv: hipMalloc(%llu B): %s", (unsigned long long)bytes,
                                 hipGetErrorString(e));
        blocks_.emplace_back(p, bytes);
        *out = static_cast<T*>(p);
        return RSS_OK;
    }

  private:
    rss_ctx* ctx_;
    std::vector<std::pair<void*, size_t>> blocks_;
};

int exclusive_scan(const uint32_t* in, uint64_t n, uint64_t* out, uint64_t* h_total,
                   DeviceBuffers& buf, hipStream_t s) {
    const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
    uint64_t* tiles;
    int rc = buf.alloc(&tiles, ntiles + 1);
    if (rc) return rc;
    if (n) {
        hipLaunchKernelGGL(scan_tile_sums, dim3((unsigned)ntiles), dim3(kThreads), 0, s, in, n, tiles);
        hipLaunchKernelGGL(scan_tile_offsets, dim3(1), dim3(kThreads), 0, s, tiles, ntiles);
        hipLaunchKernelGGL(scan_tiles, dim3((unsigned)ntiles), dim3(kThreads), 0, s, in, n, tiles, out);
        CSV_HIP_CHECK(hipGetLastError());
        CSV_HIP_CHECK(hipMemcpyAsync(h_total, tiles + ntiles, sizeof(uint64_t),
                                     hipMemcpyDeviceToHost, s));
        CSV_HIP_CHECK(hipStreamSynchronize(s));
    } else {
        *h_total = 0;
    }
    return RSS_OK;
}

// One CSV job on the device: the body text (uploaded by the caller into text()) ->
// rows -> hash / queue / counts -> formatted rows.  Buffers live until destruction.
// Rows = RowsV4 (rss_hash_device, rows re-formatted from the tuples) or RowsV6
// (rss_hash6_device, rows copied from their text spans).
template <class Rows>
class CsvJob {
  public:
    static constexpr bool kV6 = std::is_same<Rows, RowsV6>::value;
    using Tuple = typename Rows::Tuple;
    using Key = typename std::conditional<kV6, rss_key6, rss_key>::type;

    CsvJob(rss_ctx* ctx, const rss_csv_layout& layout, uint64_t blen)
        : s_(ctx->stream[0]), blen_(blen), buf_(ctx) {
        memcpy(lay_.col, layout.field_column, 4);
    }
    int alloc_text() { return buf_.alloc(&d_text_, blen_); }
    uint8_t* text() const { return d_text_; }
    // a segment's text may end before the allocated capacity (rss_csv_hash_file)
    void set_text_len(uint64_t len) { blen_ = len; }

    // newline index + parse (+ empty-line drop); RSS_ENOTSUP if not canonical
    int parse() {
        int rc;
        const uint64_t nchunks = (blen_ + kChunk - 1) / kChunk;
        uint32_t* d_cnt;
        uint64_t* d_cnt_off;
        if ((rc = buf_.alloc(&d_cnt, nchunks)) || (rc = buf_.alloc(&d_cnt_off, nchunks))) return rc;
        hipLaunchKernelGGL(count_newlines, dim3(blocks_for(nchunks, kThreads)), dim3(kThreads), 0,
                           s_, d_text_, blen_, d_cnt);
        CSV_HIP_CHECK(hipGetLastError());
        uint64_t nnl;
        if ((rc = exclusive_scan(d_cnt, nchunks, d_cnt_off, &nnl, buf_, s_))) return rc;
        uint32_t* d_pos;
        if ((rc = buf_.alloc(&d_pos, nnl))) return rc;
        hipLaunchKernelGGL(emit_newlines, dim3(blocks_for(nchunks, kThreads)), dim3(kThreads), 0,
                           s_, d_text_, blen_, d_cnt_off, d_pos);
        CSV_HIP_CHECK(hipGetLastError());
        uint32_t last_nl = 0;
        if (nnl)
            CSV_HIP_CHECK(hipMemcpyAsync(&last_nl, d_pos + nnl - 1, 4, hipMemcpyDeviceToHost, s_));
        CSV_HIP_CHECK(hipStreamSynchronize(s_));
        const uint64_t tail_start = nnl ? (uint64_t)last_nl + 1 : 0;
        const uint64_t nlines = nnl + (tail_start < blen_ ? 1 : 0);

        Tuple* d_lines;
        Span* d_line_spans = nullptr;
        uint32_t* d_is_row;
        unsigned long long* d_stat;  // [0] empty lines, [1] non-canonical lines
        if ((rc = buf_.alloc(&d_lines, nlines)) || (rc = buf_.alloc(&d_is_row, nlines)) ||
            (rc = buf_.alloc(&d_stat, 2)) || (kV6 && (rc = buf_.alloc(&d_line_spans, nlines))))
            return rc;
        CSV_HIP_CHECK(hipMemsetAsync(d_stat, 0, 2 * sizeof(unsigned long long), s_));
        if (nlines)
            hipLaunchKernelGGL(parse_lines<Rows>, dim3(blocks_for(nlines, kThreads)), dim3(kThreads),
                               0, s_, d_text_, blen_, d_pos, nnl, nlines, lay_, d_lines,
                               d_line_spans, d_is_row, d_stat, d_stat + 1);
        CSV_HIP_CHECK(hipGetLastError());
        unsigned long long stat[2];
        CSV_HIP_CHECK(hipMemcpyAsync(stat, d_stat, sizeof stat, hipMemcpyDeviceToHost, s_));
        CSV_HIP_CHECK(hipStreamSynchronize(s_));
        if (stat[1])
            return rss_set_error(RSS_ENOTSUP, "rss_csv: %llu non-canonical rows", stat[1]);
        n_ = nlines - stat[0];
        if (n_ == 0) return rss_set_error(RSS_ENOTSUP, "rss_csv: no data rows");
        d_tuples_ = d_lines;
        d_spans_ = d_line_spans;
        if (stat[0]) {
            uint64_t* d_slot;
            uint64_t kept;
            if ((rc = buf_.alloc(&d_slot, nlines)) || (rc = buf_.alloc(&d_tuples_, n_)) ||
                (kV6 && (rc = buf_.alloc(&d_spans_, n_))))
                return rc;
            if ((rc = exclusive_scan(d_is_row, nlines, d_slot, &kept, buf_, s_))) return rc;
            hipLaunchKernelGGL(compact_rows<Tuple>, dim3(blocks_for(nlines, kThreads)),
                               dim3(kThreads), 0, s_, d_lines, d_line_spans, d_is_row, d_slot,
                               nlines, d_tuples_, d_spans_);
            CSV_HIP_CHECK(hipGetLastError());
        }
        return RSS_OK;
    }

    int hash(const Key* key, uint32_t htable, uint32_t nqueues, const uint32_t* reta,
             bool want_rows, uint64_t* h_counts) {
        int rc;
        uint64_t* d_counts;
        if ((rc = buf_.alloc(&d_counts, nqueues))) return rc;
        if (want_rows && ((rc = buf_.alloc(&d_hash_, n_)) || (rc = buf_.alloc(&d_queue_, n_))))
            return rc;
        if constexpr (kV6)
            rc = reta ? rss_hash6_device_reta(key, d_tuples_, n_, htable, reta, nqueues, d_hash_,
                                              d_queue_, d_counts, 0, s_)
                      : rss_hash6_device(key, d_tuples_, n_, htable, nqueues, d_hash_, d_queue_,
                                         d_counts, 0, s_);
        else
            rc = reta ? rss_hash_device_reta(key, d_tuples_, n_, htable, reta, nqueues, d_hash_,
                                             d_queue_, d_counts, 0, s_)
                      : rss_hash_device(key, d_tuples_, n_, htable, nqueues, d_hash_, d_queue_,
                                        d_counts, 0, s_);
        if (rc) return rc;
        CSV_HIP_CHECK(hipMemcpyAsync(h_counts, d_counts, sizeof(uint64_t) * nqueues,
                                     hipMemcpyDeviceToHost, s_));
        CSV_HIP_CHECK(hipStreamSynchronize(s_));
        return RSS_OK;
    }

    // the data rows of the statistics file -> out() [0, rows_bytes())
    int format() {
        int rc;
        uint32_t* d_len;
        uint64_t* d_off;
        if ((rc = buf_.alloc(&d_len, n_)) || (rc = buf_.alloc(&d_off, n_))) return rc;
        if constexpr (kV6)
            hipLaunchKernelGGL(row_lengths6, dim3(blocks_for(n_, kThreads)), dim3(kThreads), 0, s_,
                               d_spans_, d_hash_, d_queue_, n_, d_len);
        else
            hipLaunchKernelGGL(row_lengths, dim3(blocks_for(n_, kThreads)), dim3(kThreads), 0, s_,
                               d_tuples_, d_hash_, d_queue_, n_, d_len);
        CSV_HIP_CHECK(hipGetLastError());
        if ((rc = exclusive_scan(d_len, n_, d_off, &rows_bytes_, buf_, s_))) return rc;
        if ((rc = buf_.alloc(&d_out_, rows_bytes_))) return rc;
        if constexpr (kV6)
            hipLaunchKernelGGL(write_rows6, dim3(blocks_for(n_, kThreads)), dim3(kThreads), 0, s_,
                               d_text_, d_spans_, d_hash_, d_queue_, n_, d_off, rows_bytes_, d_out_);
        else
            hipLaunchKernelGGL(write_rows, dim3(blocks_for(n_, kThreads)), dim3(kThreads), 0, s_,
                               d_tuples_, d_hash_, d_queue_, n_, lay_, d_off, rows_bytes_, d_out_);
        CSV_HIP_CHECK(hipGetLastError());
        return RSS_OK;
    }

    uint64_t rows() const { return n_; }
    uint64_t rows_bytes() const { return rows_bytes_; }
    const uint8_t* out() const { return d_out_; }

  private:
    hipStream_t s_;
    uint64_t blen_;
    Layout lay_;
    DeviceBuffers buf_;
    uint8_t* d_text_ = nullptr;
    Tuple* d_tuples_ = nullptr;
    Span* d_spans_ = nullptr;
    uint32_t* d_hash_ = nullptr;
    uint32_t* d_queue_ = nullptr;
    uint8_t* d_out_ = nullptr;
    uint64_t n_ = 0, rows_bytes_ = 0;
};

template <class Key>
int check_args(const Key* key, uint32_t htable, uint32_t nqueues) {
    if (!key) return rss_set_error(RSS_EINVAL, "rss_csv: key is NULL");
    if (htable < 1 || nqueues < 1)
        return rss_set_error(RSS_EINVAL, "rss_csv: htable (%u) and nqueues (%u) must be >= 1",
                             htable, nqueues);
    if (key->len < RSS_KEY_MIN_BYTES) return rss_set_error(RSS_EINVAL, "rss_csv: key not prepared");
    return RSS_OK;
}

constexpr size_t kStageBytes = 32u << 20;  // pinned staging per buffer (file I/O)

// rss_csv_hash_file splits bodies into line-aligned segments below the 32-bit newline
// positions' 4 GiB: 3 GiB by default; RSS_CSV_SEGMENT_BYTES (>= 2 staging buffers + 4 KiB)
// lowers it, which the tests use to exercise the segmented path on small files.
uint64_t segment_bytes() {
    uint64_t seg = 3ull << 30;
    if (const char* env = getenv("RSS_CSV_SEGMENT_BYTES")) {
        const unsigned long long v = strtoull(env, nullptr, 10);
        if (v) seg = v;
    }
    const uint64_t lo = 2 * (uint64_t)kStageBytes + 4096, hi = 0xFFFFFFFFull - 1;
    return seg < lo ? lo : (seg > hi ? hi : seg);
}

int reserve_stage(rss_ctx* ctx) {
    if (ctx->stage_bytes) return RSS_OK;
    for (int b = 0; b < 2; ++b) {
        CSV_HIP_CHECK(hipHostMalloc(&ctx->stage[b], kStageBytes, hipHostMallocDefault));
        CSV_HIP_CHECK(hipEventCreateWithFlags(&ctx->stage_done[b], hipEventDisableTiming));
    }
    ctx->stage_bytes = kStageBytes;
    return RSS_OK;
}

// full pread / write loops (EINTR-safe)
bool read_all(int fd, char* dst, size_t len, uint64_t off) {
    while (len) {
        const ssize_t r = pread(fd, dst, len, (off_t)off);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        dst += r;
        len -= (size_t)r;
        off += (uint64_t)r;
    }
    return true;
}

// pread of [off, off + len) split over up to kReadThreads threads: page-cache reads scale
// with threads (one thread ≈20 GB/s, four ≈60 GB/s on the GPU box; tools/io_probe.py), so
// the file read stops being slower than the PCIe upload it feeds.  Writes do not scale
// (≈10 GB/s from any number of threads) and stay single-threaded.
constexpr int kReadThreads = 8;
constexpr size_t kReadPiece = 4u << 20;

bool read_parallel(int fd, char* dst, size_t len, uint64_t off) {
    const size_t pieces = (len + kReadPiece - 1) / kReadPiece;
    const int nt = (int)(pieces < (size_t)kReadThreads ? pieces : (size_t)kReadThreads);
    if (nt <= 1) return read_all(fd, dst, len, off);
    std::atomic<bool> ok{true};
    std::vector<std::thread> pool;
    pool.reserve(nt);
    for (int t = 0; t < nt; ++t)
        pool.emplace_back([&, t] {
            const size_t a = len * t / nt, b = len * (t + 1) / nt;
            if (!read_all(fd, dst + a, b - a, off + a)) ok = false;
        });
    for (auto& th : pool) th.join();
    return ok;
}

bool write_all(int fd, const char* src, size_t len) {
    while (len) {
        const ssize_t w = write(fd, src, len);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) return false;
        src += w;
        len -= (size_t)w;
    }
    return true;
}

// RSS_CSV_TIMING=1: rss_csv_hash_file prints its phase times to stderr (diagnostics)
class PhaseTimer {
  public:
    explicit PhaseTimer(const char* who) : who_(who), on_(getenv("RSS_CSV_TIMING") != nullptr) {
        last_ = std::chrono::steady_clock::now();
    }
    void mark(const char* phase) {
        if (!on_) return;
        const auto now = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(now - last_).count();
        last_ = now;
        const int n = snprintf(line_ + used_, sizeof line_ - used_, " %s=%.2fms", phase, ms);
        if (n > 0 && used_ + n < (int)sizeof line_) used_ += n;
    }
    ~PhaseTimer() {  // runs after the device buffers of the call are freed
        if (!on_) return;
        mark("free");
        fprintf(stderr, "%s:%s\n", who_, line_);
    }

  private:
    const char* who_;
    bool on_;
    std::chrono::steady_clock::time_point last_;
    char line_[512] = {0};
    int used_ = 0;
};

struct Fd {
    int fd = -1;
    ~Fd() {
        if (fd >= 0) close(fd);
    }
};

template <class Rows>
int csv_hash_text_locked(const char* who, rss_ctx* ctx, const typename CsvJob<Rows>::Key* key,
                         const char* text, size_t len, uint32_t htable, uint32_t nqueues,
                         const uint32_t* reta, uint32_t flags, const char** out, size_t* out_len,
                         uint64_t* counts, size_t* n_rows) {
    if (!ctx || !text || !counts || !n_rows)
        return rss_set_error(RSS_EINVAL, "%s: NULL argument", who);
    const bool want_file = !(flags & RSS_CSV_COUNTS_ONLY);
    if (want_file && (!out || !out_len))
        return rss_set_error(RSS_EINVAL, "%s: out / out_len NULL", who);
    int rc = check_args(key, htable, nqueues);
    if (rc) return rc;
    *n_rows = 0;
    rss_csv_layout layout;
    size_t body_off;
    if (!rss_csv_header(text, len, &layout, &body_off))
        return rss_set_error(RSS_ENOTSUP, "%s: header is not canonical", who);
    const uint64_t blen = len - body_off;
    if (blen >= 0xFFFFFFFFull)  // newline positions are 32-bit
        return rss_set_error(RSS_ENOTSUP, "%s: body of %llu B exceeds 4 GiB", who,
                             (unsigned long long)blen);
    CSV_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream[0];
    CsvJob<Rows> job(ctx, layout, blen);
    if ((rc = job.alloc_text())) return rc;
    CSV_HIP_CHECK(hipMemcpyAsync(job.text(), text + body_off, blen, hipMemcpyHostToDevice, s));
    if ((rc = job.parse()) || (rc = job.hash(key, htable, nqueues, reta, want_file, counts)))
        return rc;
    *n_rows = job.rows();
    if (!want_file) return RSS_OK;
    if ((rc = job.format())) return rc;
    ctx->csv_out.resize(rss_csv_prefix_bound(nqueues) + job.rows_bytes());
    const size_t prefix = rss_csv_format_prefix(counts, nqueues, &layout, ctx->csv_out.data());
    CSV_HIP_CHECK(hipMemcpyAsync(ctx->csv_out.data() + prefix, job.out(), job.rows_bytes(),
                                 hipMemcpyDeviceToHost, s));
    CSV_HIP_CHECK(hipStreamSynchronize(s));
    *out = ctx->csv_out.data();
    *out_len = prefix + job.rows_bytes();
    return RSS_OK;
}

template <class Rows>
int csv_hash_file_locked(const char* who, rss_ctx* ctx, const typename CsvJob<Rows>::Key* key,
                         const char* in_path, const char* out_path, uint32_t htable, uint32_t nqueues,
                         const uint32_t* reta, uint32_t flags, uint64_t* counts, size_t* n_rows) {
    if (!ctx || !in_path || !counts || !n_rows)
        return rss_set_error(RSS_EINVAL, "%s: NULL argument", who);
    const bool want_file = !(flags & RSS_CSV_COUNTS_ONLY);
    if (want_file && !out_path)
        return rss_set_error(RSS_EINVAL, "%s: out_path NULL", who);
    int rc = check_args(key, htable, nqueues);
    if (rc) return rc;
    *n_rows = 0;
    PhaseTimer timer(who);
    CSV_HIP_CHECK(hipSetDevice(ctx->device));
    if ((rc = reserve_stage(ctx))) return rc;
    hipStream_t s = ctx->stream[0];
    Fd in;
    in.fd = open(in_path, O_RDONLY);
    struct stat st;
    if (in.fd < 0 || fstat(in.fd, &st) != 0 || !S_ISREG(st.st_mode))
        return rss_set_error(RSS_ENOTSUP, "%s: cannot read %s", who, in_path);
    const uint64_t len = (uint64_t)st.st_size;
    // the header must sit in the first staging buffer (a canonical one is < 64 B)
    const size_t first = (size_t)(len < kStageBytes ? len : kStageBytes);
    if (!read_parallel(in.fd, ctx->stage[0], first, 0))
        return rss_set_error(RSS_ENOTSUP, "%s: cannot read %s", who, in_path);
    rss_csv_layout layout;
    size_t body_off;
    if (!rss_csv_header(ctx->stage[0], first, &layout, &body_off))
        return rss_set_error(RSS_ENOTSUP, "%s: header is not canonical", who);
    const uint64_t blen = len - body_off;

    // Stream the body up in line-aligned segments (each below 4 GiB: newline positions
    // are 32-bit): the pread of chunk k+1 into one pinned buffer overlaps the upload of
    // chunk k from the other.  When the next chunk might not fit the current segment,
    // this chunk is cut after its last newline and the rest opens the next segment.
    // Every segment is parsed, hashed (counts summed here) and formatted in HBM; the rows
    // are written only after the last one, since the file starts with the counts.
    const uint64_t seg_cap = segment_bytes();
    std::vector<std::unique_ptr<CsvJob<Rows>>> jobs;
    std::vector<uint64_t> seg_counts(nqueues);
    memset(counts, 0, sizeof(uint64_t) * nqueues);
    uint64_t body_left = blen, dev_pos = 0;
    auto open_segment = [&]() -> int {
        jobs.emplace_back(new CsvJob<Rows>(ctx, layout, body_left < seg_cap ? body_left : seg_cap));
        dev_pos = 0;
        return jobs.back()->alloc_text();
    };
    auto close_segment = [&]() -> int {
        CsvJob<Rows>& job = *jobs.back();
        job.set_text_len(dev_pos);
        int r;
        if ((r = job.parse()) ||
            (r = job.hash(key, htable, nqueues, reta, want_file, seg_counts.data())))
            return r;
        for (uint32_t q = 0; q < nqueues; ++q) counts[q] += seg_counts[q];
        *n_rows += job.rows();
        return want_file ? job.format() : RSS_OK;
    };
    auto upload = [&](const char* src, size_t bytes) -> int {
        if (!bytes) return RSS_OK;
        CSV_HIP_CHECK(hipMemcpyAsync(jobs.back()->text() + dev_pos, src, bytes,
                                     hipMemcpyHostToDevice, s));
        dev_pos += bytes;
        body_left -= bytes;
        return RSS_OK;
    };
    if (blen && (rc = open_segment())) return rc;
    uint64_t file_pos = 0;
    for (int k = 0; file_pos < len; ++k) {
        const int b = k & 1;
        size_t got;
        if (k == 0) {
            got = first;
        } else {
            CSV_HIP_CHECK(hipEventSynchronize(ctx->stage_done[b]));  // buffer b is free again
            got = (size_t)(len - file_pos < kStageBytes ? len - file_pos : kStageBytes);
            if (!read_parallel(in.fd, ctx->stage[b], got, file_pos))
                return rss_set_error(RSS_EIO, "%s: read of %s failed", who, in_path);
        }
        const char* chunk = ctx->stage[b] + (k == 0 ? body_off : 0);
        size_t bytes = got - (k == 0 ? body_off : 0);
        file_pos += got;
        if (bytes && file_pos < len && dev_pos + bytes + kStageBytes > seg_cap) {
            // cut after this chunk's last newline; the remainder opens the next segment
            const char* nl = static_cast<const char*>(memrchr(chunk, '\n', bytes));
            if (!nl)
                return rss_set_error(RSS_ENOTSUP, "%s: a line spans %zu B", who,
                                     bytes);
            const size_t head = (size_t)(nl - chunk) + 1;
            if ((rc = upload(chunk, head)) || (rc = close_segment()) || (rc = open_segment()))
                return rc;
            chunk += head;
            bytes -= head;
        }
        if ((rc = upload(chunk, bytes))) return rc;
        CSV_HIP_CHECK(hipEventRecord(ctx->stage_done[b], s));
    }
    if (jobs.empty()) return rss_set_error(RSS_ENOTSUP, "rss_csv: no data rows");
    timer.mark("read+upload");
    if ((rc = close_segment())) return rc;
    timer.mark("parse+hash+format");
    if (!want_file) return RSS_OK;
    Fd outf;
    outf.fd = open(out_path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
    if (outf.fd < 0)  // the pandas path raises the reference's error for this path
        return rss_set_error(RSS_ENOTSUP, "%s: cannot create %s", who, out_path);
    {
        std::vector<char> prefix(rss_csv_prefix_bound(nqueues));
        const size_t plen = rss_csv_format_prefix(counts, nqueues, &layout, prefix.data());
        if (!write_all(outf.fd, prefix.data(), plen))
            return rss_set_error(RSS_EIO, "%s: write to %s failed", who, out_path);
    }
    timer.mark("open+prefix");
    // stream every segment's rows down: chunk k+1 copies into one pinned buffer while
    // chunk k is written from the other
    for (const auto& job : jobs) {
        const uint64_t total = job->rows_bytes();
        const uint64_t nchunks = (total + kStageBytes - 1) / kStageBytes;
        auto issue = [&](uint64_t k) -> int {
            const uint64_t a = k * kStageBytes;
            const size_t bytes = (size_t)(total - a < kStageBytes ? total - a : kStageBytes);
            CSV_HIP_CHECK(hipMemcpyAsync(ctx->stage[k & 1], job->out() + a, bytes,
                                         hipMemcpyDeviceToHost, s));
            CSV_HIP_CHECK(hipEventRecord(ctx->stage_done[k & 1], s));
            return RSS_OK;
        };
        if (nchunks && (rc = issue(0))) return rc;
        for (uint64_t k = 0; k < nchunks; ++k) {
            CSV_HIP_CHECK(hipEventSynchronize(ctx->stage_done[k & 1]));
            if (k + 1 < nchunks && (rc = issue(k + 1))) return rc;
            const uint64_t a = k * kStageBytes;
            const size_t bytes = (size_t)(total - a < kStageBytes ? total - a : kStageBytes);
            if (!write_all(outf.fd, ctx->stage[k & 1], bytes))
                return rss_set_error(RSS_EIO, "%s: write to %s failed", who, out_path);
        }
    }
    timer.mark("download+write");
    if (close(outf.fd) != 0) {
        outf.fd = -1;
        return rss_set_error(RSS_EIO, "%s: close of %s failed", who, out_path);
    }
    outf.fd = -1;
    timer.mark("close");
    return RSS_OK;
}

// Every entry point holds the context's lock for the whole call (struct rss_ctx) and, when
// the call fails, waits out what it left in flight before the lock is released.
template <class Rows>
int csv_hash_text(const char* who, rss_ctx* ctx, const typename CsvJob<Rows>::Key* key,
                  const char* text, size_t len, uint32_t htable, uint32_t nqueues,
                  const uint32_t* reta, uint32_t flags, const char** out, size_t* out_len,
                  uint64_t* counts, size_t* n_rows) {
    if (!ctx) return rss_set_error(RSS_EINVAL, "%s: NULL argument", who);
    std::lock_guard<std::mutex> lock(ctx->mu);
    const int rc = csv_hash_text_locked<Rows>(who, ctx, key, text, len, htable, nqueues, reta,
                                              flags, out, out_len, counts, n_rows);
    if (rc != RSS_OK) rss_ctx_quiesce(ctx);
    return rc;
}

template <class Rows>
int csv_hash_file(const char* who, rss_ctx* ctx, const typename CsvJob<Rows>::Key* key,
                  const char* in_path, const char* out_path, uint32_t htable, uint32_t nqueues,
                  const uint32_t* reta, uint32_t flags, uint64_t* counts, size_t* n_rows) {
    if (!ctx) return rss_set_error(RSS_EINVAL, "%s: NULL argument", who);
    std::lock_guard<std::mutex> lock(ctx->mu);
    const int rc = csv_hash_file_locked<Rows>(who, ctx, key, in_path, out_path, htable, nqueues,
                                              reta, flags, counts, n_rows);
    if (rc != RSS_OK) rss_ctx_quiesce(ctx);
    return rc;
}

}  // namespace

extern "C" {

int rss_csv_hash_text(rss_ctx* ctx, const rss_key* key, const char* text, size_t len,
                      uint32_t htable, uint32_t nqueues, const uint32_t* reta, uint32_t flags,
                      const char** out, size_t* out_len, uint64_t* counts, size_t* n_rows) {
    return csv_hash_text<RowsV4>("rss_csv_hash_text", ctx, key, text, len, htable, nqueues, reta,
                                 flags, out, out_len, counts, n_rows);
}

int rss_csv6_hash_text(rss_ctx* ctx, const rss_key6* key, const char* text, size_t len,
                       uint32_t htable, uint32_t nqueues, const uint32_t* reta, uint32_t flags,
                       const char** out, size_t* out_len, uint64_t* counts, size_t* n_rows) {
    return csv_hash_text<RowsV6>("rss_csv6_hash_text", ctx, key, text, len, htable, nqueues,
                                 reta, flags, out, out_len, counts, n_rows);
}

int rss_csv_hash_file(rss_ctx* ctx, const rss_key* key, const char* in_path, const char* out_path,
                      uint32_t htable, uint32_t nqueues, const uint32_t* reta, uint32_t flags,
                      uint64_t* counts, size_t* n_rows) {
    return csv_hash_file<RowsV4>("rss_csv_hash_file", ctx, key, in_path, out_path, htable,
                                 nqueues, reta, flags, counts, n_rows);
}

int rss_csv6_hash_file(rss_ctx* ctx, const rss_key6* key, const char* in_path,
                       const char* out_path, uint32_t htable, uint32_t nqueues,
                       const uint32_t* reta, uint32_t flags, uint64_t* counts, size_t* n_rows) {
    return csv_hash_file<RowsV6>("rss_csv6_hash_file", ctx, key, in_path, out_path, htable,
                                 nqueues, reta, flags, counts, n_rows);
}

}  // extern "C"

void rss_csv_release(rss_ctx* ctx) {
    for (int b = 0; b < 2; ++b) {
        if (ctx->stage[b]) (void)hipHostFree(ctx->stage[b]);
        if (ctx->stage_done[b]) (void)hipEventDestroy(ctx->stage_done[b]);
        ctx->stage[b] = nullptr;
        ctx->stage_done[b] = nullptr;
    }
    ctx->stage_bytes = 0;
    trim_pool(ctx, 0);
}


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
#include <hip/hip_runtime.h>

#include <cstring>

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

__global__ __launch_bounds__(kThreads) void parse_lines(
    const uint8_t* __restrict__ text, uint64_t len, const uint32_t* __restrict__ pos,
    uint64_t nnl, uint64_t nlines, Layout layout, rss_tuple4* tuples, uint32_t* is_row,
    unsigned long long* n_empty, unsigned long long* n_bad) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= nlines) return;
    const uint64_t s = i ? (uint64_t)pos[i - 1] + 1 : 0;
    uint64_t e = i < nnl ? pos[i] : len;
    if (e > s && text[e - 1] == '\r') --e;
    if (e == s) {  // "\n", "\r\n" or a final "\r": skipped like skip_empty_line
        is_row[i] = 0;
        atomicAdd(n_empty, 1ull);
        return;
    }
    const uint8_t* p = text + s;
    const uint8_t* end = text + e;
    uint32_t v[4];
    bool ok = true;
    for (int f = 0; f < 4 && ok; ++f) {
        const int c = layout.col[f];
        ok = c < 2 ? d_scan_ip(p, end, v[c]) : d_scan_uint<5, 65535>(p, end, v[c]);
        if (ok && f < 3) {
            ok = p < end && *p == ',';
            ++p;
        }
    }
    if (!ok || p != end) {
        atomicAdd(n_bad, 1ull);
        is_row[i] = 0;
        return;
    }
    is_row[i] = 1;
    tuples[i].sip = v[0];
    tuples[i].dip = v[1];
    tuples[i].ports = v[2] << 16 | v[3];
}

__global__ __launch_bounds__(kThreads) void compact_rows(const rss_tuple4* __restrict__ in,
                                                         const uint32_t* __restrict__ is_row,
                                                         const uint64_t* __restrict__ slot,
                                                         uint64_t nlines, rss_tuple4* out) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i < nlines && is_row[i]) out[slot[i]] = in[i];
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

__global__ __launch_bounds__(kThreads) void write_rows(const rss_tuple4* __restrict__ t,
                                                       const uint32_t* __restrict__ hash,
                                                       const uint32_t* __restrict__ queue,
                                                       uint64_t n, Layout layout,
                                                       const uint64_t* __restrict__ off,
                                                       uint8_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const rss_tuple4 r = t[i];
    const uint32_t col[4] = {r.sip, r.dip, r.ports >> 16, r.ports & 0xFFFFu};
    uint8_t* w = out + off[i];
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

// ---------------------------------------------------------------- host -------
inline unsigned blocks_for(uint64_t n, uint64_t per_block) {
    return (unsigned)((n + per_block - 1) / per_block);
}

// device allocations of one call, released on every exit path
struct DeviceBuffers {
    std::vector<void*> ptrs;
    ~DeviceBuffers() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    int alloc(T** out, uint64_t count) {
        void* p = nullptr;
        const hipError_t e = hipMalloc(&p, count ? count * sizeof(T) : 1);
        if (e != hipSuccess)
            return rss_set_error(e == hipErrorOutOfMemory ? RSS_ENOMEM : RSS_EIO,
                                 "rss_csv_hash_text: hipMalloc(%llu B): %s",
                                 (unsigned long long)(count * sizeof(T)), hipGetErrorString(e));
        ptrs.push_back(p);
        *out = static_cast<T*>(p);
        return RSS_OK;
    }
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

}  // namespace

extern "C" {

int rss_csv_hash_text(rss_ctx* ctx, const rss_key* key, const char* text, size_t len,
                      uint32_t htable, uint32_t nqueues, const uint32_t* reta, uint32_t flags,
                      const char** out, size_t* out_len, uint64_t* counts, size_t* n_rows) {
    if (!ctx || !key || !text || !counts || !n_rows)
        return rss_set_error(RSS_EINVAL, "rss_csv_hash_text: NULL argument");
    const bool want_file = !(flags & RSS_CSV_COUNTS_ONLY);
    if (want_file && (!out || !out_len))
        return rss_set_error(RSS_EINVAL, "rss_csv_hash_text: out / out_len NULL");
    if (htable < 1 || nqueues < 1)
        return rss_set_error(RSS_EINVAL, "rss_csv_hash_text: htable (%u) and nqueues (%u) must be >= 1",
                             htable, nqueues);
    *n_rows = 0;
    rss_csv_layout layout;
    size_t body_off;
    if (!rss_csv_header(text, len, &layout, &body_off))
        return rss_set_error(RSS_ENOTSUP, "rss_csv_hash_text: header is not canonical");
    const uint64_t blen = len - body_off;
    if (blen >= 0xFFFFFFFFull)  // newline positions are 32-bit
        return rss_set_error(RSS_ENOTSUP, "rss_csv_hash_text: body of %llu B exceeds 4 GiB",
                             (unsigned long long)blen);
    CSV_HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream[0];
    DeviceBuffers buf;
    int rc;
    // 1. text up, newline index
    uint8_t* d_text;
    const uint64_t nchunks = (blen + kChunk - 1) / kChunk;
    uint32_t* d_cnt;
    uint64_t* d_cnt_off;
    if ((rc = buf.alloc(&d_text, blen)) || (rc = buf.alloc(&d_cnt, nchunks)) ||
        (rc = buf.alloc(&d_cnt_off, nchunks)))
        return rc;
    CSV_HIP_CHECK(hipMemcpyAsync(d_text, text + body_off, blen, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(count_newlines, dim3(blocks_for(nchunks, kThreads)), dim3(kThreads), 0, s,
                       d_text, blen, d_cnt);
    CSV_HIP_CHECK(hipGetLastError());
    uint64_t nnl;
    if ((rc = exclusive_scan(d_cnt, nchunks, d_cnt_off, &nnl, buf, s))) return rc;
    uint32_t* d_pos;
    if ((rc = buf.alloc(&d_pos, nnl))) return rc;
    hipLaunchKernelGGL(emit_newlines, dim3(blocks_for(nchunks, kThreads)), dim3(kThreads), 0, s,
                       d_text, blen, d_cnt_off, d_pos);
    CSV_HIP_CHECK(hipGetLastError());
    uint32_t last_nl = 0;
    if (nnl)
        CSV_HIP_CHECK(hipMemcpyAsync(&last_nl, d_pos + nnl - 1, 4, hipMemcpyDeviceToHost, s));
    CSV_HIP_CHECK(hipStreamSynchronize(s));
    const uint64_t tail_start = nnl ? (uint64_t)last_nl + 1 : 0;
    const uint64_t nlines = nnl + (tail_start < blen ? 1 : 0);

    // 2. parse every line
    rss_tuple4* d_lines;
    uint32_t* d_is_row;
    unsigned long long* d_stat;  // [0] empty lines, [1] non-canonical lines
    if ((rc = buf.alloc(&d_lines, nlines)) || (rc = buf.alloc(&d_is_row, nlines)) ||
        (rc = buf.alloc(&d_stat, 2)))
        return rc;
    CSV_HIP_CHECK(hipMemsetAsync(d_stat, 0, 2 * sizeof(unsigned long long), s));
    Layout lay;
    memcpy(lay.col, layout.field_column, 4);
    if (nlines)
        hipLaunchKernelGGL(parse_lines, dim3(blocks_for(nlines, kThreads)), dim3(kThreads), 0, s,
                           d_text, blen, d_pos, nnl, nlines, lay, d_lines, d_is_row, d_stat,
                           d_stat + 1);
    CSV_HIP_CHECK(hipGetLastError());
    unsigned long long stat[2];
    CSV_HIP_CHECK(hipMemcpyAsync(stat, d_stat, sizeof stat, hipMemcpyDeviceToHost, s));
    CSV_HIP_CHECK(hipStreamSynchronize(s));
    if (stat[1]) return rss_set_error(RSS_ENOTSUP, "rss_csv_hash_text: %llu non-canonical rows", stat[1]);
    const uint64_t n = nlines - stat[0];
    if (n == 0) return rss_set_error(RSS_ENOTSUP, "rss_csv_hash_text: no data rows");

    // 3. drop empty lines (only if there are any)
    rss_tuple4* d_tuples = d_lines;
    if (stat[0]) {
        uint64_t* d_slot;
        uint64_t kept;
        if ((rc = buf.alloc(&d_slot, nlines)) || (rc = buf.alloc(&d_tuples, n))) return rc;
        if ((rc = exclusive_scan(d_is_row, nlines, d_slot, &kept, buf, s))) return rc;
        hipLaunchKernelGGL(compact_rows, dim3(blocks_for(nlines, kThreads)), dim3(kThreads), 0, s,
                           d_lines, d_is_row, d_slot, nlines, d_tuples);
        CSV_HIP_CHECK(hipGetLastError());
    }

    // 4. hash + queue + counts
    uint64_t* d_counts;
    uint32_t *d_hash = nullptr, *d_queue = nullptr;
    if ((rc = buf.alloc(&d_counts, nqueues))) return rc;
    if (want_file && ((rc = buf.alloc(&d_hash, n)) || (rc = buf.alloc(&d_queue, n)))) return rc;
    rc = reta ? rss_hash_device_reta(key, d_tuples, n, htable, reta, nqueues, d_hash, d_queue,
                                     d_counts, 0, s)
              : rss_hash_device(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, 0, s);
    if (rc) return rc;
    CSV_HIP_CHECK(hipMemcpyAsync(counts, d_counts, sizeof(uint64_t) * nqueues,
                                 hipMemcpyDeviceToHost, s));
    CSV_HIP_CHECK(hipStreamSynchronize(s));
    *n_rows = n;
    if (!want_file) return RSS_OK;

    // 5. format the rows on the device, the prefix on the host, one copy down
    uint32_t* d_len;
    uint64_t* d_off;
    if ((rc = buf.alloc(&d_len, n)) || (rc = buf.alloc(&d_off, n))) return rc;
    hipLaunchKernelGGL(row_lengths, dim3(blocks_for(n, kThreads)), dim3(kThreads), 0, s, d_tuples,
                       d_hash, d_queue, n, d_len);
    CSV_HIP_CHECK(hipGetLastError());
    uint64_t rows_bytes;
    if ((rc = exclusive_scan(d_len, n, d_off, &rows_bytes, buf, s))) return rc;
    uint8_t* d_out;
    if ((rc = buf.alloc(&d_out, rows_bytes))) return rc;
    hipLaunchKernelGGL(write_rows, dim3(blocks_for(n, kThreads)), dim3(kThreads), 0, s, d_tuples,
                       d_hash, d_queue, n, lay, d_off, d_out);
    CSV_HIP_CHECK(hipGetLastError());
    ctx->csv_out.resize(rss_csv_prefix_bound(nqueues) + rows_bytes);
    const size_t prefix = rss_csv_format_prefix(counts, nqueues, &layout, ctx->csv_out.data());
    CSV_HIP_CHECK(hipMemcpyAsync(ctx->csv_out.data() + prefix, d_out, rows_bytes,
                                 hipMemcpyDeviceToHost, s));
    CSV_HIP_CHECK(hipStreamSynchronize(s));
    *out = ctx->csv_out.data();
    *out_len = prefix + rows_bytes;
    return RSS_OK;
}

}  // extern "C"

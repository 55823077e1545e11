// rss_host.hip -- the C ABI of include/rss_toeplitz.h around the engine's launchers
// (rss_toeplitz.hip, through rss_engine.h): key preparation, the device-pointer entry points,
// contexts and the host-memory pipeline (pinned staging, two streams, the small-batch path,
// several contexts), key search from host memory, and the thread's last-error message.  No
// kernels: this file is compiled once and linked into both the product library and the
// tests' hooks build.
//
// Replaces (reference noamsto/rss_simulator_nvidia v0.0.2): Toeplitz.__init__'s key and the
// rotation schedule of __shift_key / __key_left_most_32bits (toeplitz.py:8-15, :71-98), and
// the per-row Simulator.calc_hash loop (simulator.py:74-92) as one batched host call.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rss_engine.h"
#include "rss_internal.h"
#include "rss_toeplitz.h"

namespace {
thread_local std::string g_last_error;
}  // namespace

int rss_set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

namespace {

// window remap for field selection over a tuple of `nfields` fields
void remap_windows(uint32_t* window, int nbits, const int* start, const int* width, int nfields,
                   uint32_t fields) {
    std::vector<uint32_t> out(nbits, 0);
    int pos = 0;
    for (int f = 0; f < nfields; ++f) {
        if (!(fields & (1u << f))) continue;
        for (int b = 0; b < width[f]; ++b) out[start[f] + b] = window[pos + b];
        pos += width[f];
    }
    memcpy(window, out.data(), sizeof(uint32_t) * nbits);
}

void rotation_windows(const uint8_t* key, size_t len, uint32_t* window, int nbits) {
    // after i one-bit rotations of the whole key (toeplitz.py:83-98) its leftmost 32 bits
    // are key bits (i + j) mod 8*len, j = 0..31
    const uint64_t kbits = (uint64_t)len * 8;
    for (int i = 0; i < nbits; ++i) {
        uint32_t w = 0;
        for (int j = 0; j < 32; ++j) {
            const uint64_t b = ((uint64_t)i + j) % kbits;
            w = (w << 1) | ((key[b >> 3] >> (7 - (b & 7))) & 1u);
        }
        window[i] = w;
    }
}

}  // namespace

// ------------------------------------------------------------ C ABI ---------
// (struct rss_ctx: rss_internal.h)

// (rss_internal.h) A host call that fails part-way may have left copies in flight -- an
// earlier chunk's H2D from the caller's tuples, its D2H into the caller's outputs or the
// staging.  Waiting them out before the lock is released keeps the caller's buffers and the
// next call's staging untouched once the error is reported.  Errors here are ignored: the
// first one is already in rss_last_error.
void rss_ctx_quiesce(rss_ctx* ctx) {
    for (int b = 0; b < 2; ++b)
        if (ctx->stream[b]) (void)hipStreamSynchronize(ctx->stream[b]);
}

extern "C" {

int rss_abi_version(void) { return RSS_ABI_VERSION; }

const char* rss_last_error(void) { return g_last_error.c_str(); }

int rss_key_prepare(const uint8_t* key, size_t len, rss_key* out) {
    if (!key || !out) return rss_set_error(RSS_EINVAL, "rss_key_prepare: NULL argument");
    if (len < RSS_KEY_MIN_BYTES)
        return rss_set_error(RSS_EINVAL, "rss_key_prepare: key must hold >= %d bytes, got %zu",
                             RSS_KEY_MIN_BYTES, len);
    memset(out, 0, sizeof *out);
    out->len = (uint32_t)len;
    memcpy(out->bytes, key, len < RSS_KEY_MAX_BYTES ? len : RSS_KEY_MAX_BYTES);
    // For len >= 16 bytes the rotation never wraps and only bytes 0..15 matter.
    rotation_windows(key, len, out->window, RSS_INPUT_BITS);
    return RSS_OK;
}

int rss_key_select_fields(rss_key* key, uint32_t fields) {
    if (!key || key->len < RSS_KEY_MIN_BYTES)
        return rss_set_error(RSS_EINVAL, "rss_key_select_fields: key not prepared");
    if (fields == 0 || (fields & ~RSS_FIELDS_ALL))
        return rss_set_error(RSS_EINVAL, "rss_key_select_fields: bad field mask 0x%x", fields);
    // field f spans input bits [start[f], start[f] + width[f]) of the full tuple
    static const int kStart[4] = {0, 32, 64, 80}, kWidth[4] = {32, 32, 16, 16};
    remap_windows(key->window, RSS_INPUT_BITS, kStart, kWidth, 4, fields);
    return RSS_OK;
}

int rss_key6_prepare(const uint8_t* key, size_t len, rss_key6* out) {
    if (!key || !out) return rss_set_error(RSS_EINVAL, "rss_key6_prepare: NULL argument");
    if (len < RSS_KEY_MIN_BYTES)
        return rss_set_error(RSS_EINVAL, "rss_key6_prepare: key must hold >= %d bytes, got %zu",
                             RSS_KEY_MIN_BYTES, len);
    memset(out, 0, sizeof *out);
    out->len = (uint32_t)len;
    rotation_windows(key, len, out->window, RSS_INPUT6_BITS);
    return RSS_OK;
}

int rss_key6_select_fields(rss_key6* key, uint32_t fields) {
    if (!key || key->len < RSS_KEY_MIN_BYTES)
        return rss_set_error(RSS_EINVAL, "rss_key6_select_fields: key not prepared");
    if (fields == 0 || (fields & ~RSS_FIELDS_ALL))
        return rss_set_error(RSS_EINVAL, "rss_key6_select_fields: bad field mask 0x%x", fields);
    static const int kStart[4] = {0, 128, 256, 272}, kWidth[4] = {128, 128, 16, 16};
    remap_windows(key->window, RSS_INPUT6_BITS, kStart, kWidth, 4, fields);
    return RSS_OK;
}

int rss_hash6_device(const rss_key6* key, const rss_tuple6* d_tuples, size_t n, uint32_t htable,
                     uint32_t nqueues, uint32_t* d_hash, void* d_queue, uint64_t* d_counts,
                     uint32_t flags, void* stream) {
    return rss::launch_hash6(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, flags,
                             static_cast<hipStream_t>(stream), nullptr, nullptr);
}

int rss_hash6_device_ws(const rss_key6* key, const rss_tuple6* d_tuples, size_t n,
                        uint32_t htable, uint32_t nqueues, uint32_t* d_hash, void* d_queue,
                        uint64_t* d_counts, uint32_t flags, uint64_t* d_workspace, void* stream) {
    if (d_counts && (!d_workspace || ((uintptr_t)d_workspace & 7u)))
        return rss_set_error(RSS_EINVAL, "rss_hash6_device_ws: workspace NULL or not 8-byte aligned");
    return rss::launch_hash6(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, flags,
                             static_cast<hipStream_t>(stream), nullptr, d_workspace);
}

int rss_hash6_device_reta(const rss_key6* key, const rss_tuple6* d_tuples, size_t n,
                          uint32_t htable, const uint32_t* reta, uint32_t nqueues,
                          uint32_t* d_hash, void* d_queue, uint64_t* d_counts, uint32_t flags,
                          void* stream) {
    if (!reta) return rss_set_error(RSS_EINVAL, "rss_hash6_device_reta: reta is NULL");
    return rss::launch_hash6(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, flags,
                             static_cast<hipStream_t>(stream), reta);
}

int rss_device_count(int* out) {
    if (!out) return rss_set_error(RSS_EINVAL, "rss_device_count: NULL argument");
    *out = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return RSS_OK;
    }
    int count = 0;
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) != hipSuccess) continue;
        if (strncmp(prop.gcnArchName, "gfx950", 6) == 0) ++count;
    }
    *out = count;
    return RSS_OK;
}

int rss_hash_device(const rss_key* key, const rss_tuple4* d_tuples, size_t n, uint32_t htable,
                    uint32_t nqueues, uint32_t* d_hash, void* d_queue, uint64_t* d_counts,
                    uint32_t flags, void* stream) {
    return rss::launch_hash(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, flags,
                            static_cast<hipStream_t>(stream), nullptr, nullptr);
}

int rss_counts_workspace_bytes(uint32_t nqueues, size_t* out) {
    if (!out) return rss_set_error(RSS_EINVAL, "rss_counts_workspace_bytes: NULL argument");
    if (nqueues < 1) return rss_set_error(RSS_EINVAL, "rss_counts_workspace_bytes: nqueues must be >= 1");
    // a reserved word (ws[0], the rounds 2-3 fold's ticket; the size is ABI) + one arrival
    // accumulator per queue + the balanced tail's unit counter (fold_counts, walk_rows)
    *out = sizeof(uint64_t) * ((size_t)nqueues + 2);
    return RSS_OK;
}

int rss_hash_device_ws(const rss_key* key, const rss_tuple4* d_tuples, size_t n, uint32_t htable,
                       uint32_t nqueues, uint32_t* d_hash, void* d_queue, uint64_t* d_counts,
                       uint32_t flags, uint64_t* d_workspace, void* stream) {
    if (d_counts && (!d_workspace || ((uintptr_t)d_workspace & 7u)))
        return rss_set_error(RSS_EINVAL, "rss_hash_device_ws: workspace NULL or not 8-byte aligned");
    return rss::launch_hash(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, flags,
                            static_cast<hipStream_t>(stream), nullptr, d_workspace);
}

int rss_hash_device_reta(const rss_key* key, const rss_tuple4* d_tuples, size_t n,
                         uint32_t htable, const uint32_t* reta, uint32_t nqueues, uint32_t* d_hash,
                         void* d_queue, uint64_t* d_counts, uint32_t flags, void* stream) {
    if (!reta) return rss_set_error(RSS_EINVAL, "rss_hash_device_reta: reta is NULL");
    return rss::launch_hash(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, flags,
                            static_cast<hipStream_t>(stream), reta);
}

int rss_key_search_device(const uint32_t* d_windows, size_t nkeys, const rss_tuple4* d_tuples,
                          size_t n, uint32_t htable, uint32_t nqueues, uint64_t* d_counts,
                          void* stream) {
    return rss::launch_search(d_windows, nkeys, d_tuples, n, htable, nqueues, d_counts,
                              static_cast<hipStream_t>(stream));
}

int rss_generate_tuples(uint64_t seed, uint64_t first_index, size_t n, rss_tuple4* d_tuples,
                        void* stream) {
    if (n == 0) return RSS_OK;
    if (!d_tuples) return rss_set_error(RSS_EINVAL, "rss_generate_tuples: tuples is NULL");
    return rss::launch_generate(seed, first_index, n, d_tuples, static_cast<hipStream_t>(stream));
}

void rss_ctx_destroy(rss_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    rss_csv_release(ctx);
    for (int b = 0; b < 2; ++b) {
        if (ctx->stream[b]) (void)hipStreamSynchronize(ctx->stream[b]);
        (void)hipFree(ctx->d_in[b]);
        (void)hipFree(ctx->d_hash[b]);
        (void)hipFree(ctx->d_queue[b]);
        (void)hipFree(ctx->d_counts[b]);
        (void)hipHostFree(ctx->h_in[b]);
        (void)hipHostFree(ctx->h_hash[b]);
        (void)hipHostFree(ctx->h_queue[b]);
        if (ctx->stream[b]) (void)hipStreamDestroy(ctx->stream[b]);
    }
    (void)hipHostFree(ctx->h_counts);
    delete ctx;
}

int rss_ctx_create(int device, rss_ctx** out) {
    if (!out) return rss_set_error(RSS_EINVAL, "rss_ctx_create: NULL argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        return rss_set_error(RSS_ENODEV, "rss_ctx_create: no HIP device visible");
    }
    if (device < 0 || device >= ndev)
        return rss_set_error(RSS_EINVAL, "rss_ctx_create: device %d out of range [0, %d)", device, ndev);
    hipDeviceProp_t prop;
    RSS_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return rss_set_error(RSS_ENODEV, "rss_ctx_create: device %d is %s, this build targets gfx950",
                             device, prop.gcnArchName);
    rss_ctx* ctx = new rss_ctx();
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    for (int b = 0; b < 2 && e == hipSuccess; ++b)
        e = hipStreamCreateWithFlags(&ctx->stream[b], hipStreamNonBlocking);
    if (e != hipSuccess) {
        rss_ctx_destroy(ctx);
        return rss_set_error(RSS_EIO, "rss_ctx_create: %s", hipGetErrorString(e));
    }
    *out = ctx;
    return RSS_OK;
}

}  // extern "C"

// Grows the context's staging to `chunk` output tuples, `in_bytes` of input per slot and
// `nqueues` counts (never shrinks).
static int ctx_reserve(rss_ctx* ctx, size_t chunk, size_t in_bytes, uint32_t nqueues) {
    if (ctx->in_cap < in_bytes) {
        for (int b = 0; b < 2; ++b) {
            (void)hipFree(ctx->d_in[b]);
            (void)hipHostFree(ctx->h_in[b]);
            ctx->d_in[b] = ctx->h_in[b] = nullptr;
        }
        ctx->in_cap = 0;
        for (int b = 0; b < 2; ++b) {
            RSS_HIP_CHECK(hipMalloc(&ctx->d_in[b], in_bytes));
            RSS_HIP_CHECK(hipHostMalloc(&ctx->h_in[b], in_bytes, hipHostMallocDefault));
        }
        RSS_HIP_CHECK(hipHostGetDevicePointer(&ctx->alias_in, ctx->h_in[0], 0));
        ctx->in_cap = in_bytes;
    }
    if (ctx->chunk < chunk) {
        for (int b = 0; b < 2; ++b) {
            (void)hipFree(ctx->d_hash[b]);
            (void)hipFree(ctx->d_queue[b]);
            (void)hipHostFree(ctx->h_hash[b]);
            (void)hipHostFree(ctx->h_queue[b]);
            ctx->d_hash[b] = ctx->d_queue[b] = nullptr;
            ctx->h_hash[b] = ctx->h_queue[b] = nullptr;
        }
        ctx->chunk = 0;
        for (int b = 0; b < 2; ++b) {
            RSS_HIP_CHECK(hipMalloc(&ctx->d_hash[b], chunk * sizeof(uint32_t)));
            RSS_HIP_CHECK(hipMalloc(&ctx->d_queue[b], chunk * sizeof(uint32_t)));
            RSS_HIP_CHECK(hipHostMalloc(&ctx->h_hash[b], chunk * sizeof(uint32_t), hipHostMallocDefault));
            RSS_HIP_CHECK(hipHostMalloc(&ctx->h_queue[b], chunk * sizeof(uint32_t), hipHostMallocDefault));
        }
        RSS_HIP_CHECK(hipHostGetDevicePointer(&ctx->alias_hash, ctx->h_hash[0], 0));
        RSS_HIP_CHECK(hipHostGetDevicePointer(&ctx->alias_queue, ctx->h_queue[0], 0));
        ctx->chunk = chunk;
    }
    if (ctx->counts_cap < nqueues) {
        for (int b = 0; b < 2; ++b) {
            (void)hipFree(ctx->d_counts[b]);
            ctx->d_counts[b] = nullptr;
        }
        (void)hipHostFree(ctx->h_counts);
        ctx->h_counts = nullptr;
        ctx->counts_cap = 0;
        for (int b = 0; b < 2; ++b)
            RSS_HIP_CHECK(hipMalloc(&ctx->d_counts[b], sizeof(uint64_t) * nqueues));
        RSS_HIP_CHECK(hipHostMalloc(&ctx->h_counts, sizeof(uint64_t) * nqueues, hipHostMallocDefault));
        ctx->counts_cap = nqueues;
    }
    return RSS_OK;
}

// The two tuple layouts share the host path -- staging, small batches, the pipeline --
// and differ in their tuple, key and launcher.
struct Ipv4 {
    using Tuple = rss_tuple4;
    using Key = rss_key;
    static constexpr const char* kWho = "rss_hash_host";
    static int launch(const Key* key, const Tuple* t, size_t n, uint32_t htable, uint32_t nqueues,
                      uint32_t* hash, void* queue, uint64_t* counts, uint32_t flags, hipStream_t s,
                      const uint32_t* reta) {
        return rss::launch_hash(key, t, n, htable, nqueues, hash, queue, counts, flags, s, reta);
    }
};

struct Ipv6 {
    using Tuple = rss_tuple6;
    using Key = rss_key6;
    static constexpr const char* kWho = "rss_hash6_host";
    static int launch(const Key* key, const Tuple* t, size_t n, uint32_t htable, uint32_t nqueues,
                      uint32_t* hash, void* queue, uint64_t* counts, uint32_t flags, hipStream_t s,
                      const uint32_t* reta) {
        return rss::launch_hash6(key, t, n, htable, nqueues, hash, queue, counts, flags, s, reta);
    }
};

// Small host batches -- a reference-style caller hashing one row per call
// (Toeplitz.compute_hash from Simulator.__calc_entry_hash, simulator.py:80-92) -- are
// bound by per-call overhead, not bytes: one stream, no pointer-attribute queries, the
// kernel reading the tuples from and writing hash / queue straight into slot 0's pinned
// staging (mapped into the device address space), the counts landing in pinned memory,
// one synchronisation.  Same kernel and results as the pipelined path.
constexpr size_t kSmallBatch = (size_t)1 << 14;

template <class L>
static int hash_host_small(rss_ctx* ctx, const typename L::Key* key,
                           const typename L::Tuple* h_tuples, size_t n, uint32_t htable,
                           uint32_t nqueues, uint32_t* h_hash, uint32_t* h_queue,
                           uint64_t* h_counts, uint32_t flags, const uint32_t* reta) {
    using Tuple = typename L::Tuple;
    int rc = ctx_reserve(ctx, std::max(ctx->chunk, kSmallBatch), kSmallBatch * sizeof(Tuple),
                         h_counts ? nqueues : 1);
    if (rc) return rc;
    hipStream_t s = ctx->stream[0];
    memcpy(ctx->h_in[0], h_tuples, n * sizeof(Tuple));
    rc = L::launch(key, static_cast<const Tuple*>(ctx->alias_in), n, htable, nqueues,
                   h_hash ? static_cast<uint32_t*>(ctx->alias_hash) : nullptr,
                   h_queue ? ctx->alias_queue : nullptr, h_counts ? ctx->d_counts[0] : nullptr, 0,
                   s, reta);
    if (rc) return rc;
    if (h_counts)
        RSS_HIP_CHECK(hipMemcpyAsync(ctx->h_counts, ctx->d_counts[0], sizeof(uint64_t) * nqueues,
                                     hipMemcpyDeviceToHost, s));
    RSS_HIP_CHECK(hipStreamSynchronize(s));
    if (h_hash) memcpy(h_hash, ctx->h_hash[0], n * 4);
    if (h_queue) memcpy(h_queue, ctx->h_queue[0], n * 4);
    if (h_counts) {
        if (!(flags & RSS_FLAG_ACCUMULATE)) memset(h_counts, 0, sizeof(uint64_t) * nqueues);
        for (uint32_t q = 0; q < nqueues; ++q) h_counts[q] += ctx->h_counts[q];
    }
    return RSS_OK;
}

// memcpy split over up to 8 threads, 1 MiB or more each, from 4 MiB on (below that a thread
// start costs more than it saves): the pinned staging copies, not PCIe or the kernel, bound
// rss_hash_host (one thread moves ~10 GB/s; a 4M-tuple slot is 80 MB each way)
static void par_memcpy(void* dst, const void* src, size_t bytes) {
    constexpr size_t kPerThread = (size_t)1 << 20, kSplitFrom = (size_t)4 << 20;
    const size_t nt = bytes < kSplitFrom ? 1 : std::min<size_t>(8, bytes / kPerThread);
    if (nt <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> pool;
    for (size_t k = 1; k < nt; ++k)
        pool.emplace_back([=] {
            const size_t a = bytes * k / nt, b = bytes * (k + 1) / nt;
            memcpy(static_cast<char*>(dst) + a, static_cast<const char*>(src) + a, b - a);
        });
    memcpy(dst, src, bytes / nt);
    for (auto& t : pool) t.join();
}

// Whether [p, p + bytes) is page-locked host memory (rss_host_alloc, hipHostMalloc,
// hipHostRegister) that the copy engines can read / write directly.
static bool host_pinned(const void* p, size_t bytes) {
    if (!p || !bytes) return true;
    const char* ends[2] = {static_cast<const char*>(p), static_cast<const char*>(p) + bytes - 1};
    for (const char* q : ends) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (a.type != hipMemoryTypeHost) return false;
    }
    return true;
}

template <class L>
static int hash_host_pipeline(rss_ctx* ctx, const typename L::Key* key,
                              const typename L::Tuple* h_tuples, size_t n, uint32_t htable,
                              uint32_t nqueues, uint32_t* h_hash, uint32_t* h_queue,
                              uint64_t* h_counts, uint32_t flags, const uint32_t* reta) {
    using Tuple = typename L::Tuple;
    // 48 MB of input per slot, in 64K-tuple steps: 4M IPv4 tuples (+ 32 MB out), 1.38M IPv6
    // tuples (+ 11 MB out)
    constexpr size_t kChunkMax = (((size_t)48 << 20) / sizeof(Tuple)) & ~(size_t)0xFFFF;
    // at least four chunks once a batch has 1M tuples, so that copies and the kernel overlap
    // from the second chunk on
    constexpr size_t kStep = (size_t)1 << 16, kChunkMin = (size_t)1 << 18;
    const size_t quarter = ((n + 3) / 4 + kStep - 1) / kStep * kStep;
    const size_t chunk = n <= kChunkMin ? (n ? n : 1)
                                        : std::min(kChunkMax, std::max(kChunkMin, quarter));
    int rc = ctx_reserve(ctx, chunk, chunk * sizeof(Tuple), nqueues);
    if (rc) return rc;
    for (int b = 0; b < 2; ++b)
        RSS_HIP_CHECK(hipMemsetAsync(ctx->d_counts[b], 0, sizeof(uint64_t) * nqueues, ctx->stream[b]));

    // Double-buffered pipeline: while slot b runs H2D -> kernel -> D2H on its
    // stream, the host fills the other slot's pinned input and drains its output.
    // Caller buffers that are already page-locked skip the staging copy: the copy
    // engines move them directly, so only PCIe bounds the pipeline.
    const bool in_direct = host_pinned(h_tuples, n * sizeof(Tuple));
    const bool hash_direct = host_pinned(h_hash, h_hash ? n * 4 : 0);
    const bool queue_direct = host_pinned(h_queue, h_queue ? n * 4 : 0);
    const size_t nchunks = (n + chunk - 1) / chunk;
    size_t pending_off[2] = {0, 0}, pending_len[2] = {0, 0};
    auto drain = [&](int b) -> int {
        RSS_HIP_CHECK(hipStreamSynchronize(ctx->stream[b]));
        if (pending_len[b]) {
            if (h_hash && !hash_direct)
                par_memcpy(h_hash + pending_off[b], ctx->h_hash[b], pending_len[b] * 4);
            if (h_queue && !queue_direct)
                par_memcpy(h_queue + pending_off[b], ctx->h_queue[b], pending_len[b] * 4);
            pending_len[b] = 0;
        }
        return RSS_OK;
    };
    for (size_t c = 0; c < nchunks; ++c) {
        const int b = (int)(c & 1);
        const size_t off = c * chunk;
        const size_t len = (n - off) < chunk ? (n - off) : chunk;
        hipStream_t s = ctx->stream[b];
        // staged slots are reused only after the host has drained them; direct copies
        // are ordered behind the slot's previous chunk by the stream itself
        if (!(in_direct && hash_direct && queue_direct)) {
            rc = drain(b);
            if (rc) return rc;
        }
        const void* up = h_tuples + off;
        if (!in_direct) {
            par_memcpy(ctx->h_in[b], up, len * sizeof(Tuple));
            up = ctx->h_in[b];
        }
        RSS_HIP_CHECK(hipMemcpyAsync(ctx->d_in[b], up, len * sizeof(Tuple), hipMemcpyHostToDevice, s));
        rc = L::launch(key, static_cast<const Tuple*>(ctx->d_in[b]), len, htable, nqueues,
                       h_hash ? ctx->d_hash[b] : nullptr, h_queue ? ctx->d_queue[b] : nullptr,
                       ctx->d_counts[b], RSS_FLAG_ACCUMULATE, s, reta);  // u32 queues on the host path
        if (rc) return rc;
        if (h_hash)
            RSS_HIP_CHECK(hipMemcpyAsync(hash_direct ? h_hash + off : ctx->h_hash[b],
                                         ctx->d_hash[b], len * 4, hipMemcpyDeviceToHost, s));
        if (h_queue)
            RSS_HIP_CHECK(hipMemcpyAsync(queue_direct ? h_queue + off : ctx->h_queue[b],
                                         ctx->d_queue[b], len * 4, hipMemcpyDeviceToHost, s));
        pending_off[b] = off;
        pending_len[b] = len;
    }
    for (int b = 0; b < 2; ++b) {
        rc = drain(b);
        if (rc) return rc;
    }
    if (h_counts) {
        std::vector<uint64_t> tmp(nqueues);
        if (!(flags & RSS_FLAG_ACCUMULATE)) memset(h_counts, 0, sizeof(uint64_t) * nqueues);
        for (int b = 0; b < 2; ++b) {
            RSS_HIP_CHECK(hipMemcpy(tmp.data(), ctx->d_counts[b], sizeof(uint64_t) * nqueues,
                                    hipMemcpyDeviceToHost));
            for (uint32_t q = 0; q < nqueues; ++q) h_counts[q] += tmp[q];
        }
    }
    return RSS_OK;
}

// Every host-memory entry point: argument checks, the context's lock for the whole call
// (struct rss_ctx), the small-batch path or the pipeline, and on failure the wait for
// whatever the call left in flight (rss_ctx_quiesce) before the lock is released.
template <class L>
static int hash_host_locked(rss_ctx* ctx, const typename L::Key* key,
                            const typename L::Tuple* h_tuples, size_t n, uint32_t htable,
                            uint32_t nqueues, uint32_t* h_hash, uint32_t* h_queue,
                            uint64_t* h_counts, uint32_t flags, const uint32_t* reta) {
    if (!ctx) return rss_set_error(RSS_EINVAL, "%s: ctx is NULL", L::kWho);
    if (n && !h_tuples) return rss_set_error(RSS_EINVAL, "%s: tuples is NULL", L::kWho);
    if (htable < 1 || nqueues < 1)
        return rss_set_error(RSS_EINVAL, "%s: htable (%u) and nqueues (%u) must be >= 1", L::kWho,
                             htable, nqueues);
    std::lock_guard<std::mutex> lock(ctx->mu);
    RSS_HIP_CHECK(hipSetDevice(ctx->device));
    const int rc = n > 0 && n <= kSmallBatch
                       ? hash_host_small<L>(ctx, key, h_tuples, n, htable, nqueues, h_hash,
                                            h_queue, h_counts, flags, reta)
                       : hash_host_pipeline<L>(ctx, key, h_tuples, n, htable, nqueues, h_hash,
                                               h_queue, h_counts, flags, reta);
    if (rc != RSS_OK) rss_ctx_quiesce(ctx);
    return rc;
}

extern "C" {

int rss_hash_host(rss_ctx* ctx, const rss_key* key, const rss_tuple4* h_tuples, size_t n,
                  uint32_t htable, uint32_t nqueues, uint32_t* h_hash, uint32_t* h_queue,
                  uint64_t* h_counts, uint32_t flags) {
    return hash_host_locked<Ipv4>(ctx, key, h_tuples, n, htable, nqueues, h_hash, h_queue,
                                  h_counts, flags, nullptr);
}

int rss_hash_host_reta(rss_ctx* ctx, const rss_key* key, const rss_tuple4* h_tuples, size_t n,
                       uint32_t htable, const uint32_t* reta, uint32_t nqueues, uint32_t* h_hash,
                       uint32_t* h_queue, uint64_t* h_counts, uint32_t flags) {
    if (!reta) return rss_set_error(RSS_EINVAL, "rss_hash_host_reta: reta is NULL");
    return hash_host_locked<Ipv4>(ctx, key, h_tuples, n, htable, nqueues, h_hash, h_queue,
                                  h_counts, flags, reta);
}

int rss_hash6_host(rss_ctx* ctx, const rss_key6* key, const rss_tuple6* h_tuples, size_t n,
                   uint32_t htable, uint32_t nqueues, uint32_t* h_hash, uint32_t* h_queue,
                   uint64_t* h_counts, uint32_t flags) {
    return hash_host_locked<Ipv6>(ctx, key, h_tuples, n, htable, nqueues, h_hash, h_queue,
                                  h_counts, flags, nullptr);
}

int rss_hash6_host_reta(rss_ctx* ctx, const rss_key6* key, const rss_tuple6* h_tuples, size_t n,
                        uint32_t htable, const uint32_t* reta, uint32_t nqueues, uint32_t* h_hash,
                        uint32_t* h_queue, uint64_t* h_counts, uint32_t flags) {
    if (!reta) return rss_set_error(RSS_EINVAL, "rss_hash6_host_reta: reta is NULL");
    return hash_host_locked<Ipv6>(ctx, key, h_tuples, n, htable, nqueues, h_hash, h_queue,
                                  h_counts, flags, reta);
}

int rss_hash_host_multi(rss_ctx* const* ctxs, int nctx, const rss_key* key,
                        const rss_tuple4* h_tuples, size_t n, uint32_t htable,
                        const uint32_t* reta, uint32_t nqueues, uint32_t* h_hash,
                        uint32_t* h_queue, uint64_t* h_counts, uint32_t flags) {
    if (!ctxs || nctx < 1 || !key)
        return rss_set_error(RSS_EINVAL, "rss_hash_host_multi: NULL argument or no contexts");
    for (int i = 0; i < nctx; ++i) {
        if (!ctxs[i]) return rss_set_error(RSS_EINVAL, "rss_hash_host_multi: context %d is NULL", i);
        for (int j = 0; j < i; ++j)
            if (ctxs[j] == ctxs[i])
                return rss_set_error(RSS_EINVAL, "rss_hash_host_multi: contexts %d and %d are the same",
                                     j, i);
    }
    if (n && !h_tuples) return rss_set_error(RSS_EINVAL, "rss_hash_host_multi: tuples is NULL");
    if (htable < 1 || nqueues < 1)
        return rss_set_error(RSS_EINVAL, "rss_hash_host_multi: htable (%u) and nqueues (%u) must be >= 1",
                             htable, nqueues);
    // contiguous ranges, exactly sharding.shard_range's: n / nctx each, the first n % nctx
    // ranges one longer
    const size_t base = n / (size_t)nctx, extra = n % (size_t)nctx;
    std::vector<std::vector<uint64_t>> part(nctx, std::vector<uint64_t>(h_counts ? nqueues : 0));
    std::vector<int> rcs(nctx, RSS_OK);
    std::vector<std::string> errs(nctx);
    auto work = [&](int i) {
        const size_t a = base * (size_t)i + std::min((size_t)i, extra);
        const size_t b = a + base + ((size_t)i < extra ? 1 : 0);
        const int rc = hash_host_locked<Ipv4>(ctxs[i], key, h_tuples ? h_tuples + a : nullptr, b - a,
                                              htable, nqueues, h_hash ? h_hash + a : nullptr,
                                              h_queue ? h_queue + a : nullptr,
                                              h_counts ? part[i].data() : nullptr, 0, reta);
        if (rc) {
            rcs[i] = rc;
            errs[i] = g_last_error;  // thread-local: carried back to the calling thread
        }
    };
    std::vector<std::thread> pool;
    for (int i = 1; i < nctx; ++i) pool.emplace_back(work, i);
    work(0);
    for (auto& t : pool) t.join();
    for (int i = 0; i < nctx; ++i)
        if (rcs[i]) return rss_set_error(rcs[i], "rss_hash_host_multi: context %d: %s", i, errs[i].c_str());
    if (h_counts) {
        if (!(flags & RSS_FLAG_ACCUMULATE)) memset(h_counts, 0, sizeof(uint64_t) * nqueues);
        for (int i = 0; i < nctx; ++i)
            for (uint32_t q = 0; q < nqueues; ++q) h_counts[q] += part[i][q];
    }
    return RSS_OK;
}

int rss_host_alloc(size_t bytes, void** out) {
    if (!out) return rss_set_error(RSS_EINVAL, "rss_host_alloc: NULL argument");
    *out = nullptr;
    RSS_HIP_CHECK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return RSS_OK;
}

void rss_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int rss_key_search_host(rss_ctx* ctx, const rss_key* keys, size_t nkeys,
                        const rss_tuple4* h_tuples, size_t n, uint32_t htable, uint32_t nqueues,
                        uint64_t* h_counts) {
    if (!ctx || !keys || !h_counts || nkeys == 0)
        return rss_set_error(RSS_EINVAL, "rss_key_search_host: NULL argument or no keys");
    if (n && !h_tuples) return rss_set_error(RSS_EINVAL, "rss_key_search_host: tuples is NULL");
    std::lock_guard<std::mutex> lock(ctx->mu);  // (struct rss_ctx)
    RSS_HIP_CHECK(hipSetDevice(ctx->device));
    std::vector<uint32_t> windows(nkeys * RSS_INPUT_BITS);
    for (size_t k = 0; k < nkeys; ++k) {
        if (keys[k].len < RSS_KEY_MIN_BYTES)
            return rss_set_error(RSS_EINVAL, "rss_key_search_host: key %zu not prepared", k);
        memcpy(&windows[k * RSS_INPUT_BITS], keys[k].window, sizeof keys[k].window);
    }
    uint32_t* d_w = nullptr;
    rss_tuple4* d_t = nullptr;
    uint64_t* d_c = nullptr;
    hipStream_t s = ctx->stream[0];
    auto cleanup = [&] {
        (void)hipStreamSynchronize(s);
        (void)hipFree(d_w);
        (void)hipFree(d_t);
        (void)hipFree(d_c);
    };
    int rc = RSS_OK;
    hipError_t e = hipMalloc(&d_w, windows.size() * sizeof(uint32_t));
    if (e == hipSuccess && n) e = hipMalloc(&d_t, n * sizeof(rss_tuple4));
    if (e == hipSuccess) e = hipMalloc(&d_c, nkeys * nqueues * sizeof(uint64_t));
    if (e == hipSuccess)
        e = hipMemcpyAsync(d_w, windows.data(), windows.size() * sizeof(uint32_t),
                           hipMemcpyHostToDevice, s);
    if (e == hipSuccess && n)
        e = hipMemcpyAsync(d_t, h_tuples, n * sizeof(rss_tuple4), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) {
        cleanup();
        return rss_set_error(e == hipErrorOutOfMemory ? RSS_ENOMEM : RSS_EIO, "rss_key_search_host: %s",
                             hipGetErrorString(e));
    }
    rc = rss::launch_search(d_w, nkeys, d_t, n, htable, nqueues, d_c, s);
    if (rc == RSS_OK) {
        e = hipMemcpyAsync(h_counts, d_c, nkeys * nqueues * sizeof(uint64_t),
                           hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess)
            rc = rss_set_error(RSS_EIO, "rss_key_search_host: %s", hipGetErrorString(e));
    }
    cleanup();
    return rc;
}

}  // extern "C"


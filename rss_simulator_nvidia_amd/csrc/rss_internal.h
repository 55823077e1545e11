// rss_internal.h -- declarations shared by the library's translation units (not ABI).
#pragma once

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <utility>
#include <vector>

#include "rss_toeplitz.h"

#define RSS_HIDDEN __attribute__((visibility("hidden")))

// HIP's own definition (hip_runtime_api.h); repeated so the g++-built sources need
// no HIP headers
typedef struct ihipStream_t* hipStream_t;
typedef struct ihipEvent_t* hipEvent_t;

// Host-pipeline context (rss_ctx_create): device, streams and staging buffers of
// rss_hash_host / rss_hash6_host, plus the host output buffer of rss_csv_hash_text.
//
// Every entry point that takes a context holds `mu` for the whole call (the staging
// buffers, streams and scratch below are one caller's at a time): the reference-compatible
// classes share one process-wide context, and a caller may drive them from many threads
// as it could the reference's Toeplitz.compute_hash, which copies its key per call
// (toeplitz.py:59) and so is reentrant.
struct rss_ctx {
    std::mutex mu;
    int device = 0;
    size_t chunk = 0;   // tuples per output staging buffer (hash, queue)
    size_t in_cap = 0;  // bytes per input staging buffer (IPv4 or IPv6 tuples)
    hipStream_t stream[2] = {nullptr, nullptr};
    void* d_in[2] = {nullptr, nullptr};
    uint32_t* d_hash[2] = {nullptr, nullptr};
    uint32_t* d_queue[2] = {nullptr, nullptr};
    uint64_t* d_counts[2] = {nullptr, nullptr};
    uint32_t counts_cap = 0;
    void* h_in[2] = {nullptr, nullptr};
    uint32_t* h_hash[2] = {nullptr, nullptr};
    uint32_t* h_queue[2] = {nullptr, nullptr};
    // small batches (rss_hash_host, n <= kSmallBatch): device aliases of slot 0's pinned
    // staging, read / written by the kernel in place, and a pinned landing buffer for the
    // counts
    void* alias_in = nullptr;
    void* alias_hash = nullptr;
    void* alias_queue = nullptr;
    uint64_t* h_counts = nullptr;
    std::vector<char> csv_out;  // rss_csv_hash_text's statistics file image
    // rss_csv_hash_file: two pinned staging buffers for the streamed file I/O
    char* stage[2] = {nullptr, nullptr};
    hipEvent_t stage_done[2] = {nullptr, nullptr};
    size_t stage_bytes = 0;
    // device blocks (pointer, bytes) the CSV device path keeps between calls
    std::vector<std::pair<void*, size_t>> csv_pool;
};

// rss_csv_device.hip: release the CSV device path's staging and pooled blocks of a context
RSS_HIDDEN void rss_csv_release(rss_ctx* ctx);

// rss_host.hip: wait out whatever a failed call left in flight on the context's streams
// (copies from or into the caller's buffers and the staging), called under `mu` before an
// entry point returns an error.
RSS_HIDDEN void rss_ctx_quiesce(rss_ctx* ctx);

// Record the thread's rss_last_error() message; returns `code`.
RSS_HIDDEN int rss_set_error(int code, const char* fmt, ...)
    __attribute__((format(printf, 2, 3)));

// rss_csv.cpp: canonical header of a file image -> column layout and the byte offset
// of the first data row; false if the header is not canonical or no row follows.
RSS_HIDDEN bool rss_csv_header(const char* data, size_t len, rss_csv_layout* layout,
                               size_t* body_offset);

// rss_csv.cpp: the part of write_statistics' output before the data rows (per-queue
// counts of the non-empty queues, then the table header); returns its length.  `out`
// needs rss_csv_prefix_bound(nqueues) bytes.
RSS_HIDDEN size_t rss_csv_prefix_bound(uint32_t nqueues);
RSS_HIDDEN size_t rss_csv_format_prefix(const uint64_t* counts, uint32_t nqueues,
                                        const rss_csv_layout* layout, char* out);

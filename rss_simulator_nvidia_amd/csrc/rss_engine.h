// rss_engine.h -- the engine's launchers (rss_toeplitz.hip) as the C ABI (rss_host.hip) calls
// them, and the HIP error macro both use.  Internal, not ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "rss_internal.h"
#include "rss_toeplitz.h"

// return the failing HIP call as RSS_ENOMEM / RSS_EIO with rss_last_error() set
#define RSS_HIP_CHECK(expr)                                                        \
    do {                                                                           \
        hipError_t e_ = (expr);                                                    \
        if (e_ != hipSuccess)                                                      \
            return rss_set_error(e_ == hipErrorOutOfMemory ? RSS_ENOMEM : RSS_EIO, \
                                 "%s failed: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

namespace rss {

// rss_hash_device[_ws|_reta] on `stream` (reta / ws may be NULL): include/rss_toeplitz.h
RSS_HIDDEN int launch_hash(const rss_key* key, const rss_tuple4* d_tuples, size_t n,
                           uint32_t htable, uint32_t nqueues, uint32_t* d_hash, void* d_queue,
                           uint64_t* d_counts, uint32_t flags, hipStream_t stream,
                           const uint32_t* reta = nullptr, uint64_t* ws = nullptr);
// rss_hash6_device[_ws|_reta]
RSS_HIDDEN int launch_hash6(const rss_key6* key, const rss_tuple6* d_tuples, size_t n,
                            uint32_t htable, uint32_t nqueues, uint32_t* d_hash, void* d_queue,
                            uint64_t* d_counts, uint32_t flags, hipStream_t stream,
                            const uint32_t* reta = nullptr, uint64_t* ws = nullptr);
// rss_key_search_device
RSS_HIDDEN int launch_search(const uint32_t* d_windows, size_t nkeys, const rss_tuple4* d_tuples,
                             size_t n, uint32_t htable, uint32_t nqueues, uint64_t* d_counts,
                             hipStream_t stream);
// rss_generate_tuples (n > 0, d_tuples non-NULL)
RSS_HIDDEN int launch_generate(uint64_t seed, uint64_t first_index, size_t n,
                               rss_tuple4* d_tuples, hipStream_t stream);

}  // namespace rss

// rss_toeplitz.hip -- CDNA4 (gfx950) RSS Toeplitz engine: kernels + C ABI.
//
// Hot path replaced (reference noamsto/rss_simulator_nvidia v0.0.2):
//   Toeplitz.compute_hash            rss_simulator/toeplitz.py:46-69
//   Simulator.calc_hash / entry hash rss_simulator/simulator.py:74-92
//   Simulator.calc_queue_number      rss_simulator/simulator.py:94-98
//   value_counts in write_statistics rss_simulator/simulator.py:107-113
//
// Kernel shape: one lane per tuple, 4 consecutive tuples per lane
// per iteration (3 x dwordx4 loads, dwordx4 hash/queue stores), persistent
// grid-stride launch of 2 x 1024-thread workgroups per CU.  The Toeplitz hash is
// evaluated from 24 nibble tables (16 entries each, the XOR of the key windows a
// 4-bit input value selects) replicated 32x in LDS so that lane l always reads
// bank l: 24 conflict-free ds_read_b32 + ~48 VALU per tuple instead of the
// reference's 96-step bit-serial loop.  The per-queue histogram is privatised per
// lane column in LDS and folded into global uint64 counts once per workgroup.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rss_toeplitz.h"

namespace {

// ---------------------------------------------------------------- errors ----
thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define RSS_HIP_CHECK(expr)                                                        \
    do {                                                                           \
        hipError_t e_ = (expr);                                                    \
        if (e_ != hipSuccess)                                                      \
            return set_error(e_ == hipErrorOutOfMemory ? RSS_ENOMEM : RSS_EIO,     \
                             "%s failed: %s", #expr, hipGetErrorString(e_));       \
    } while (0)

// ------------------------------------------------------------ constants -----
constexpr int kBlock = 1024;            // threads per workgroup (16 waves)
constexpr int kBlocksPerCU = 2;         // 2 x 16 waves = 32 waves/CU
constexpr int kCopies = 32;             // LUT replicas: lane l reads bank (l & 31)
constexpr uint32_t kLutDwords = RSS_NIBBLES * 16 * kCopies;  // 12288 dwords
constexpr uint32_t kLutBytes = kLutDwords * 4;              // 48 KiB
static_assert(kLutBytes == 48 * 1024, "LUT layout: 24 tables x 16 values x 32 replicas");
constexpr uint32_t kBinBytesMax = 32 * 1024;                // histogram LDS budget

enum QueueMode { QM_MASK = 0, QM_FAST16 = 1, QM_FAST32 = 2 };
enum HistMode { HIST_PRIVATE = 0, HIST_SHARED = 1, HIST_GLOBAL = 2, HIST_NONE = 3 };

// Everything a launch needs, passed by value in the kernarg segment (1.6 KiB).
struct LaunchParams {
    uint32_t lut[RSS_NIBBLES][16];
    const rss_tuple4* tuples;
    uint32_t* hash_out;
    uint32_t* queue_out;
    unsigned long long* counts;
    uint64_t n;
    uint64_t h_m64;     // ceil(2^64 / H) for the non-power-of-two htable path
    uint32_t h_mask;    // H - 1 when H is a power of two
    uint32_t H;
    uint32_t Q;
    uint32_t q_mask;    // Q - 1 (power of two) or ~0u when Q >= H (identity)
    uint32_t q_m32;     // ceil(2^32 / Q): exact b % Q for b, Q < 2^16
    uint32_t pad_;
    uint64_t q_m64;     // ceil(2^64 / Q): exact b % Q for any 32-bit b, Q
};

// ------------------------------------------------------------- device -------
// Toeplitz hash of one 96-bit input (w0 = src ip, w1 = dst ip, w2 = ports) from
// the lane-replicated nibble tables.  Table t, value v, replica c lives at byte
// t*2048 + v*128 + c*4 of the static LDS LUT, so the byte address is the nibble
// moved to bits 7..10 OR the lane's replica offset (v_lshrrev + v_and_or_b32),
// and the table offset folds into the ds_read_b32 immediate.  lane4 must be
// opaque to the compiler (see rss_toeplitz_kernel): if it can prove the OR is
// disjoint it rewrites it as an add and splits v_and_or_b32 into two ops.
__device__ __forceinline__ uint32_t toeplitz_lut(const uint32_t* __restrict__ lut, uint32_t w0,
                                                 uint32_t w1, uint32_t w2, uint32_t lane4) {
    const char* base = reinterpret_cast<const char*>(lut);
    uint32_t r[RSS_NIBBLES];
#pragma unroll
    for (int t = 0; t < RSS_NIBBLES; ++t) {
        const uint32_t w = t < 8 ? w0 : (t < 16 ? w1 : w2);
        const int sh = 28 - 4 * (t & 7);  // nibble occupies bits sh..sh+3
        const uint32_t moved = sh >= 7 ? (w >> (sh - 7)) : (w << (7 - sh));
        const uint32_t off = (moved & 0x780u) | lane4;
        r[t] = *reinterpret_cast<const uint32_t*>(base + t * 2048 + off);
    }
    uint32_t h = 0;
#pragma unroll
    for (int t = 0; t < RSS_NIBBLES; ++t) h ^= r[t];
    return h;
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
    } else if constexpr (kQMode == QM_FAST16) {
        return __umulhi(p.q_m32 * b, p.Q);  // b < 2^16, Q < 2^16
    } else {
        const uint64_t low = p.q_m64 * (uint64_t)b;
        return (uint32_t)__umul64hi(low, (uint64_t)p.Q);
    }
}

template <int kHist>
__device__ __forceinline__ void count_queue(uint32_t* bins, uint32_t q, uint32_t lane,
                                            const LaunchParams& p) {
    if constexpr (kHist == HIST_PRIVATE) {
        __hip_atomic_fetch_add(&bins[q * kCopies + lane], 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (kHist == HIST_SHARED) {
        __hip_atomic_fetch_add(&bins[q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if constexpr (kHist == HIST_GLOBAL) {
        atomicAdd(&p.counts[q], 1ull);
    }
}

template <bool kHPow2, int kQMode, int kHist>
__device__ __forceinline__ void one_tuple(const uint32_t* lds, uint32_t* bins, uint64_t i,
                                          uint32_t lane, const LaunchParams& p) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(p.tuples) + 3 * i;
    const uint32_t h = toeplitz_lut(lds, src[0], src[1], src[2], lane * 4);
    const uint32_t q = queue_of<kQMode>(bucket_of<kHPow2>(h, p), p);
    if (p.hash_out) p.hash_out[i] = h;
    if (p.queue_out) p.queue_out[i] = q;
    count_queue<kHist>(bins, q, lane, p);
}

template <bool kHPow2, int kQMode, int kHist, bool kVec4>
__global__ __launch_bounds__(kBlock) void rss_toeplitz_kernel(const LaunchParams p) {
    __shared__ uint32_t smem[kLutDwords];  // static: table offsets fold into ds_read
    extern __shared__ uint32_t bins[];      // histogram bins, sized at launch
    const uint32_t tid = threadIdx.x;

    // Prologue: replicate the 24x16 nibble table 32x (entry-major, replica-minor).
    for (uint32_t e = tid; e < kLutDwords; e += kBlock) smem[e] = p.lut[e >> 9][(e >> 5) & 15];
    const uint32_t nbins =
        kHist == HIST_PRIVATE ? p.Q * kCopies : (kHist == HIST_SHARED ? p.Q : 0u);
    for (uint32_t e = tid; e < nbins; e += kBlock) bins[e] = 0;
    __syncthreads();

    const uint32_t lane = tid & (kCopies - 1);
    uint32_t lane4 = lane * 4;
    asm volatile("" : "+v"(lane4));  // hide the known-zero bits (see toeplitz_lut)
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + tid;
    const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
    uint64_t tail_begin = 0;

    if constexpr (kVec4) {
        // 4 consecutive tuples per lane: 48 B = 3 x dwordx4, 16-B aligned.
        const uint4* __restrict__ src = reinterpret_cast<const uint4*>(p.tuples);
        const uint64_t ngroups = p.n >> 2;
        for (uint64_t g = gtid; g < ngroups; g += gstride) {
            const uint4 a = src[3 * g + 0];
            const uint4 b = src[3 * g + 1];
            const uint4 c = src[3 * g + 2];
            uint4 h, q;
            h.x = toeplitz_lut(smem, a.x, a.y, a.z, lane4);
            h.y = toeplitz_lut(smem, a.w, b.x, b.y, lane4);
            h.z = toeplitz_lut(smem, b.z, b.w, c.x, lane4);
            h.w = toeplitz_lut(smem, c.y, c.z, c.w, lane4);
            q.x = queue_of<kQMode>(bucket_of<kHPow2>(h.x, p), p);
            q.y = queue_of<kQMode>(bucket_of<kHPow2>(h.y, p), p);
            q.z = queue_of<kQMode>(bucket_of<kHPow2>(h.z, p), p);
            q.w = queue_of<kQMode>(bucket_of<kHPow2>(h.w, p), p);
            if (p.hash_out) reinterpret_cast<uint4*>(p.hash_out)[g] = h;
            if (p.queue_out) reinterpret_cast<uint4*>(p.queue_out)[g] = q;
            count_queue<kHist>(bins, q.x, lane, p);
            count_queue<kHist>(bins, q.y, lane, p);
            count_queue<kHist>(bins, q.z, lane, p);
            count_queue<kHist>(bins, q.w, lane, p);
        }
        tail_begin = ngroups << 2;
    }
    for (uint64_t i = tail_begin + gtid; i < p.n; i += gstride)
        one_tuple<kHPow2, kQMode, kHist>(smem, bins, i, lane, p);

    // Epilogue: fold this workgroup's bins into the global uint64 counts.
    if constexpr (kHist == HIST_PRIVATE || kHist == HIST_SHARED) {
        __syncthreads();
        for (uint32_t q = tid; q < p.Q; q += kBlock) {
            uint32_t s;
            if constexpr (kHist == HIST_PRIVATE) {
                s = 0;
                for (uint32_t c = 0; c < kCopies; ++c) s += bins[q * kCopies + ((c + q) & 31)];
            } else {
                s = bins[q];
            }
            if (s) atomicAdd(&p.counts[q], (unsigned long long)s);
        }
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

// --------------------------------------------------------------- host -------
struct DeviceInfo {
    int cu_count = 0;
};

std::mutex g_dev_mutex;
std::vector<DeviceInfo> g_devices;

int device_info(DeviceInfo* out) {
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

template <bool kHPow2, int kQMode, int kHist>
KernelFn pick_vec(bool vec4) {
    return vec4 ? rss_toeplitz_kernel<kHPow2, kQMode, kHist, true>
                : rss_toeplitz_kernel<kHPow2, kQMode, kHist, false>;
}

template <bool kHPow2, int kQMode>
KernelFn pick_hist(int hist, bool vec4) {
    switch (hist) {
        case HIST_PRIVATE: return pick_vec<kHPow2, kQMode, HIST_PRIVATE>(vec4);
        case HIST_SHARED: return pick_vec<kHPow2, kQMode, HIST_SHARED>(vec4);
        case HIST_GLOBAL: return pick_vec<kHPow2, kQMode, HIST_GLOBAL>(vec4);
        default: return pick_vec<kHPow2, kQMode, HIST_NONE>(vec4);
    }
}

template <bool kHPow2>
KernelFn pick_queue(int qmode, int hist, bool vec4) {
    switch (qmode) {
        case QM_MASK: return pick_hist<kHPow2, QM_MASK>(hist, vec4);
        case QM_FAST16: return pick_hist<kHPow2, QM_FAST16>(hist, vec4);
        default: return pick_hist<kHPow2, QM_FAST32>(hist, vec4);
    }
}

bool is_pow2(uint32_t x) { return x && !(x & (x - 1)); }
bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

// ceil(2^64 / d) as Lemire's M = floor((2^64 - 1) / d) + 1 (wraps to 0 for d = 1,
// which still yields the correct remainder 0).
uint64_t magic64(uint32_t d) { return UINT64_MAX / d + 1; }
uint32_t magic32(uint32_t d) { return UINT32_MAX / d + 1; }

int launch_hash(const rss_key* key, const rss_tuple4* d_tuples, size_t n, uint32_t htable,
                uint32_t nqueues, uint32_t* d_hash, uint32_t* d_queue, uint64_t* d_counts,
                uint32_t flags, hipStream_t stream) {
    if (!key) return set_error(RSS_EINVAL, "rss_hash_device: key is NULL");
    if (key->len < RSS_KEY_MIN_BYTES)
        return set_error(RSS_EINVAL, "rss_hash_device: key not prepared (len=%u)", key->len);
    if (htable < 1 || nqueues < 1)
        return set_error(RSS_EINVAL, "rss_hash_device: htable (%u) and nqueues (%u) must be >= 1",
                         htable, nqueues);
    if (n && !d_tuples) return set_error(RSS_EINVAL, "rss_hash_device: tuples is NULL");
    if (d_counts && !(flags & RSS_FLAG_ACCUMULATE))
        RSS_HIP_CHECK(hipMemsetAsync(d_counts, 0, sizeof(uint64_t) * nqueues, stream));
    if (n == 0) return RSS_OK;

    LaunchParams p;
    memset(&p, 0, sizeof p);
    memcpy(p.lut, key->nibble_lut, sizeof p.lut);
    p.tuples = d_tuples;
    p.hash_out = d_hash;
    p.queue_out = d_queue;
    p.counts = reinterpret_cast<unsigned long long*>(d_counts);
    p.n = n;
    p.H = htable;
    p.Q = nqueues;
    const bool h_pow2 = is_pow2(htable);
    p.h_mask = htable - 1;
    p.h_m64 = magic64(htable);
    int qmode;
    if (nqueues >= htable) {  // bucket < htable <= nqueues: remainder is the bucket itself
        qmode = QM_MASK;
        p.q_mask = 0xFFFFFFFFu;
    } else if (is_pow2(nqueues)) {
        qmode = QM_MASK;
        p.q_mask = nqueues - 1;
    } else if (htable <= 65536u) {  // bucket < 2^16 and nqueues < htable <= 2^16
        qmode = QM_FAST16;
        p.q_m32 = magic32(nqueues);
    } else {
        qmode = QM_FAST32;
        p.q_m64 = magic64(nqueues);
    }
    int hist;
    uint32_t bin_bytes = 0;
    if (!d_counts) {
        hist = HIST_NONE;
    } else if ((uint64_t)nqueues * kCopies * 4 <= kBinBytesMax) {
        hist = HIST_PRIVATE;
        bin_bytes = nqueues * kCopies * 4;
    } else if ((uint64_t)nqueues * 4 <= kBinBytesMax) {
        hist = HIST_SHARED;
        bin_bytes = nqueues * 4;
    } else {
        hist = HIST_GLOBAL;
    }
    const bool vec4 = aligned16(d_tuples) && (!d_hash || aligned16(d_hash)) &&
                      (!d_queue || aligned16(d_queue));
    KernelFn fn = h_pow2 ? pick_queue<true>(qmode, hist, vec4) : pick_queue<false>(qmode, hist, vec4);

    DeviceInfo info;
    int rc = device_info(&info);
    if (rc) return rc;
    const uint64_t per_lane = vec4 ? 4 : 1;
    const uint64_t want = (n + per_lane * kBlock - 1) / (per_lane * kBlock);
    const uint64_t cap = (uint64_t)info.cu_count * kBlocksPerCU;
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    const uint32_t shmem = bin_bytes;  // dynamic part; the 48 KiB LUT is static
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kBlock), shmem, stream, p);
    RSS_HIP_CHECK(hipGetLastError());
    return RSS_OK;
}

}  // namespace

// ------------------------------------------------------------ C ABI ---------
struct rss_ctx {
    int device = 0;
    size_t chunk = 0;  // tuples per staging buffer
    hipStream_t stream[2] = {nullptr, nullptr};
    rss_tuple4* d_in[2] = {nullptr, nullptr};
    uint32_t* d_hash[2] = {nullptr, nullptr};
    uint32_t* d_queue[2] = {nullptr, nullptr};
    uint64_t* d_counts[2] = {nullptr, nullptr};
    uint32_t counts_cap = 0;
    rss_tuple4* h_in[2] = {nullptr, nullptr};
    uint32_t* h_hash[2] = {nullptr, nullptr};
    uint32_t* h_queue[2] = {nullptr, nullptr};
};

extern "C" {

int rss_abi_version(void) { return RSS_ABI_VERSION; }

const char* rss_last_error(void) { return g_last_error.c_str(); }

int rss_key_prepare(const uint8_t* key, size_t len, rss_key* out) {
    if (!key || !out) return set_error(RSS_EINVAL, "rss_key_prepare: NULL argument");
    if (len < RSS_KEY_MIN_BYTES)
        return set_error(RSS_EINVAL, "rss_key_prepare: key must hold >= %d bytes, got %zu",
                         RSS_KEY_MIN_BYTES, len);
    memset(out, 0, sizeof *out);
    out->len = (uint32_t)len;
    memcpy(out->bytes, key, len < RSS_KEY_MAX_BYTES ? len : RSS_KEY_MAX_BYTES);
    // After i one-bit rotations of the whole key (toeplitz.py:83-98) its leftmost
    // 32 bits are key bits (i + j) mod 8*len, j = 0..31.  For len >= 16 bytes the
    // index never wraps and only bytes 0..15 matter.
    const uint64_t nbits = (uint64_t)len * 8;
    auto bit = [&](uint64_t b) -> uint32_t { return (key[b >> 3] >> (7 - (b & 7))) & 1u; };
    for (int i = 0; i < RSS_INPUT_BITS; ++i) {
        uint32_t w = 0;
        for (int j = 0; j < 32; ++j) w = (w << 1) | bit(((uint64_t)i + j) % nbits);
        out->window[i] = w;
    }
    for (int t = 0; t < RSS_NIBBLES; ++t)
        for (uint32_t v = 0; v < 16; ++v) {
            uint32_t x = 0;
            for (int j = 0; j < 4; ++j)
                if (v & (8u >> j)) x ^= out->window[4 * t + j];
            out->nibble_lut[t][v] = x;
        }
    return RSS_OK;
}

int rss_device_count(int* out) {
    if (!out) return set_error(RSS_EINVAL, "rss_device_count: NULL argument");
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
                    uint32_t nqueues, uint32_t* d_hash, uint32_t* d_queue, uint64_t* d_counts,
                    uint32_t flags, void* stream) {
    return launch_hash(key, d_tuples, n, htable, nqueues, d_hash, d_queue, d_counts, flags,
                       static_cast<hipStream_t>(stream));
}

int rss_generate_tuples(uint64_t seed, uint64_t first_index, size_t n, rss_tuple4* d_tuples,
                        void* stream) {
    if (n == 0) return RSS_OK;
    if (!d_tuples) return set_error(RSS_EINVAL, "rss_generate_tuples: tuples is NULL");
    DeviceInfo info;
    int rc = device_info(&info);
    if (rc) return rc;
    const uint64_t want = (n + 255) / 256;
    const uint64_t cap = (uint64_t)info.cu_count * 8;
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    hipLaunchKernelGGL(rss_generate_kernel, dim3(grid), dim3(256), 0,
                       static_cast<hipStream_t>(stream), seed, first_index, (uint64_t)n,
                       reinterpret_cast<uint32_t*>(d_tuples));
    RSS_HIP_CHECK(hipGetLastError());
    return RSS_OK;
}

void rss_ctx_destroy(rss_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
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
    delete ctx;
}

int rss_ctx_create(int device, rss_ctx** out) {
    if (!out) return set_error(RSS_EINVAL, "rss_ctx_create: NULL argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        return set_error(RSS_ENODEV, "rss_ctx_create: no HIP device visible");
    }
    if (device < 0 || device >= ndev)
        return set_error(RSS_EINVAL, "rss_ctx_create: device %d out of range [0, %d)", device, ndev);
    hipDeviceProp_t prop;
    RSS_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_error(RSS_ENODEV, "rss_ctx_create: device %d is %s, this build targets gfx950",
                         device, prop.gcnArchName);
    rss_ctx* ctx = new rss_ctx();
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    for (int b = 0; b < 2 && e == hipSuccess; ++b)
        e = hipStreamCreateWithFlags(&ctx->stream[b], hipStreamNonBlocking);
    if (e != hipSuccess) {
        rss_ctx_destroy(ctx);
        return set_error(RSS_EIO, "rss_ctx_create: %s", hipGetErrorString(e));
    }
    *out = ctx;
    return RSS_OK;
}

static int ctx_reserve(rss_ctx* ctx, size_t chunk, uint32_t nqueues) {
    if (ctx->chunk < chunk) {
        for (int b = 0; b < 2; ++b) {
            (void)hipFree(ctx->d_in[b]);
            (void)hipFree(ctx->d_hash[b]);
            (void)hipFree(ctx->d_queue[b]);
            (void)hipHostFree(ctx->h_in[b]);
            (void)hipHostFree(ctx->h_hash[b]);
            (void)hipHostFree(ctx->h_queue[b]);
            ctx->d_in[b] = nullptr;
            ctx->d_hash[b] = ctx->d_queue[b] = nullptr;
            ctx->h_in[b] = nullptr;
            ctx->h_hash[b] = ctx->h_queue[b] = nullptr;
        }
        ctx->chunk = 0;
        for (int b = 0; b < 2; ++b) {
            RSS_HIP_CHECK(hipMalloc(&ctx->d_in[b], chunk * sizeof(rss_tuple4)));
            RSS_HIP_CHECK(hipMalloc(&ctx->d_hash[b], chunk * sizeof(uint32_t)));
            RSS_HIP_CHECK(hipMalloc(&ctx->d_queue[b], chunk * sizeof(uint32_t)));
            RSS_HIP_CHECK(hipHostMalloc(&ctx->h_in[b], chunk * sizeof(rss_tuple4), hipHostMallocDefault));
            RSS_HIP_CHECK(hipHostMalloc(&ctx->h_hash[b], chunk * sizeof(uint32_t), hipHostMallocDefault));
            RSS_HIP_CHECK(hipHostMalloc(&ctx->h_queue[b], chunk * sizeof(uint32_t), hipHostMallocDefault));
        }
        ctx->chunk = chunk;
    }
    if (ctx->counts_cap < nqueues) {
        for (int b = 0; b < 2; ++b) {
            (void)hipFree(ctx->d_counts[b]);
            ctx->d_counts[b] = nullptr;
        }
        ctx->counts_cap = 0;
        for (int b = 0; b < 2; ++b)
            RSS_HIP_CHECK(hipMalloc(&ctx->d_counts[b], sizeof(uint64_t) * nqueues));
        ctx->counts_cap = nqueues;
    }
    return RSS_OK;
}

int rss_hash_host(rss_ctx* ctx, const rss_key* key, const rss_tuple4* h_tuples, size_t n,
                  uint32_t htable, uint32_t nqueues, uint32_t* h_hash, uint32_t* h_queue,
                  uint64_t* h_counts, uint32_t flags) {
    if (!ctx) return set_error(RSS_EINVAL, "rss_hash_host: ctx is NULL");
    if (n && !h_tuples) return set_error(RSS_EINVAL, "rss_hash_host: tuples is NULL");
    if (htable < 1 || nqueues < 1)
        return set_error(RSS_EINVAL, "rss_hash_host: htable (%u) and nqueues (%u) must be >= 1",
                         htable, nqueues);
    RSS_HIP_CHECK(hipSetDevice(ctx->device));
    constexpr size_t kChunkMax = (size_t)1 << 22;  // 4M tuples: 48 MB in + 32 MB out per slot
    const size_t chunk = n < kChunkMax ? (n ? n : 1) : kChunkMax;
    int rc = ctx_reserve(ctx, chunk, nqueues);
    if (rc) return rc;
    for (int b = 0; b < 2; ++b)
        RSS_HIP_CHECK(hipMemsetAsync(ctx->d_counts[b], 0, sizeof(uint64_t) * nqueues, ctx->stream[b]));

    // Double-buffered pipeline: while slot b runs H2D -> kernel -> D2H on its
    // stream, the host fills the other slot's pinned input and drains its output.
    const size_t nchunks = (n + chunk - 1) / chunk;
    size_t pending_off[2] = {0, 0}, pending_len[2] = {0, 0};
    auto drain = [&](int b) -> int {
        RSS_HIP_CHECK(hipStreamSynchronize(ctx->stream[b]));
        if (pending_len[b]) {
            if (h_hash) memcpy(h_hash + pending_off[b], ctx->h_hash[b], pending_len[b] * 4);
            if (h_queue) memcpy(h_queue + pending_off[b], ctx->h_queue[b], pending_len[b] * 4);
            pending_len[b] = 0;
        }
        return RSS_OK;
    };
    for (size_t c = 0; c < nchunks; ++c) {
        const int b = (int)(c & 1);
        rc = drain(b);
        if (rc) return rc;
        const size_t off = c * chunk;
        const size_t len = (n - off) < chunk ? (n - off) : chunk;
        memcpy(ctx->h_in[b], h_tuples + off, len * sizeof(rss_tuple4));
        hipStream_t s = ctx->stream[b];
        RSS_HIP_CHECK(hipMemcpyAsync(ctx->d_in[b], ctx->h_in[b], len * sizeof(rss_tuple4),
                                     hipMemcpyHostToDevice, s));
        rc = launch_hash(key, ctx->d_in[b], len, htable, nqueues, h_hash ? ctx->d_hash[b] : nullptr,
                         h_queue ? ctx->d_queue[b] : nullptr, ctx->d_counts[b],
                         RSS_FLAG_ACCUMULATE, s);
        if (rc) return rc;
        if (h_hash)
            RSS_HIP_CHECK(hipMemcpyAsync(ctx->h_hash[b], ctx->d_hash[b], len * 4,
                                         hipMemcpyDeviceToHost, s));
        if (h_queue)
            RSS_HIP_CHECK(hipMemcpyAsync(ctx->h_queue[b], ctx->d_queue[b], len * 4,
                                         hipMemcpyDeviceToHost, s));
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

}  // extern "C"

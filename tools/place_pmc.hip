// place_pmc.hip -- the HBM placement tier under PMC counters (tool, not product).
//
// DESIGN.md §3 "Placement": the same full-u8 launch over the same data runs in a fast or a
// slow tier depending only on which allocations hold the input, hash and queue buffers.
// This program allocates the bench's buffer shapes (2 inputs of 12n B, K output pairs of
// 4n + n B, in a recorded order) and launches, for every (input, output pair) candidate:
//   2 untimed + R timed full-u8 launches, R hash-only launches, R queue-only launches
// (all rss_toeplitz_kernel, RSS_FLAG_ACCUMULATE so no memset dispatch in between), printing
// per-candidate HIP-event medians, virtual addresses and allocation order.  Run under
// `rocprofv3 --pmc <group>` (one counter group per process: tools/place_pmc.sh) the
// per-dispatch counters are joined to the candidates by tools/place_pmc_summarize.py
// through this fixed launch order.  A tier is a property of allocations in one process, so
// each pass re-measures its own candidates' times next to its counters.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/place_pmc.hip \
//          -L rss_simulator_nvidia_amd -lrss_toeplitz \
//          -Wl,-rpath,'$ORIGIN/../rss_simulator_nvidia_amd' -o tools/place_pmc
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rss_toeplitz.h"

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// The bench's byte mix without hashing (12 B read, 4 + 1 B written with nt stores,
// grid-stride, 4 tuples per lane -- the product kernel's access shape), recording for every
// workgroup its XCD (HW_REG_XCC_ID) and its start / end wall clock (100 MHz): does a slow
// placement slow every XCD, or do some XCDs finish late while the others idle?
__global__ __launch_bounds__(1024) void stream_trace(const uint4* __restrict__ src,
                                                     uint32_t* __restrict__ hash_out,
                                                     uint32_t* __restrict__ queue_out, uint64_t n,
                                                     unsigned long long* rec) {
    __shared__ unsigned long long t0;
    if (threadIdx.x == 0) t0 = wall_clock64();
    __syncthreads();
    const uint64_t ng = n >> 2;
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * 1024) {
        const uint4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
        uint32_t* o = hash_out + 4 * g;
        __builtin_nontemporal_store(a.x ^ a.y ^ a.z, o);
        __builtin_nontemporal_store(a.w ^ b.x ^ b.y, o + 1);
        __builtin_nontemporal_store(b.z ^ b.w ^ c.x, o + 2);
        __builtin_nontemporal_store(c.y ^ c.z ^ c.w, o + 3);
        __builtin_nontemporal_store((a.x ^ c.w) & 0x17171717u, queue_out + g);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        rec[3 * blockIdx.x + 0] = xcc & 0xFu;
        rec[3 * blockIdx.x + 1] = t0;
        rec[3 * blockIdx.x + 2] = wall_clock64();
    }
}

// The same stream with its tail balanced between workgroups: rows (one grid-stride step
// of the whole grid) [0, static_rows) are processed as above; the rest are handed out as
// units (one row x one workgroup slot = 1024 lane-groups) in increasing order through a
// global counter, one claim per workgroup in flight (prefetched one unit ahead), so a
// workgroup (an XCD) that streams faster takes more of the tail.  ctl[0] = next unit,
// ctl[1] = workgroups done; the last workgroup to finish resets both (self-resetting).
// rec as stream_trace, plus rec[3 * gridDim.x + w] = units workgroup w claimed.
__global__ __launch_bounds__(1024) void stream_bal(const uint4* __restrict__ src,
                                                   uint32_t* __restrict__ hash_out,
                                                   uint32_t* __restrict__ queue_out, uint64_t n,
                                                   unsigned long long* rec,
                                                   unsigned long long* ctl, uint64_t static_rows) {
    __shared__ unsigned long long t0, s_unit;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) t0 = wall_clock64();
    const uint64_t ng = n >> 2;
    const uint64_t G = (uint64_t)gridDim.x * 1024;
    const uint64_t nrows = (ng + G - 1) / G;
    const uint64_t srows = static_rows < nrows ? static_rows : nrows;
    const uint64_t first_unit = srows * gridDim.x, nunits = nrows * gridDim.x;
    auto body = [&](uint64_t g) {
        const uint4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
        uint32_t* o = hash_out + 4 * g;
        __builtin_nontemporal_store(a.x ^ a.y ^ a.z, o);
        __builtin_nontemporal_store(a.w ^ b.x ^ b.y, o + 1);
        __builtin_nontemporal_store(b.z ^ b.w ^ c.x, o + 2);
        __builtin_nontemporal_store(c.y ^ c.z ^ c.w, o + 3);
        __builtin_nontemporal_store((a.x ^ c.w) & 0x17171717u, queue_out + g);
    };
    unsigned long long claim = 0;
    if (tid == 0) claim = atomicAdd(&ctl[0], 1ull);  // first tail unit, in flight meanwhile
    for (uint64_t row = 0; row < srows; ++row) {
        const uint64_t g = row * G + (uint64_t)blockIdx.x * 1024 + tid;
        if (g < ng) body(g);
    }
    if (tid == 0) s_unit = claim;
    __syncthreads();
    uint64_t u = first_unit + s_unit;
    uint64_t mine = 0;
    while (u < nunits) {
        __syncthreads();  // every lane has read s_unit
        if (tid == 0) claim = atomicAdd(&ctl[0], 1ull);  // the next unit, while this one streams
        const uint64_t g = (u / gridDim.x) * G + (u % gridDim.x) * 1024 + tid;
        if (g < ng) body(g);
        ++mine;
        if (tid == 0) s_unit = claim;
        __syncthreads();
        u = first_unit + s_unit;
    }
    if (tid == 0) {
        // this workgroup's last claim was past the end: it claims no more; the last one
        // to get here resets the counters for the next launch
        if (atomicAdd(&ctl[1], 1ull) == gridDim.x - 1) {
            atomicExch(&ctl[0], 0ull);
            atomicExch(&ctl[1], 0ull);
        }
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        rec[3 * blockIdx.x + 0] = xcc & 0xFu;
        rec[3 * blockIdx.x + 1] = t0;
        rec[3 * blockIdx.x + 2] = wall_clock64();
        rec[3 * gridDim.x + blockIdx.x] = mine;
    }
}

int main(int argc, char** argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 12;      // output pairs
    const int R = argc > 2 ? atoi(argv[2]) : 5;       // timed launches per mode
    const uint64_t n = argc > 3 ? strtoull(argv[3], 0, 0) : (1ull << 28);
    const uint32_t H = 128, Q = 24;
    if (K < 1 || K > 64 || R < 1 || R > 50 || n == 0 || (n & 3)) {
        fprintf(stderr, "usage: place_pmc [K<=64] [R<=50] [n, multiple of 4]\n");
        return 2;
    }
    const uint8_t key_bytes[40] = {0x23, 0x0d, 0x44, 0x3d, 0x8c, 0x2c, 0x6e, 0x64, 0xd4, 0x1a,
                                   0xf3, 0x44, 0x49, 0x9b, 0x21, 0x74, 0xfd, 0x1a, 0x9d, 0xc1,
                                   0xdd, 0x76, 0x77, 0x37, 0x38, 0x51, 0x66, 0x85, 0x7b, 0xdc,
                                   0x48, 0xa8, 0x3e, 0x55, 0x08, 0xc1, 0x63, 0xaf, 0x01, 0x9d};
    rss_key key;
    if (rss_key_prepare(key_bytes, 40, &key)) return 1;

    // "ballast G": hold G GiB allocated (and touched) before the candidates, to see whether
    // the tier follows the allocation order / the physical range the allocator hands out
    const bool ballast_mode = argc > 4 && strcmp(argv[4], "ballast") == 0;
    const double ballast_gib = ballast_mode && argc > 5 ? atof(argv[5]) : 0.0;
    std::vector<void*> ballast;
    for (double got = 0; got + 0.5 <= ballast_gib; got += 1.0) {
        void* b;
        CK(hipMalloc(&b, 1ull << 30));
        CK(hipMemset(b, 0, 1ull << 30));
        ballast.push_back(b);
    }
    // allocation order as ResidentBatch: input 0, the output pairs (hash then queue), input 1
    int order = 0;
    void* in[2];
    std::vector<void*> hs(K), qs(K);
    std::vector<int> h_order(K), q_order(K);
    int in_order[2];
    CK(hipMalloc(&in[0], n * 12));
    in_order[0] = order++;
    for (int k = 0; k < K; ++k) {
        CK(hipMalloc(&hs[k], n * 4));
        h_order[k] = order++;
        CK(hipMalloc(&qs[k], n));
        q_order[k] = order++;
    }
    CK(hipMalloc(&in[1], n * 12));
    in_order[1] = order++;
    unsigned long long* counts;
    CK(hipMalloc(&counts, Q * 8));
    CK(hipMemset(counts, 0, Q * 8));
    for (int i = 0; i < 2; ++i)
        if (rss_generate_tuples(0x5EED, 0, n, (rss_tuple4*)in[i], nullptr)) return 1;
    CK(hipDeviceSynchronize());

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto launch = [&](int i, int k, bool h, bool q) {
        if (rss_hash_device(&key, (const rss_tuple4*)in[i], n, H, Q, h ? (uint32_t*)hs[k] : nullptr,
                            q ? qs[k] : nullptr, (uint64_t*)counts,
                            RSS_FLAG_QUEUE_U8 | RSS_FLAG_ACCUMULATE, nullptr)) {
            fprintf(stderr, "rss_hash_device: %s\n", rss_last_error());
            exit(1);
        }
    };
    auto median_of = [&](int i, int k, bool h, bool q) {
        std::vector<float> t(R);
        for (int r = 0; r < R; ++r) {
            CK(hipEventRecord(e0, nullptr));
            launch(i, k, h, q);
            CK(hipEventRecord(e1, nullptr));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&t[r], e0, e1));
        }
        std::sort(t.begin(), t.end());
        return t[R / 2];
    };

    if (ballast_mode) {  // full-u8 medians only, per candidate, with the ballast held
        const bool free_first = argc > 6 && strcmp(argv[6], "free") == 0;
        if (free_first) {  // release the ballast before timing (the candidates stay put)
            for (void* b : ballast) CK(hipFree(b));
            ballast.clear();
        }
        printf("ballast %.0f GiB%s:", ballast_gib, free_first ? " (freed)" : "");
        for (int i = 0; i < 2; ++i)
            for (int k = 0; k < K; ++k) {
                launch(i, k, true, true);
                launch(i, k, true, true);
                printf(" %.3f", median_of(i, k, true, true));
            }
        printf("\n");
        for (void* b : ballast) CK(hipFree(b));
        return 0;
    }
    const bool baltrace = argc > 4 && strcmp(argv[4], "balance") == 0;
    if (baltrace) {
        // per candidate: static stream vs tail-balanced stream at several static fractions
        // (same buffers, alternating), per-XCD last end and units taken
        int cus = 0;
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        unsigned long long *rec, *ctl;
        CK(hipMalloc(&rec, (size_t)cus * 4 * 8));
        CK(hipMalloc(&ctl, 16));
        CK(hipMemset(ctl, 0, 16));
        std::vector<unsigned long long> h(cus * 4);
        const uint64_t G = (uint64_t)cus * 1024, nrows = ((n >> 2) + G - 1) / G;
        const double fracs[4] = {1.0, 0.95, 0.90, 0.85};
        auto summarize = [&](const char* name, float ms, bool units) {
            CK(hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long tmin = ~0ull;
            for (int w = 0; w < cus; ++w) tmin = std::min(tmin, h[3 * w + 1]);
            double last[8] = {0};
            unsigned long long u[8] = {0};
            for (int w = 0; w < cus; ++w) {
                const int x = (int)(h[3 * w] & 7);
                last[x] = std::max(last[x], (h[3 * w + 2] - tmin) / 100.0);
                if (units) u[x] += h[3 * cus + w];
            }
            printf("  %-16s %.4f ms  last:", name, ms);
            for (int x = 0; x < 8; ++x) printf(" %.1f", last[x]);
            if (units) {
                printf("  units:");
                for (int x = 0; x < 8; ++x) printf(" %llu", u[x]);
            }
            printf("\n");
        };
        int cand = 0;
        for (int i = 0; i < 2; ++i)
            for (int k = 0; k < K; ++k, ++cand) {
                printf("bal cand %d in=%d out=%d full_ms=%.4f rows=%llu\n", cand, i, k,
                       median_of(i, k, true, true), (unsigned long long)nrows);
                for (int rep = 0; rep < 2; ++rep)
                    for (double f : fracs) {
                        const uint64_t srows = (uint64_t)(f * nrows);
                        std::vector<float> ts(R);
                        for (int r = 0; r < R; ++r) {
                            CK(hipEventRecord(e0, nullptr));
                            if (f >= 1.0)
                                hipLaunchKernelGGL(stream_trace, dim3(cus), dim3(1024), 0, nullptr,
                                                   (const uint4*)in[i], (uint32_t*)hs[k],
                                                   (uint32_t*)qs[k], n, rec);
                            else
                                hipLaunchKernelGGL(stream_bal, dim3(cus), dim3(1024), 0, nullptr,
                                                   (const uint4*)in[i], (uint32_t*)hs[k],
                                                   (uint32_t*)qs[k], n, rec, ctl, srows);
                            CK(hipEventRecord(e1, nullptr));
                            CK(hipEventSynchronize(e1));
                            CK(hipEventElapsedTime(&ts[r], e0, e1));
                        }
                        std::sort(ts.begin(), ts.end());
                        char name[32];
                        snprintf(name, sizeof name, f >= 1.0 ? "static" : "tail %.2f", 1.0 - f);
                        summarize(name, ts[R / 2], f < 1.0);
                    }
                fflush(stdout);
            }
        CK(hipFree(rec));
        CK(hipFree(ctl));
        return 0;
    }
    const bool wgtrace = argc > 4 && strcmp(argv[4], "wgtrace") == 0;
    if (wgtrace) {
        // per candidate: the product's full-u8 median, then the traced stream; per XCD the
        // number of workgroups, their mean duration and the last end, in us from the
        // earliest start (wall clock: 100 MHz)
        int cus = 0;
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        unsigned long long* rec;
        CK(hipMalloc(&rec, (size_t)cus * 3 * 8));
        std::vector<unsigned long long> h(cus * 3);
        int cand = 0;
        for (int i = 0; i < 2; ++i)
            for (int k = 0; k < K; ++k, ++cand) {
                launch(i, k, true, true);
                launch(i, k, true, true);
                const float full = median_of(i, k, true, true);
                std::vector<float> ts(R);
                for (int r = 0; r < R; ++r) {
                    CK(hipEventRecord(e0, nullptr));
                    hipLaunchKernelGGL(stream_trace, dim3(cus), dim3(1024), 0, nullptr,
                                       (const uint4*)in[i], (uint32_t*)hs[k], (uint32_t*)qs[k], n, rec);
                    CK(hipEventRecord(e1, nullptr));
                    CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&ts[r], e0, e1));
                }
                std::sort(ts.begin(), ts.end());
                CK(hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost));
                unsigned long long tmin = ~0ull;
                for (int w = 0; w < cus; ++w) tmin = std::min(tmin, h[3 * w + 1]);
                double dur[8] = {0}, last[8] = {0};
                int cnt[8] = {0};
                for (int w = 0; w < cus; ++w) {
                    const int x = (int)(h[3 * w] & 7);
                    cnt[x]++;
                    dur[x] += (h[3 * w + 2] - h[3 * w + 1]) / 100.0;
                    last[x] = std::max(last[x], (h[3 * w + 2] - tmin) / 100.0);
                }
                printf("wg cand %d in=%d out=%d full_ms=%.4f stream_ms=%.4f xcd:", cand, i, k, full,
                       ts[R / 2]);
                for (int x = 0; x < 8; ++x)
                    printf(" [%d n=%d mean=%.1f last=%.1f]", x, cnt[x], cnt[x] ? dur[x] / cnt[x] : 0.0,
                           last[x]);
                printf("\n");
                fflush(stdout);
            }
        CK(hipFree(rec));
        return 0;
    }

    printf("place_pmc n=%llu K=%d R=%d launches_per_candidate=%d "
           "(2 warm full, %d full, %d hash-only, %d queue-only; rss_toeplitz_kernel only)\n",
           (unsigned long long)n, K, R, 2 + 3 * R, R, R, R);
    int cand = 0;
    for (int i = 0; i < 2; ++i)
        for (int k = 0; k < K; ++k, ++cand) {
            launch(i, k, true, true);
            launch(i, k, true, true);
            const float full = median_of(i, k, true, true);
            const float honly = median_of(i, k, true, false);
            const float qonly = median_of(i, k, false, true);
            printf("cand %d in=%d out=%d order in=%d h=%d q=%d va in=%p h=%p q=%p "
                   "full_ms=%.4f hash_only_ms=%.4f queue_only_ms=%.4f\n",
                   cand, i, k, in_order[i], h_order[k], q_order[k], in[i], hs[k], qs[k], full,
                   honly, qonly);
            fflush(stdout);
        }
    CK(hipDeviceSynchronize());
    for (int k = 0; k < K; ++k) {
        CK(hipFree(hs[k]));
        CK(hipFree(qs[k]));
    }
    CK(hipFree(in[0]));
    CK(hipFree(in[1]));
    CK(hipFree(counts));
    return 0;
}

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

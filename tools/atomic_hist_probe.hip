// Can global u32 atomics histogram many queues at the stream rate?  (VERDICT r03 item 3's
// suggestion: per-XCD global u32 bins -- one copy per HW_REG_XCC_ID, 1 MiB at Q = 262144,
// inside an XCD's 4 MiB L2 -- added with non-returning atomics.)
//
// Each lane takes tuples i (grid-stride), derives a uniform queue q = splitmix64(i) % Q (no
// memory read: the time is the atomics alone) and adds 1 into bins[copy * Q + q] with a
// non-returning device-scope atomicAdd; copy = the workgroup's XCD (per-XCD bins) or 0 (one
// shared copy).  "none" computes q and keeps a per-lane checksum only: the ALU floor.  Every
// run checks that the bins sum to n (no add lost across XCDs).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/atomic_hist_probe tools/atomic_hist_probe.hip
//   tools/atomic_hist_probe [log2_n=28]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// mode 0: none (checksum), 1: one shared copy, 2: per-XCD copies
__global__ __launch_bounds__(1024) void probe(uint32_t* bins, uint32_t* sink, uint64_t n,
                                              uint32_t qmask, int mode) {
    uint32_t xcc = 0;
    if (mode == 2) asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uint32_t* b = bins + (size_t)(xcc & 7u) * (qmask + 1);
    const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t i = gtid; i < n; i += stride) {
        const uint32_t q = (uint32_t)splitmix(i) & qmask;
        if (mode == 0)
            acc += q;
        else
            __hip_atomic_fetch_add(&b[q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (mode == 0 && acc == 0x12345678u) sink[0] = acc;  // keeps the loop
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const uint64_t n = 1ull << lg;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *bins, *sink;
    const uint32_t qmax = 262144;
    CHECK(hipMalloc(&bins, sizeof(uint32_t) * qmax * 8));
    CHECK(hipMalloc(&sink, 4));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const char* names[] = {"none", "shared", "per_xcd"};
    for (uint32_t Q : {131072u, 262144u}) {
        for (int mode = 0; mode < 3; ++mode) {
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                CHECK(hipMemset(bins, 0, sizeof(uint32_t) * qmax * 8));
                CHECK(hipEventRecord(a));
                hipLaunchKernelGGL(probe, dim3(cus * 2), dim3(1024), 0, 0, bins, sink, n, Q - 1, mode);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, a, b));
                if (rep && ms < best) best = ms;  // rep 0 warms up
            }
            uint64_t total = 0;
            if (mode) {
                std::vector<uint32_t> h((size_t)qmax * 8);
                CHECK(hipMemcpy(h.data(), bins, h.size() * 4, hipMemcpyDeviceToHost));
                for (uint32_t v : h) total += v;
            }
            printf("{\"Q\": %u, \"mode\": \"%s\", \"n\": %llu, \"ms\": %.4f, \"G_adds_per_s\": %.2f, "
                   "\"sum_ok\": %s}\n",
                   Q, names[mode], (unsigned long long)n, best, mode ? n / (best * 1e6) : 0.0,
                   mode ? (total == n ? "true" : "false") : "null");
            fflush(stdout);
        }
    }
    return 0;
}

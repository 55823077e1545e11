// kbench.hip -- design-space microbenchmark for the Toeplitz kernel (tool, not product).
//
// Times, on 2^28 resident synthetic tuples (H = 128, Q = 24), on one MI355X:
//   * memory ceilings: read-only (12 B/tuple) and read+write (20 B/tuple) streams
//     with the same access shape as the product kernel;
//   * LUT variants: chunk width B in {4, 6, 8} bits, LDS replicas R, workgroup
//     size, tuples per lane per iteration, software prefetch, full vs counts-only;
// and checks every variant's hash/queue/count output against the product kernel
// (librss_toeplitz.so through the C ABI).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/kbench.hip \
//          -L rss_simulator_nvidia_amd -lrss_toeplitz -o tools/kbench
#include <hip/hip_runtime.h>

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

struct Params {
    const uint32_t* tuples;
    uint32_t* hash_out;
    uint32_t* queue_out;
    unsigned long long* counts;
    uint64_t n;
    uint32_t Q, q_m32, h_mask;
    uint32_t window[96];
};

// ------------------------------------------------------------ memory ceilings
template <bool kWrite>
__global__ __launch_bounds__(1024) void mem_ceiling(Params p) {
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    uint32_t acc = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * 1024) {
        uint4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
        uint4 h = make_uint4(a.x ^ a.y ^ a.z, a.w ^ b.x ^ b.y, b.z ^ b.w ^ c.x, c.y ^ c.z ^ c.w);
        if constexpr (kWrite) {
            reinterpret_cast<uint4*>(p.hash_out)[g] = h;
            reinterpret_cast<uint4*>(p.queue_out)[g] = make_uint4(h.x & 23, h.y & 23, h.z & 23, h.w & 23);
        } else {
            acc ^= h.x ^ h.y ^ h.z ^ h.w;
        }
    }
    if (!kWrite && acc == 0x12345678u) p.counts[0] = acc;  // keep the loads alive
}

// 12 B read + 4 B hash + 1 B queue written, nontemporal stores: the bench's byte mix
__global__ __launch_bounds__(1024) void mem_ceiling_q8(Params p) {
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * 1024) {
        uint4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
        uint32_t* o = p.hash_out + 4 * g;
        __builtin_nontemporal_store(a.x ^ a.y ^ a.z, o);
        __builtin_nontemporal_store(a.w ^ b.x ^ b.y, o + 1);
        __builtin_nontemporal_store(b.z ^ b.w ^ c.x, o + 2);
        __builtin_nontemporal_store(c.y ^ c.z ^ c.w, o + 3);
        __builtin_nontemporal_store((a.x ^ c.w) & 0x17171717u, p.queue_out + g);
    }
}

// IPv6 byte mix: 36 B read (9 x 16-B loads per lane for 4 tuples) + 4 B hash + 1 B queue
__global__ __launch_bounds__(1024) void mem_ceiling6_q8(Params p) {
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * 1024) {
        uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint4 x = src[9 * g + k];
            acc[k & 3] ^= x.x ^ x.y ^ x.z ^ x.w;
        }
        uint32_t* o = p.hash_out + 4 * g;
        __builtin_nontemporal_store(acc[0], o);
        __builtin_nontemporal_store(acc[1], o + 1);
        __builtin_nontemporal_store(acc[2], o + 2);
        __builtin_nontemporal_store(acc[3], o + 3);
        __builtin_nontemporal_store((acc[0] ^ acc[3]) & 0x17171717u, p.queue_out + g);
    }
}

// the same IPv6 byte mix with lane-contiguous loads: instruction k of a wave reads bytes
// [1024 k, 1024 k + 1024) of the wave's 9 KiB block (256 tuples), 16 B per lane -- the shape a
// kernel that reassembled tuples across lanes would read; kRead = read-only (36 R)
template <bool kRead>
__global__ __launch_bounds__(1024) void mem_ceiling6_contig(Params p) {
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * 1024 + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * 1024) >> 6;
    const uint64_t nblocks = p.n >> 8;  // 256 tuples = 576 uint4 per block
    uint32_t keep = 0;
    for (uint64_t b = wave; b < nblocks; b += nwaves) {
        const uint4* blk = src + b * 576;
        uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint4 x = blk[64 * k + lane];
            acc[k & 3] ^= x.x ^ x.y ^ x.z ^ x.w;
        }
        if constexpr (kRead) {
            keep ^= acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
        } else {
            const uint64_t g = b * 64 + lane;  // the lane's 4 tuples' outputs, as the product
            uint32_t* o = p.hash_out + 4 * g;
            __builtin_nontemporal_store(acc[0], o);
            __builtin_nontemporal_store(acc[1], o + 1);
            __builtin_nontemporal_store(acc[2], o + 2);
            __builtin_nontemporal_store(acc[3], o + 3);
            __builtin_nontemporal_store((acc[0] ^ acc[3]) & 0x17171717u, p.queue_out + g);
        }
    }
    if (kRead && keep == 0x12345678u) p.counts[0] = keep;
}

// IPv6 read-only stream in the product's shape (9 x 16-B loads per lane at a 144-B stride)
__global__ __launch_bounds__(1024) void mem_ceiling6_read(Params p) {
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    uint32_t keep = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * 1024) {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint4 x = src[9 * g + k];
            keep ^= x.x ^ x.y ^ x.z ^ x.w;
        }
    }
    if (keep == 0x12345678u) p.counts[0] = keep;
}

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
// practical HBM ceilings for other read / write mixes on the same box: a float4 copy
// (1 R : 1 W, the microarch guide's 6.29 TB/s shape) and a write-only fill
__global__ __launch_bounds__(1024) void mem_copy16(const uint4* __restrict__ src,
                                                   uint4* __restrict__ dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 1024)
        dst[i] = src[i];
}
__global__ __launch_bounds__(1024) void mem_fill16(uint4* __restrict__ dst, uint64_t n16) {
    const u32x4v v = {threadIdx.x, blockIdx.x, 7u, 9u};
    u32x4v* d = reinterpret_cast<u32x4v*>(dst);
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 1024)
        __builtin_nontemporal_store(v, d + i);
}

// access-shape probes for the 12R+5W mix (outputs not meaningful: memory timing only).
// kShape 0: the product's shape (lane reads its 4 tuples as 3 x 16 B at a 48-B stride);
// 1: lane-contiguous loads (instruction k of a wave reads bytes [1024k, 1024k+1024) of the
// wave's 3 KiB block), same 5 B/tuple of stores; 2: as 0 with the queue bytes of 4
// consecutive groups kept in registers and written as one 16-B store (lane owns 16
// consecutive tuples per iteration: 12 x 16-B loads, 4 x 16-B hash stores)
template <int kShape>
__global__ __launch_bounds__(1024) void mem_shape(Params p) {
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    const uint32_t lane = threadIdx.x & 63;
    if constexpr (kShape == 3 || kShape == 4) {
        // whole tuples per load: a wave's block is 256 tuples; instruction j loads tuples
        // 64j + lane (one 12-B dwordx3 per lane = 768 contiguous bytes per instruction).
        // kShape 3: hash as 4 dword stores (tuples 64j + lane), queue as 4 byte stores;
        // kShape 4: queue bytes regrouped through ds_bpermute so lane l stores the 4 queue
        // bytes of tuples 4l..4l+3 as one dword (as the product), hashes as in 3
        struct U3 { uint32_t x, y, z; };
        const U3* t3 = reinterpret_cast<const U3*>(p.tuples);
        const uint64_t wave = ((uint64_t)blockIdx.x * 1024 + threadIdx.x) >> 6;
        const uint64_t nwaves = ((uint64_t)gridDim.x * 1024) >> 6;
        const uint64_t nblocks = p.n >> 8;
        uint8_t* q8 = reinterpret_cast<uint8_t*>(p.queue_out);
        for (uint64_t b = wave; b < nblocks; b += nwaves) {
            const uint64_t base = b << 8;
            uint32_t h[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const U3 t = t3[base + 64 * j + lane];
                h[j] = t.x ^ t.y ^ t.z;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(h[j], p.hash_out + base + 64 * j + lane);
            if constexpr (kShape == 3) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    __builtin_nontemporal_store((uint8_t)(h[j] & 0x17), q8 + base + 64 * j + lane);
            } else {
                // lane l needs queues of tuples 4l + i, held by lane (4l + i) % 64 in h[(4l + i) / 64]
                uint32_t packed = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t src = (4 * lane + i) & 63, j = (4 * lane + i) >> 6;
                    uint32_t v[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) v[jj] = __builtin_amdgcn_ds_bpermute(src << 2, h[jj] & 0x17);
                    packed |= (j == 0 ? v[0] : j == 1 ? v[1] : j == 2 ? v[2] : v[3]) << (8 * i);
                }
                __builtin_nontemporal_store(packed, reinterpret_cast<uint32_t*>(q8) + (base >> 2) + lane);
            }
        }
        return;
    }
    if constexpr (kShape == 2) {
        const uint64_t ng16 = ng >> 2;
        for (uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x; g < ng16; g += (uint64_t)gridDim.x * 1024) {
            uint32_t qv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t gg = 4 * g + j;
                uint4 a = src[3 * gg], b = src[3 * gg + 1], c = src[3 * gg + 2];
                uint32_t* o = p.hash_out + 4 * gg;
                __builtin_nontemporal_store(a.x ^ a.y ^ a.z, o);
                __builtin_nontemporal_store(a.w ^ b.x ^ b.y, o + 1);
                __builtin_nontemporal_store(b.z ^ b.w ^ c.x, o + 2);
                __builtin_nontemporal_store(c.y ^ c.z ^ c.w, o + 3);
                qv[j] = (a.x ^ c.w) & 0x17171717u;
            }
            uint32_t* oq = p.queue_out + 4 * g;
            __builtin_nontemporal_store(qv[0], oq);
            __builtin_nontemporal_store(qv[1], oq + 1);
            __builtin_nontemporal_store(qv[2], oq + 2);
            __builtin_nontemporal_store(qv[3], oq + 3);
        }
        return;
    }
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * 1024) {
        uint4 a, b, c;
        if constexpr (kShape == 0) {
            a = src[3 * g]; b = src[3 * g + 1]; c = src[3 * g + 2];
        } else {
            const uint64_t w0 = 3 * (g - lane);  // the wave's first uint4
            if (w0 + 192 > 3 * ng) { a = src[3 * g]; b = src[3 * g + 1]; c = src[3 * g + 2]; }
            else { a = src[w0 + lane]; b = src[w0 + 64 + lane]; c = src[w0 + 128 + lane]; }
        }
        uint32_t* o = p.hash_out + 4 * g;
        __builtin_nontemporal_store(a.x ^ a.y ^ a.z, o);
        __builtin_nontemporal_store(a.w ^ b.x ^ b.y, o + 1);
        __builtin_nontemporal_store(b.z ^ b.w ^ c.x, o + 2);
        __builtin_nontemporal_store(c.y ^ c.z ^ c.w, o + 3);
        __builtin_nontemporal_store((a.x ^ c.w) & 0x17171717u, p.queue_out + g);
    }
}

// store-shape probes for the 12R+5W mix: kMode 0 = plain stores, 1 = hash only (12R+4W),
// 2 = queue bytes gathered through LDS into one 16-B store per lane every 4th group
template <int kMode>
__global__ __launch_bounds__(1024) void mem_probe(Params p) {
    __shared__ uint32_t stage[1024];
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x; g < ng; g += stride) {
        uint4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
        uint4 h = make_uint4(a.x ^ a.y ^ a.z, a.w ^ b.x ^ b.y, b.z ^ b.w ^ c.x, c.y ^ c.z ^ c.w);
        const uint32_t qw = (a.x ^ c.w) & 0x17171717u;
        if (kMode == 0) {
            reinterpret_cast<uint4*>(p.hash_out)[g] = h;
            p.queue_out[g] = qw;
        } else if (kMode == 1) {
            uint32_t* o = p.hash_out + 4 * g;
            __builtin_nontemporal_store(h.x, o); __builtin_nontemporal_store(h.y, o + 1);
            __builtin_nontemporal_store(h.z, o + 2); __builtin_nontemporal_store(h.w, o + 3);
        } else {
            uint32_t* o = p.hash_out + 4 * g;
            __builtin_nontemporal_store(h.x, o); __builtin_nontemporal_store(h.y, o + 1);
            __builtin_nontemporal_store(h.z, o + 2); __builtin_nontemporal_store(h.w, o + 3);
            // lane l of each group of 4 lanes gathers the 16 queue bytes of lanes 4k..4k+3
            stage[threadIdx.x] = qw;
            __builtin_amdgcn_wave_barrier();
            if ((threadIdx.x & 3) == 0) {
                const uint32_t* s4 = stage + threadIdx.x;
                uint32_t* oq = p.queue_out + g;  // g is 4-aligned for lane%4 == 0
                __builtin_nontemporal_store(s4[0], oq); __builtin_nontemporal_store(s4[1], oq + 1);
                __builtin_nontemporal_store(s4[2], oq + 2); __builtin_nontemporal_store(s4[3], oq + 3);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// read-policy / traversal probes: kNT = nontemporal loads, kChunk = each workgroup
// streams one contiguous slice instead of grid-stride, kWrite = 12R+5W (nt stores)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool kNT, bool kChunk, bool kWrite>
__global__ __launch_bounds__(1024) void mem_stream(Params p) {
    const u32x4* src = reinterpret_cast<const u32x4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    uint64_t g0, g1, step;
    if (kChunk) {
        const uint64_t per = (ng + gridDim.x - 1) / gridDim.x;
        g0 = (uint64_t)blockIdx.x * per + threadIdx.x;
        g1 = min(ng, (uint64_t)(blockIdx.x + 1) * per);
        step = 1024;
    } else {
        g0 = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
        g1 = ng;
        step = (uint64_t)gridDim.x * 1024;
    }
    uint32_t acc = 0;
    for (uint64_t g = g0; g < g1; g += step) {
        u32x4 a, b, c;
        if (kNT) {
            a = __builtin_nontemporal_load(src + 3 * g);
            b = __builtin_nontemporal_load(src + 3 * g + 1);
            c = __builtin_nontemporal_load(src + 3 * g + 2);
        } else {
            a = src[3 * g]; b = src[3 * g + 1]; c = src[3 * g + 2];
        }
        const uint32_t h0 = a.x ^ a.y ^ a.z, h1 = a.w ^ b.x ^ b.y, h2 = b.z ^ b.w ^ c.x,
                       h3 = c.y ^ c.z ^ c.w;
        if (kWrite) {
            uint32_t* o = p.hash_out + 4 * g;
            __builtin_nontemporal_store(h0, o); __builtin_nontemporal_store(h1, o + 1);
            __builtin_nontemporal_store(h2, o + 2); __builtin_nontemporal_store(h3, o + 3);
            __builtin_nontemporal_store((a.x ^ c.w) & 0x17171717u, p.queue_out + g);
        } else {
            acc ^= h0 ^ h1 ^ h2 ^ h3;
        }
    }
    if (!kWrite && acc == 0x12345678u) p.counts[0] = acc;
}

// store-policy / mapping probes for the 12R+5W mix (the bench's byte mix):
//   kPol 0 = nt stores (as product), 1 = sc1 stores, 2 = sc0 sc1 stores, 3 = sc0 sc1 nt,
//   4 = plain stores; kXcd = workgroup w streams tiles of XCD (w % 8)'s contiguous eighth;
//   kUnroll = 2 iterations' loads issued before either is consumed
template <int kPol>
__device__ __forceinline__ void store4(uint32_t* dst, u32x4 v) {
    if constexpr (kPol == 0) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
    } else if constexpr (kPol == 1) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(v) : "memory");
    } else if constexpr (kPol == 2) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(dst), "v"(v) : "memory");
    } else if constexpr (kPol == 3) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(dst), "v"(v) : "memory");
    } else {
        *reinterpret_cast<u32x4*>(dst) = v;
    }
}
template <int kPol>
__device__ __forceinline__ void store1(uint32_t* dst, uint32_t v) {
    if constexpr (kPol == 0) {
        __builtin_nontemporal_store(v, dst);
    } else if constexpr (kPol == 1) {
        asm volatile("global_store_dword %0, %1, off sc1" ::"v"(dst), "v"(v) : "memory");
    } else if constexpr (kPol == 2) {
        asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(dst), "v"(v) : "memory");
    } else if constexpr (kPol == 3) {
        asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(dst), "v"(v) : "memory");
    } else {
        *dst = v;
    }
}

template <int kPol, bool kXcd, bool kUnroll>
__global__ __launch_bounds__(1024) void mem_policy(Params p) {
    const u32x4* src = reinterpret_cast<const u32x4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    uint64_t g0, step;
    if (kXcd) {  // grid = 8 * m workgroups; XCD x = w % 8 owns groups [x*ng/8, (x+1)*ng/8)
        const uint32_t x = blockIdx.x & 7, l = blockIdx.x >> 3, m = gridDim.x >> 3;
        g0 = x * (ng / 8) + (uint64_t)l * 1024 + threadIdx.x;
        step = (uint64_t)m * 1024;
        const uint64_t g1 = (x + 1) * (ng / 8);
        for (uint64_t g = g0; g < g1; g += step) {
            u32x4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
            u32x4 h = {a.x ^ a.y ^ a.z, a.w ^ b.x ^ b.y, b.z ^ b.w ^ c.x, c.y ^ c.z ^ c.w};
            store4<kPol>(p.hash_out + 4 * g, h);
            store1<kPol>(p.queue_out + g, (a.x ^ c.w) & 0x17171717u);
        }
        return;
    }
    g0 = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    step = (uint64_t)gridDim.x * 1024;
    uint64_t g = g0;
    if (kUnroll) {
        for (; g + step < ng; g += 2 * step) {
            const uint64_t g2 = g + step;
            u32x4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
            u32x4 a2 = src[3 * g2], b2 = src[3 * g2 + 1], c2 = src[3 * g2 + 2];
            u32x4 h = {a.x ^ a.y ^ a.z, a.w ^ b.x ^ b.y, b.z ^ b.w ^ c.x, c.y ^ c.z ^ c.w};
            u32x4 h2 = {a2.x ^ a2.y ^ a2.z, a2.w ^ b2.x ^ b2.y, b2.z ^ b2.w ^ c2.x, c2.y ^ c2.z ^ c2.w};
            store4<kPol>(p.hash_out + 4 * g, h);
            store1<kPol>(p.queue_out + g, (a.x ^ c.w) & 0x17171717u);
            store4<kPol>(p.hash_out + 4 * g2, h2);
            store1<kPol>(p.queue_out + g2, (a2.x ^ c2.w) & 0x17171717u);
        }
    }
    for (; g < ng; g += step) {
        u32x4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
        u32x4 h = {a.x ^ a.y ^ a.z, a.w ^ b.x ^ b.y, b.z ^ b.w ^ c.x, c.y ^ c.z ^ c.w};
        store4<kPol>(p.hash_out + 4 * g, h);
        store1<kPol>(p.queue_out + g, (a.x ^ c.w) & 0x17171717u);
    }
}

// work-distribution probe for the 12R+5W mix: instead of a static grid-stride share,
// every wave claims chunks of kIters x 64 lane-groups (4 tuples each) from eight
// per-XCD heads (own XCD first, then the others), so a CU / XCD that streams slower
// is helped by the rest at the end of the launch.  heads[8] must be zero at launch.
template <int kIters, bool kWrite>
__global__ __launch_bounds__(1024) void mem_dyn(Params p, unsigned* heads) {
    const u32x4* src = reinterpret_cast<const u32x4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    constexpr uint64_t kChunk = (uint64_t)kIters * 64;
    const uint64_t nchunks = (ng + kChunk - 1) / kChunk;
    const uint32_t per_head = (uint32_t)((nchunks + 7) / 8);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7;
    uint32_t k = 0;  // heads found empty so far (wave-uniform)
    auto claim = [&]() -> uint64_t {
        while (k < 8) {
            const uint32_t h = (xcd + k) & 7;
            uint32_t v = 0;
            if (lane == 0) v = atomicAdd(&heads[h], 1u);
            v = __builtin_amdgcn_readfirstlane(v);
            const uint64_t c = (uint64_t)h * per_head + v;
            if (v < per_head && c < nchunks) return c;
            ++k;
        }
        return ~0ull;
    };
    uint32_t acc = 0;
    uint64_t c = claim();
    while (c != ~0ull) {
        const uint64_t next = claim();  // in flight while this chunk streams
        const uint64_t g1 = min(ng, (c + 1) * kChunk);
        for (uint64_t g = c * kChunk + lane; g < g1; g += 64) {
            const u32x4 a = src[3 * g], b = src[3 * g + 1], cc = src[3 * g + 2];
            const uint32_t h0 = a.x ^ a.y ^ a.z, h1 = a.w ^ b.x ^ b.y, h2 = b.z ^ b.w ^ cc.x,
                           h3 = cc.y ^ cc.z ^ cc.w;
            if (kWrite) {
                uint32_t* o = p.hash_out + 4 * g;
                __builtin_nontemporal_store(h0, o); __builtin_nontemporal_store(h1, o + 1);
                __builtin_nontemporal_store(h2, o + 2); __builtin_nontemporal_store(h3, o + 3);
                __builtin_nontemporal_store((a.x ^ cc.w) & 0x17171717u, p.queue_out + g);
            } else {
                acc ^= h0 ^ h1 ^ h2 ^ h3;
            }
        }
        c = next;
    }
    if (!kWrite && acc == 0x12345678u) p.counts[0] = acc;
}

// ------------------------------------------------------------ LUT variants
// chunk t covers input bits [t*B, t*B + B) of the 96-bit MSB-first string.
template <int B>
__device__ __forceinline__ uint32_t chunk_addr(const uint32_t (&w)[3], int t, uint32_t lane4,
                                               int rshift) {
    // returns (chunk value << rshift) | lane4, rshift = log2(R * 4)
    const int s = t * B, wi = s >> 5, o = s & 31;
    const uint32_t mask = ((1u << B) - 1) << rshift;
    if (o + B <= 32) {
        const int sh = 32 - o - B - rshift;  // right shift that lands the chunk at rshift
        const uint32_t moved = sh >= 0 ? (w[wi] >> sh) : (w[wi] << -sh);
        return (moved & mask) | lane4;
    }
    const uint32_t v = __builtin_amdgcn_alignbit(w[wi], w[wi + 1], 64 - o - B);
    return ((v << rshift) & mask) | lane4;
}

template <int B, int R>
__device__ __forceinline__ uint32_t hash_lut(const char* lds, const uint32_t (&w)[3], uint32_t lane4) {
    constexpr int C = 96 / B, E = 1 << B;
    constexpr int RS = R == 32 ? 7 : (R == 16 ? 6 : (R == 8 ? 5 : (R == 4 ? 4 : (R == 2 ? 3 : 2))));
    constexpr int TB = E * R * 4;  // table bytes
    uint32_t r[C];
#pragma unroll
    for (int t = 0; t < C; ++t)
        r[t] = *reinterpret_cast<const uint32_t*>(lds + t * TB + chunk_addr<B>(w, t, lane4, RS));
    uint32_t h = 0;
#pragma unroll
    for (int t = 0; t < C; ++t) h ^= r[t];
    return h;
}

// Nine 11/10-bit tables (the key-search partition with 4-byte entries): 60 KiB, so two
// 1024-thread workgroups fit a CU (32 waves instead of 16), at 9 lookups per tuple
// instead of 8.  Every table base is below 64 KiB: it folds into the ds_read offset.
__host__ __device__ constexpr int t9_bit(int t, int b) {  // input bit of index bit b
    return t == 0 ? 31 - b : t == 1 ? 20 - b : t == 2 ? 63 - b
         : t == 3 ? (b < 5 ? 84 - b : 73 - b)
         : t == 4 ? 9 - b : t == 5 ? 52 - b : t == 6 ? 95 - b : t == 7 ? 79 - b : 41 - b;
}
__host__ __device__ constexpr uint32_t t9_base(int t) {
    return t == 0 ? 0u : t == 1 ? 8192u : t == 2 ? 16384u : t == 3 ? 24576u : t == 4 ? 28672u
         : t == 5 ? 32768u : t == 6 ? 40960u : t == 7 ? 49152u : 57344u;
}
__host__ __device__ constexpr int t9_width(int t) { return (t == 3 || t == 4 || t == 8) ? 10 : 11; }

template <int kT>
__device__ __forceinline__ uint32_t t9_off(uint32_t w0, uint32_t w1, uint32_t w2) {
    if constexpr (kT == 0) return (w0 << 2) & 0x1FFCu;
    if constexpr (kT == 1) return (w0 >> 9) & 0x1FFCu;
    if constexpr (kT == 2) return (w1 << 2) & 0x1FFCu;
    if constexpr (kT == 3) return ((w2 >> 9) & 0x7Cu) | ((w2 >> 20) & 0xF80u);
    if constexpr (kT == 4) return (w0 >> 20) & 0xFFCu;
    if constexpr (kT == 5) return (w1 >> 9) & 0x1FFCu;
    if constexpr (kT == 6) return (w2 << 2) & 0x1FFCu;
    if constexpr (kT == 7) return (w2 >> 14) & 0x1FFCu;
    return (w1 >> 20) & 0xFFCu;
}
template <int kT>
__device__ __forceinline__ uint32_t t9_term(const char* lds, uint32_t w0, uint32_t w1, uint32_t w2) {
    return *reinterpret_cast<const uint32_t*>(lds + t9_base(kT) + t9_off<kT>(w0, w1, w2));
}
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t hash9(const char* l, uint32_t w0, uint32_t w1, uint32_t w2) {
    return x3(x3(t9_term<0>(l, w0, w1, w2), t9_term<1>(l, w0, w1, w2), t9_term<2>(l, w0, w1, w2)),
              x3(t9_term<3>(l, w0, w1, w2), t9_term<4>(l, w0, w1, w2), t9_term<5>(l, w0, w1, w2)),
              x3(t9_term<6>(l, w0, w1, w2), t9_term<7>(l, w0, w1, w2), t9_term<8>(l, w0, w1, w2)));
}
template <int kT>
__device__ __forceinline__ void t9_build(uint32_t* lut, const uint32_t* window, uint32_t tid) {
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 10; ++j) x ^= ((tid >> j) & 1u) ? window[t9_bit(kT, j)] : 0u;
    uint32_t* dst = lut + t9_base(kT) / 4;
    dst[tid] = x;
    if constexpr (t9_width(kT) == 11) dst[tid + 1024] = x ^ window[t9_bit(kT, 10)];
}

template <bool kWrite>
__global__ __launch_bounds__(1024, 2) void lut9_kernel(Params p) {
    __shared__ uint32_t lut[61440 / 4];
    __shared__ uint32_t bins[24 * 32];
    const uint32_t tid = threadIdx.x;
    t9_build<0>(lut, p.window, tid); t9_build<1>(lut, p.window, tid); t9_build<2>(lut, p.window, tid);
    t9_build<3>(lut, p.window, tid); t9_build<4>(lut, p.window, tid); t9_build<5>(lut, p.window, tid);
    t9_build<6>(lut, p.window, tid); t9_build<7>(lut, p.window, tid); t9_build<8>(lut, p.window, tid);
    for (uint32_t e = tid; e < p.Q * 32; e += 1024) bins[e] = 0;
    __syncthreads();
    const char* lds = reinterpret_cast<const char*>(lut);
    const uint32_t col = tid & 31;
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + tid; g < ng; g += stride) {
        const uint4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
        uint32_t h[4] = {hash9(lds, a.x, a.y, a.z), hash9(lds, a.w, b.x, b.y),
                         hash9(lds, b.z, b.w, c.x), hash9(lds, c.y, c.z, c.w)};
        uint32_t q[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) q[t] = __umulhi(p.q_m32 * (h[t] & p.h_mask), p.Q);
        if (kWrite) {
            uint32_t* o = p.hash_out + 4 * g;
            __builtin_nontemporal_store(h[0], o); __builtin_nontemporal_store(h[1], o + 1);
            __builtin_nontemporal_store(h[2], o + 2); __builtin_nontemporal_store(h[3], o + 3);
            __builtin_nontemporal_store(q[0] | q[1] << 8 | q[2] << 16 | q[3] << 24, p.queue_out + g);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
            __hip_atomic_fetch_add(&bins[q[t] * 32 + col], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    for (uint32_t k = tid; k < p.Q; k += 1024) {
        uint32_t s = 0;
        for (uint32_t c2 = 0; c2 < 32; ++c2) s += bins[k * 32 + ((c2 + k) & 31)];
        if (s) atomicAdd(&p.counts[k], (unsigned long long)s);
    }
}

template <int B, int R, int BLOCK, bool kWrite, bool kPrefetch, bool kQ8 = false, bool kNT = false>
__global__ __launch_bounds__(BLOCK) void lut_kernel(Params p) {
    constexpr int C = 96 / B, E = 1 << B;
    constexpr int DW = C * E * R;
    __shared__ uint32_t lut[DW];
    __shared__ uint32_t bins[64 * 32];
    for (int e = threadIdx.x; e < DW; e += BLOCK) {
        const int t = e / (E * R), v = (e / R) % E;
        uint32_t x = 0;
        for (int j = 0; j < B; ++j)
            if (v & (1 << (B - 1 - j))) x ^= p.window[t * B + j];
        lut[e] = x;
    }
    for (int e = threadIdx.x; e < (int)p.Q * 32; e += BLOCK) bins[e] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 31;
    uint32_t lane4 = (lane & (R - 1)) * 4;
    asm volatile("" : "+v"(lane4));
    const char* lds = reinterpret_cast<const char*>(lut);
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint4 a, b, c;
    if (kPrefetch && g < ng) { a = src[3 * g]; b = src[3 * g + 1]; c = src[3 * g + 2]; }
    for (; g < ng; g += stride) {
        if (!kPrefetch) { a = src[3 * g]; b = src[3 * g + 1]; c = src[3 * g + 2]; }
        const uint32_t w0[3] = {a.x, a.y, a.z}, w1[3] = {a.w, b.x, b.y};
        const uint32_t w2[3] = {b.z, b.w, c.x}, w3[3] = {c.y, c.z, c.w};
        if (kPrefetch && g + stride < ng) {
            a = src[3 * (g + stride)]; b = src[3 * (g + stride) + 1]; c = src[3 * (g + stride) + 2];
        }
        uint4 h, q;
        h.x = hash_lut<B, R>(lds, w0, lane4);
        h.y = hash_lut<B, R>(lds, w1, lane4);
        h.z = hash_lut<B, R>(lds, w2, lane4);
        h.w = hash_lut<B, R>(lds, w3, lane4);
        q.x = __umulhi(p.q_m32 * (h.x & p.h_mask), p.Q);
        q.y = __umulhi(p.q_m32 * (h.y & p.h_mask), p.Q);
        q.z = __umulhi(p.q_m32 * (h.z & p.h_mask), p.Q);
        q.w = __umulhi(p.q_m32 * (h.w & p.h_mask), p.Q);
        if (kWrite) {
            if (kNT) {
                uint32_t* o = p.hash_out + 4 * g;
                __builtin_nontemporal_store(h.x, o); __builtin_nontemporal_store(h.y, o + 1);
                __builtin_nontemporal_store(h.z, o + 2); __builtin_nontemporal_store(h.w, o + 3);
            } else {
                reinterpret_cast<uint4*>(p.hash_out)[g] = h;
            }
            if (kQ8) {
                reinterpret_cast<uint32_t*>(p.queue_out)[g] = q.x | q.y << 8 | q.z << 16 | q.w << 24;
            } else if (kNT) {
                uint32_t* o = p.queue_out + 4 * g;
                __builtin_nontemporal_store(q.x, o); __builtin_nontemporal_store(q.y, o + 1);
                __builtin_nontemporal_store(q.z, o + 2); __builtin_nontemporal_store(q.w, o + 3);
            } else {
                reinterpret_cast<uint4*>(p.queue_out)[g] = q;
            }
        }
        atomicAdd(&bins[q.x * 32 + lane], 1u);
        atomicAdd(&bins[q.y * 32 + lane], 1u);
        atomicAdd(&bins[q.z * 32 + lane], 1u);
        atomicAdd(&bins[q.w * 32 + lane], 1u);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < p.Q; q += BLOCK) {
        uint32_t s = 0;
        for (int k = 0; k < 32; ++k) s += bins[q * 32 + ((k + q) & 31)];
        if (s) atomicAdd(&p.counts[q], (unsigned long long)s);
    }
}


// 8 consecutive tuples per lane: 96 B = 6 x dwordx4 in, 2 x dwordx4 hashes + dwordx2 u8 queues out
template <bool kWrite>
__global__ __launch_bounds__(1024) void lut12_tpl8(Params p) {
    constexpr int C = 8, E = 4096;
    __shared__ uint32_t lut[C * E];
    __shared__ uint32_t bins[64 * 32];
    for (int e = threadIdx.x; e < C * E; e += 1024) {
        const int t = e / E, v = e % E;
        uint32_t x = 0;
        for (int j = 0; j < 12; ++j)
            if (v & (1 << (11 - j))) x ^= p.window[t * 12 + j];
        lut[e] = x;
    }
    for (int e = threadIdx.x; e < (int)p.Q * 32; e += 1024) bins[e] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 31;
    uint32_t lane4 = 0;
    asm volatile("" : "+v"(lane4));
    const char* lds = reinterpret_cast<const char*>(lut);
    const uint4* src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 3;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + threadIdx.x; g < ng; g += stride) {
        uint4 v[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) v[k] = src[6 * g + k];
        const uint32_t* w = reinterpret_cast<const uint32_t*>(v);
        uint32_t h[8], q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t ww[3] = {w[3 * k], w[3 * k + 1], w[3 * k + 2]};
            h[k] = hash_lut<12, 1>(lds, ww, lane4);
            q[k] = __umulhi(p.q_m32 * (h[k] & p.h_mask), p.Q);
        }
        if (kWrite) {
            uint32_t* o = p.hash_out + 8 * g;
#pragma unroll
            for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(h[k], o + k);
            uint32_t* oq = p.queue_out + 2 * g;
            __builtin_nontemporal_store(q[0] | q[1] << 8 | q[2] << 16 | q[3] << 24, oq);
            __builtin_nontemporal_store(q[4] | q[5] << 8 | q[6] << 16 | q[7] << 24, oq + 1);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) atomicAdd(&bins[q[k] * 32 + lane], 1u);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < p.Q; q += 1024) {
        uint32_t s = 0;
        for (int k = 0; k < 32; ++k) s += bins[q * 32 + ((k + q) & 31)];
        if (s) atomicAdd(&p.counts[q], (unsigned long long)s);
    }
}

// ------------------------------------------------------------------ harness
static int g_cus = 256;

template <typename F>
static float time_ms(F launch, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// ------------------------------------------------ counts-only, no LDS tables
// For a power-of-two H <= 256 the histogram needs only hash & (H-1), i.e. <= 8 bits: each
// table term fits a byte.  Cut each input byte into 3 + 3 + 2-bit fields (36 fields); an
// 8-entry byte table is two dwords, and v_perm_b32 looks up four selector bytes in it at
// once.  A lane's four tuples are byte-transposed (8 v_perm per word) so that one selector
// dword holds the same field of all four tuples: one v_perm = one field of four tuples.
struct PermParams {
    const uint32_t* tuples;
    unsigned long long* counts;
    uint64_t n;
    uint32_t Q, q_m16;
    uint32_t lo[36], hi[36];  // field f: entries 0..3 in lo[f], 4..7 in hi[f]
};

__device__ __forceinline__ uint32_t vperm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}

__device__ __forceinline__ void transpose4(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3,
                                           uint32_t& t0, uint32_t& t1, uint32_t& t2, uint32_t& t3) {
    const uint32_t A = vperm(x1, x0, 0x05010400u), B = vperm(x1, x0, 0x07030602u);
    const uint32_t C = vperm(x3, x2, 0x05010400u), D = vperm(x3, x2, 0x07030602u);
    t0 = vperm(C, A, 0x05040100u);
    t1 = vperm(C, A, 0x07060302u);
    t2 = vperm(D, B, 0x05040100u);
    t3 = vperm(D, B, 0x07060302u);
}

// the three fields of byte-transposed dword t (byte j of word k of four tuples)
template <int kF>
__device__ __forceinline__ uint32_t perm_byte(const PermParams& p, uint32_t t, uint32_t acc) {
    const uint32_t f0 = vperm(p.hi[kF], p.lo[kF], t & 0x07070707u);
    const uint32_t f1 = vperm(p.hi[kF + 1], p.lo[kF + 1], (t >> 3) & 0x07070707u);
    const uint32_t f2 = vperm(p.lo[kF + 2], p.lo[kF + 2], (t >> 6) & 0x03030303u);
    (void)acc;
    return __builtin_amdgcn_bitop3_b32(f0, f1, f2, 0x96);
}

template <int kK>
__device__ __forceinline__ uint32_t perm_word(const PermParams& p, uint32_t x0, uint32_t x1,
                                              uint32_t x2, uint32_t x3, uint32_t acc) {
    uint32_t t0, t1, t2, t3;
    transpose4(x0, x1, x2, x3, t0, t1, t2, t3);
    const uint32_t x = perm_byte<kK * 12 + 0>(p, t0, 0), y = perm_byte<kK * 12 + 3>(p, t1, 0);
    const uint32_t z = perm_byte<kK * 12 + 6>(p, t2, 0), w = perm_byte<kK * 12 + 9>(p, t3, 0);
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(acc, x, y, 0x96), z, w, 0x96);
}

__global__ __launch_bounds__(1024) void perm_counts_kernel(const PermParams p) {
    extern __shared__ uint32_t pbins[];
    const uint32_t tid = threadIdx.x, col = tid & 31;
    for (uint32_t e = tid; e < p.Q * 32; e += 1024) pbins[e] = 0;
    __syncthreads();
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(p.tuples);
    const uint64_t ng = p.n >> 2;
    for (uint64_t g = (uint64_t)blockIdx.x * 1024 + tid; g < ng; g += (uint64_t)gridDim.x * 1024) {
        const uint4 a = src[3 * g], b = src[3 * g + 1], c = src[3 * g + 2];
        uint32_t acc = perm_word<0>(p, a.x, a.w, b.z, c.y, 0u);
        acc = perm_word<1>(p, a.y, b.x, b.w, c.z, acc);
        acc = perm_word<2>(p, a.z, b.y, c.x, c.w, acc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t bk = (acc >> (8 * i)) & 0xFFu;
            const uint32_t q = bk - __umul24(__umul24(bk, p.q_m16) >> 16, p.Q);
            __hip_atomic_fetch_add(&pbins[q * 32 + col], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    for (uint32_t q = tid; q < p.Q; q += 1024) {
        uint32_t s = 0;
        for (uint32_t c2 = 0; c2 < 32; ++c2) s += pbins[q * 32 + ((c2 + q) & 31)];
        if (s) atomicAdd(&p.counts[q], (unsigned long long)s);
    }
}

static PermParams perm_params(const rss_key& key, const uint32_t* tup, unsigned long long* counts,
                              uint64_t n, uint32_t H, uint32_t Q) {
    PermParams pp{};
    pp.tuples = tup;
    pp.counts = counts;
    pp.n = n;
    pp.Q = Q;
    pp.q_m16 = (65536u + Q - 1) / Q;
    for (int k = 0; k < 3; ++k)
        for (int j = 0; j < 4; ++j)
            for (int f = 0; f < 3; ++f) {
                const int id = (k * 4 + j) * 3 + f, s = 8 * j + 3 * f, len = f < 2 ? 3 : 2;
                uint8_t e[8] = {};
                for (int v = 0; v < (1 << len); ++v)
                    for (int bb = 0; bb < len; ++bb)
                        if ((v >> bb) & 1) e[v] ^= (uint8_t)(key.window[32 * k + 31 - (s + bb)] & (H - 1));
                pp.lo[id] = e[0] | e[1] << 8 | e[2] << 16 | (uint32_t)e[3] << 24;
                pp.hi[id] = e[4] | e[5] << 8 | e[6] << 16 | (uint32_t)e[7] << 24;
            }
    return pp;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 28);
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const uint32_t H = 128, Q = 24;
    CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint8_t key_bytes[40] = {0x23, 0x0d, 0x44, 0x3d, 0x8c, 0x2c, 0x6e, 0x64, 0xd4, 0x1a,
                                   0xf3, 0x44, 0x49, 0x9b, 0x21, 0x74, 0xfd, 0x1a, 0x9d, 0xc1,
                                   0xdd, 0x76, 0x77, 0x37, 0x38, 0x51, 0x66, 0x85, 0x7b, 0xdc,
                                   0x48, 0xa8, 0x3e, 0x55, 0x08, 0xc1, 0x63, 0xaf, 0x01, 0x9d};
    rss_key key;
    if (rss_key_prepare(key_bytes, 40, &key)) return 1;
    uint32_t *tup, *h0, *q0, *h1, *q1;
    unsigned long long *c0, *c1;
    CK(hipMalloc(&tup, n * 12));
    CK(hipMalloc(&h0, n * 4));
    CK(hipMalloc(&q0, n * 4));
    CK(hipMalloc(&h1, n * 4));
    CK(hipMalloc(&q1, n * 4));
    CK(hipMalloc(&c0, Q * 8));
    CK(hipMalloc(&c1, Q * 8));
    if (rss_generate_tuples(0x5EED, 0, n, (rss_tuple4*)tup, nullptr)) return 1;
    CK(hipDeviceSynchronize());

    auto prod = [&](bool write, uint32_t flags = 0) {
        if (rss_hash_device(&key, (rss_tuple4*)tup, n, H, Q, write ? h0 : nullptr, write ? q0 : nullptr,
                            (uint64_t*)c0, flags, nullptr)) {
            fprintf(stderr, "prod failed: %s\n", rss_last_error());
            exit(1);
        }
    };
    const double gb_r = n * 12.0 / 1e9, gb_rw = n * 20.0 / 1e9;
    float t = time_ms([&] { prod(true); }, reps);
    printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", "product full", t, n / t / 1e6, gb_rw / t * 1e3);
    t = time_ms([&] { prod(false); }, reps);
    printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", "product counts", t, n / t / 1e6, gb_r / t * 1e3);
    t = time_ms([&] { prod(true, RSS_FLAG_QUEUE_U8); }, reps);
    printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", "product full u8", t, n / t / 1e6, n * 17e-9 / t * 1e3);
    prod(true);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> rh0(n), rq0(n), rh1(n), rq1(n);
    std::vector<unsigned long long> rc0(Q), rc1(Q);
    CK(hipMemcpy(rh0.data(), h0, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rq0.data(), q0, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rc0.data(), c0, Q * 8, hipMemcpyDeviceToHost));

    Params p;
    p.tuples = tup;
    p.hash_out = h1;
    p.queue_out = q1;
    p.counts = c1;
    p.n = n;
    p.Q = Q;
    p.q_m32 = 0xFFFFFFFFu / Q + 1;
    p.h_mask = H - 1;
    memcpy(p.window, key.window, sizeof p.window);

    const char* filter = argc > 3 ? argv[3] : "";
    for (int wpc : {1, 2}) {
        if (!strstr("mem", filter)) break;
        char name[64];
        snprintf(name, sizeof name, "mem read-only grid=%dx", wpc);
        t = time_ms([&] { hipLaunchKernelGGL(mem_ceiling<false>, dim3(g_cus * wpc), dim3(1024), 0, 0, p); }, reps);
        printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", name, t, n / t / 1e6, gb_r / t * 1e3);
        snprintf(name, sizeof name, "mem read+write grid=%dx", wpc);
        t = time_ms([&] { hipLaunchKernelGGL(mem_ceiling<true>, dim3(g_cus * wpc), dim3(1024), 0, 0, p); }, reps);
        printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", name, t, n / t / 1e6, gb_rw / t * 1e3);
    }

    if (strstr("copy", filter)) {  // same-box ceilings of other mixes (1 GiB each way)
        const uint64_t n16 = n / 4;  // n * 4 bytes
        const double gb = n16 * 16e-9;
        for (int wpc : {1, 2, 4}) {
            t = time_ms([&] { hipLaunchKernelGGL(mem_copy16, dim3(g_cus * wpc), dim3(1024), 0, 0,
                                                 (const uint4*)tup, (uint4*)h1, n16); }, reps);
            printf("copy float4 1R:1W grid=%dx                %8.3f ms  %6.0f GB/s (R+W)\n", wpc, t,
                   2 * gb / t * 1e3);
            t = time_ms([&] { hipLaunchKernelGGL(mem_fill16, dim3(g_cus * wpc), dim3(1024), 0, 0,
                                                 (uint4*)h1, n16); }, reps);
            printf("fill float4 nt write-only grid=%dx        %8.3f ms  %6.0f GB/s\n", wpc, t, gb / t * 1e3);
        }
        t = time_ms([&] { CK(hipMemcpyAsync(h1, tup, n16 * 16, hipMemcpyDeviceToDevice, 0)); }, reps);
        printf("hipMemcpy DtoD 1 GiB                       %8.3f ms  %6.0f GB/s (R+W)\n", t, 2 * gb / t * 1e3);
        p.hash_out = h1;
        p.queue_out = q1;
        t = time_ms([&] { hipLaunchKernelGGL(mem_ceiling_q8, dim3(g_cus), dim3(1024), 0, 0, p); }, reps);
        printf("mem 12R+5W nt grid=1x                      %8.3f ms  %6.0f GB/s\n", t, n * 17e-9 / t * 1e3);
        t = time_ms([&] { prod(true, RSS_FLAG_QUEUE_U8); }, reps);
        printf("product full u8 (again)                    %8.3f ms  %6.0f GB/s\n", t, n * 17e-9 / t * 1e3);
    }

    if (strstr("place", filter)) {
        // physical placement: K output pairs (hash 4n B + queue n B) and two input copies
        // allocated up front; the product and the 12R+5W streams timed on each combination
        // in one process, so a placement-dependent rate shows up as a per-buffer difference
        constexpr int K = 6;
        uint32_t* hs[K];
        uint32_t* qs[K];
        for (int k = 0; k < K; ++k) {
            CK(hipMalloc(&hs[k], n * 4));
            CK(hipMalloc(&qs[k], n));
        }
        uint32_t* tup2;
        CK(hipMalloc(&tup2, n * 12));
        if (rss_generate_tuples(0x5EED, 0, n, (rss_tuple4*)tup2, nullptr)) return 1;
        CK(hipDeviceSynchronize());
        const uint32_t* ins[2] = {tup, tup2};
        for (int in = 0; in < 2; ++in)
            for (int k = 0; k < K; ++k) {
                const float tp = time_ms([&] {
                    if (rss_hash_device(&key, (const rss_tuple4*)ins[in], n, H, Q, hs[k], qs[k],
                                        (uint64_t*)c0, RSS_FLAG_QUEUE_U8, nullptr)) exit(1);
                }, reps);
                Params pp = p;
                pp.tuples = ins[in];
                pp.hash_out = hs[k];
                pp.queue_out = qs[k];
                const float ts = time_ms([&] { hipLaunchKernelGGL(mem_ceiling_q8, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
                const float tc = time_ms([&] { hipLaunchKernelGGL((mem_stream<false, true, true>), dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
                float tpol[4];
                void (*pk[4])(Params) = {mem_policy<4, false, false>, mem_policy<1, false, false>,
                                         mem_policy<2, false, false>, mem_policy<0, true, false>};
                for (int v = 0; v < 4; ++v)
                    tpol[v] = time_ms([&] { hipLaunchKernelGGL(pk[v], dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
                printf("place in=%d out=%d (in %p h %p q %p)  product %.3f  stream %.3f  chunked %.3f  "
                       "plain %.3f  sc1 %.3f  sc0sc1 %.3f  xcd %.3f ms\n",
                       in, k, (const void*)ins[in], (void*)hs[k], (void*)qs[k], tp, ts, tc, tpol[0],
                       tpol[1], tpol[2], tpol[3]);
            }
        // each buffer on its own: write-only fill and read-only sweep of hash buffer k, and
        // the product with hash and queue buffers taken from different pairs
        for (int k = 0; k < K; ++k) {
            const uint64_t n16 = n / 4;
            const float tf = time_ms([&] { hipLaunchKernelGGL(mem_fill16, dim3(g_cus), dim3(1024), 0, 0, (uint4*)hs[k], n16); }, reps);
            Params pr = p;
            pr.tuples = hs[k];
            pr.n = n / 3 * 1;  // n/3 tuples of 12 B = 4n B = the hash buffer
            const float tr = time_ms([&] { hipLaunchKernelGGL(mem_ceiling<false>, dim3(g_cus), dim3(1024), 0, 0, pr); }, reps);
            printf("buffer h%d  fill %.3f ms (%.0f GB/s)  read %.3f ms (%.0f GB/s)\n", k, tf,
                   n16 * 16e-9 / tf * 1e3, tr, (n / 3) * 12e-9 / tr * 1e3);
        }
        for (int kh = 0; kh < K; kh += K - 1)
            for (int kq = 0; kq < K; kq += K - 1) {
                const float tp = time_ms([&] {
                    if (rss_hash_device(&key, (const rss_tuple4*)tup, n, H, Q, hs[kh], qs[kq],
                                        (uint64_t*)c0, RSS_FLAG_QUEUE_U8, nullptr)) exit(1);
                }, reps);
                const float th = time_ms([&] {
                    if (rss_hash_device(&key, (const rss_tuple4*)tup, n, H, Q, hs[kh], nullptr,
                                        (uint64_t*)c0, 0, nullptr)) exit(1);
                }, reps);
                printf("mix h%d q%d  product %.3f ms   hash-only product %.3f ms\n", kh, kq, tp, th);
            }
        for (int k = 0; k < K; ++k) {
            CK(hipFree(hs[k]));
            CK(hipFree(qs[k]));
        }
        CK(hipFree(tup2));
    }

    if (strstr("contig", filter)) {
        // allocation kind vs the 12R+5W rate: K output pairs and one input from plain hipMalloc,
        // the same from hipExtMallocWithFlags(hipDeviceMallocContiguous), and K output pairs carved
        // at 1 GiB steps from one large hipMalloc pool; product + stream per combination
        constexpr int K = 4;
        uint32_t *hp[K], *qp[K], *hc[K] = {}, *qc[K] = {};
        for (int k = 0; k < K; ++k) {
            CK(hipMalloc(&hp[k], n * 4));
            CK(hipMalloc(&qp[k], n));
        }
        uint32_t* tc = nullptr;
        if (hipExtMallocWithFlags((void**)&tc, n * 12, hipDeviceMallocContiguous) != hipSuccess) {
            printf("contiguous input allocation refused\n");
            tc = nullptr;
            (void)hipGetLastError();
        }
        for (int k = 0; k < K; ++k) {
            if (hipExtMallocWithFlags((void**)&hc[k], n * 4, hipDeviceMallocContiguous) != hipSuccess ||
                hipExtMallocWithFlags((void**)&qc[k], n, hipDeviceMallocContiguous) != hipSuccess) {
                printf("contiguous output allocation %d refused\n", k);
                (void)hipGetLastError();
                hc[k] = qc[k] = nullptr;
            }
        }
        const size_t pool_stride = size_t(1) << 30, pair = n * 5;
        uint8_t* pool = nullptr;
        CK(hipMalloc(&pool, pool_stride * (K - 1) + pair));
        if (tc) {
            CK(hipMemcpy(tc, tup, n * 12, hipMemcpyDeviceToDevice));
        }
        CK(hipDeviceSynchronize());
        auto both = [&](const char* what, const uint32_t* in, uint32_t* h, uint32_t* q) {
            if (!in || !h || !q) return;
            const float tp = time_ms([&] {
                if (rss_hash_device(&key, (const rss_tuple4*)in, n, H, Q, h, q, (uint64_t*)c0,
                                    RSS_FLAG_QUEUE_U8, nullptr)) exit(1);
            }, reps);
            Params pp = p;
            pp.tuples = in;
            pp.hash_out = h;
            pp.queue_out = q;
            const float ts = time_ms([&] { hipLaunchKernelGGL(mem_ceiling_q8, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
            printf("contig %-28s (in %p h %p q %p)  product %.3f  stream %.3f ms\n", what,
                   (const void*)in, (void*)h, (void*)q, tp, ts);
        };
        char name[64];
        for (int round = 0; round < 2; ++round)
            for (int k = 0; k < K; ++k) {
                snprintf(name, sizeof name, "in=malloc out=malloc%d", k);
                both(name, tup, hp[k], qp[k]);
                snprintf(name, sizeof name, "in=malloc out=contig%d", k);
                both(name, tup, hc[k], qc[k]);
                snprintf(name, sizeof name, "in=contig out=malloc%d", k);
                both(name, tc, hp[k], qp[k]);
                snprintf(name, sizeof name, "in=contig out=contig%d", k);
                both(name, tc, hc[k], qc[k]);
                snprintf(name, sizeof name, "in=malloc out=pool+%dGiB", k);
                both(name, tup, (uint32_t*)(pool + k * pool_stride), (uint32_t*)(pool + k * pool_stride + n * 4));
            }
        for (int k = 0; k < K; ++k) {
            CK(hipFree(hp[k]));
            CK(hipFree(qp[k]));
            if (hc[k]) CK(hipFree(hc[k]));
            if (qc[k]) CK(hipFree(qc[k]));
        }
        if (tc) CK(hipFree(tc));
        CK(hipFree(pool));
    }

    if (strstr("ipv6mem", filter)) {
        // the IPv6 kernel (rss_hash6_device, u8 queues) against its 36 R + 5 W stream, same
        // buffers: n/3 tuples of 36 B fill the 12n-byte tuple buffer
        const uint64_t n6 = n / 3;
        rss_key6 k6;
        if (rss_key6_prepare(key_bytes, 40, &k6)) exit(1);
        Params pp = p;
        pp.n = n6;
        pp.hash_out = h1;
        pp.queue_out = q1;
        for (int round = 0; round < 3; ++round) {
            const float tk = time_ms([&] {
                if (rss_hash6_device(&k6, (const rss_tuple6*)tup, n6, H, Q, h1, q1, (uint64_t*)c1,
                                     RSS_FLAG_QUEUE_U8, nullptr)) exit(1);
            }, reps);
            const float tc = time_ms([&] {
                if (rss_hash6_device(&k6, (const rss_tuple6*)tup, n6, H, Q, nullptr, nullptr, (uint64_t*)c1,
                                     0, nullptr)) exit(1);
            }, reps);
            const float ts = time_ms([&] { hipLaunchKernelGGL(mem_ceiling6_q8, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
            const float tr = time_ms([&] { hipLaunchKernelGGL(mem_ceiling<false>, dim3(g_cus), dim3(1024), 0, 0, p); }, reps);
            printf("ipv6mem  ipv6 full u8 %.3f ms (%.0f GB/s)  ipv6 counts %.3f ms (%.0f GB/s read)  "
                   "stream 36R+5W %.3f ms (%.0f GB/s)  read-only 12n %.3f ms (%.0f GB/s)\n",
                   tk, n6 * 41e-9 / tk * 1e3, tc, n6 * 36e-9 / tc * 1e3, ts, n6 * 41e-9 / ts * 1e3,
                   tr, n * 12e-9 / tr * 1e3);
        }
    }

    if (strstr("ipv6shape", filter)) {
        // IPv6's load shape: the product's lane-owned 144 B (9 x 16-B loads at a 144-B stride)
        // against lane-contiguous 1 KiB wave loads, 36 R + 5 W and read-only, same buffers
        Params pp = p;
        pp.n = (n / 3) & ~255ull;
        pp.hash_out = h1;
        pp.queue_out = q1;
        const double gbw = pp.n * 41e-9, gbr = pp.n * 36e-9;
        for (int round = 0; round < 3; ++round) {
            const float s0 = time_ms([&] { hipLaunchKernelGGL(mem_ceiling6_q8, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
            const float s1 = time_ms([&] { hipLaunchKernelGGL(mem_ceiling6_contig<false>, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
            const float r0 = time_ms([&] { hipLaunchKernelGGL(mem_ceiling6_read, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
            const float r1 = time_ms([&] { hipLaunchKernelGGL(mem_ceiling6_contig<true>, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
            printf("ipv6shape  36R+5W strided %.3f ms (%.0f GB/s)  contiguous %.3f ms (%.0f GB/s)  "
                   "36R strided %.3f ms (%.0f GB/s)  contiguous %.3f ms (%.0f GB/s)\n",
                   s0, gbw / s0 * 1e3, s1, gbw / s1 * 1e3, r0, gbr / r0 * 1e3, r1, gbr / r1 * 1e3);
        }
    }

    if (strstr("shapeplace", filter)) {
        // the load shape on placements of every tier: product access (lane-owned 48 B) vs
        // lane-contiguous 1 KiB wave loads, 12R+5W without compute, per output pair
        constexpr int K = 6;
        uint32_t *hs[K], *qs[K];
        for (int k = 0; k < K; ++k) {
            CK(hipMalloc(&hs[k], n * 4));
            CK(hipMalloc(&qs[k], n));
        }
        for (int round = 0; round < 2; ++round)
            for (int k = 0; k < K; ++k) {
                Params pp = p;
                pp.hash_out = hs[k];
                pp.queue_out = qs[k];
                const float tp = time_ms([&] {
                    if (rss_hash_device(&key, (const rss_tuple4*)tup, n, H, Q, hs[k], qs[k], (uint64_t*)c0,
                                        RSS_FLAG_QUEUE_U8, nullptr)) exit(1);
                }, reps);
                const float s0 = time_ms([&] { hipLaunchKernelGGL(mem_shape<0>, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
                const float s1 = time_ms([&] { hipLaunchKernelGGL(mem_shape<1>, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
                const float s1x2 = time_ms([&] { hipLaunchKernelGGL(mem_shape<1>, dim3(2 * g_cus), dim3(1024), 0, 0, pp); }, reps);
                const float s0x2 = time_ms([&] { hipLaunchKernelGGL(mem_shape<0>, dim3(2 * g_cus), dim3(1024), 0, 0, pp); }, reps);
                const float s3 = time_ms([&] { hipLaunchKernelGGL(mem_shape<3>, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
                const float s3x2 = time_ms([&] { hipLaunchKernelGGL(mem_shape<3>, dim3(2 * g_cus), dim3(1024), 0, 0, pp); }, reps);
                const float s4 = time_ms([&] { hipLaunchKernelGGL(mem_shape<4>, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
                const float s4x2 = time_ms([&] { hipLaunchKernelGGL(mem_shape<4>, dim3(2 * g_cus), dim3(1024), 0, 0, pp); }, reps);
                const float t9x2 = time_ms([&] {
                    CK(hipMemsetAsync(c1, 0, Q * 8, 0));
                    hipLaunchKernelGGL(lut9_kernel<true>, dim3(2 * g_cus), dim3(1024), 0, 0, pp);
                }, reps);
                printf("shapeplace pair %d  T9 x2 (60 KiB LUT, 2 WGs/CU) %.3f ms\n", k, t9x2);
                printf("shapeplace pair %d  product %.3f  shape0 %.3f  shape0x2 %.3f  shape1 %.3f  shape1x2 %.3f  "
                       "shape3 %.3f  shape3x2 %.3f  shape4 %.3f  shape4x2 %.3f ms\n",
                       k, tp, s0, s0x2, s1, s1x2, s3, s3x2, s4, s4x2);
            }
        for (int k = 0; k < K; ++k) {
            CK(hipFree(hs[k]));
            CK(hipFree(qs[k]));
        }
    }

    if (strstr("pads", filter)) {
        // allocation size vs tier: K output pairs for each padding of the hash and queue
        // allocations (0, 2 MiB, 64 MiB, 256 MiB extra), kinds allocated round-robin
        constexpr int K = 5, P = 4;
        const size_t pads[P] = {0, size_t(2) << 20, size_t(64) << 20, size_t(256) << 20};
        uint32_t *hs[P][K], *qs[P][K];
        for (int k = 0; k < K; ++k)
            for (int pi = 0; pi < P; ++pi) {
                CK(hipMalloc(&hs[pi][k], n * 4 + pads[pi]));
                CK(hipMalloc(&qs[pi][k], n + pads[pi]));
            }
        for (int pi = 0; pi < P; ++pi)
            for (int k = 0; k < K; ++k) {
                const float tp = time_ms([&] {
                    if (rss_hash_device(&key, (const rss_tuple4*)tup, n, H, Q, hs[pi][k], qs[pi][k],
                                        (uint64_t*)c0, RSS_FLAG_QUEUE_U8, nullptr)) exit(1);
                }, reps);
                printf("pads pad=%zuMiB pair %d  product %.3f ms\n", pads[pi] >> 20, k, tp);
            }
        for (int k = 0; k < K; ++k)
            for (int pi = 0; pi < P; ++pi) {
                CK(hipFree(hs[pi][k]));
                CK(hipFree(qs[pi][k]));
            }
    }

    if (strstr("parts", filter)) {
        // is a placement tier a property of a whole allocation or of its sub-ranges?  For K
        // output pairs: the product over all n tuples, then over each quarter of the tuples
        // (writing the matching quarter of the hash / queue buffers), per-launch times
        // scaled x4 for comparison
        constexpr int K = 6;
        uint32_t *hs[K], *qs[K];
        for (int k = 0; k < K; ++k) {
            CK(hipMalloc(&hs[k], n * 4));
            CK(hipMalloc(&qs[k], n));
        }
        const uint64_t m = n / 4;
        for (int k = 0; k < K; ++k) {
            const float tf = time_ms([&] {
                if (rss_hash_device(&key, (const rss_tuple4*)tup, n, H, Q, hs[k], qs[k], (uint64_t*)c0,
                                    RSS_FLAG_QUEUE_U8, nullptr)) exit(1);
            }, reps);
            float tq[4];
            for (int part = 0; part < 4; ++part)
                tq[part] = 4 * time_ms([&] {
                    if (rss_hash_device(&key, (const rss_tuple4*)tup + part * m, m, H, Q, hs[k] + part * m,
                                        (uint8_t*)qs[k] + part * m, (uint64_t*)c0, RSS_FLAG_QUEUE_U8,
                                        nullptr)) exit(1);
                }, 4 * reps);
            printf("parts pair %d  whole %.3f  quarters x4 %.3f %.3f %.3f %.3f ms\n", k, tf, tq[0], tq[1],
                   tq[2], tq[3]);
        }
        for (int k = 0; k < K; ++k) {
            CK(hipFree(hs[k]));
            CK(hipFree(qs[k]));
        }
    }

    if (strstr("qsize", filter)) {
        // does the queue allocation's size (n B, as u8 queues need, vs 4n B, as the bench
        // allocates for its u32 line) change how often a placement lands in the fast tier?
        // K pairs of each kind, allocated alternately, all against the same input
        constexpr int K = 6;
        uint32_t *hs[2][K], *qs[2][K];
        for (int k = 0; k < K; ++k)
            for (int kind = 0; kind < 2; ++kind) {
                CK(hipMalloc(&hs[kind][k], n * 4));
                CK(hipMalloc(&qs[kind][k], kind == 0 ? n : 4 * n));
            }
        for (int round = 0; round < 2; ++round)
            for (int kind = 0; kind < 2; ++kind)
                for (int k = 0; k < K; ++k) {
                    const float tp = time_ms([&] {
                        if (rss_hash_device(&key, (const rss_tuple4*)tup, n, H, Q, hs[kind][k], qs[kind][k],
                                            (uint64_t*)c0, RSS_FLAG_QUEUE_U8, nullptr)) exit(1);
                    }, reps);
                    printf("qsize %s pair %d (h %p q %p)  product %.3f ms\n", kind == 0 ? "q=n " : "q=4n", k,
                           (void*)hs[kind][k], (void*)qs[kind][k], tp);
                }
        for (int k = 0; k < K; ++k)
            for (int kind = 0; kind < 2; ++kind) {
                CK(hipFree(hs[kind][k]));
                CK(hipFree(qs[kind][k]));
            }
    }

    if (strstr("perm", filter)) {
        const PermParams pp = perm_params(key, tup, c1, n, H, Q);
        for (int wpc : {1, 2}) {
            CK(hipMemset(c1, 0, Q * 8));
            hipLaunchKernelGGL(perm_counts_kernel, dim3(g_cus * wpc), dim3(1024), Q * 32 * 4, 0, pp);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(rc1.data(), c1, Q * 8, hipMemcpyDeviceToHost));
            printf("perm counts grid=%dx check: %s\n", wpc, rc1 == rc0 ? "OK" : "MISMATCH");
        }
        for (int round = 0; round < 3; ++round) {
            t = time_ms([&] { prod(false); }, reps);
            printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", "product counts", t, n / t / 1e6, gb_r / t * 1e3);
            for (int wpc : {1, 2}) {
                t = time_ms([&] {
                    CK(hipMemsetAsync(c1, 0, Q * 8, 0));
                    hipLaunchKernelGGL(perm_counts_kernel, dim3(g_cus * wpc), dim3(1024), Q * 32 * 4, 0, pp);
                }, reps);
                printf("perm counts grid=%dx                      %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", wpc, t,
                       n / t / 1e6, gb_r / t * 1e3);
            }
            t = time_ms([&] { hipLaunchKernelGGL(mem_ceiling<false>, dim3(g_cus), dim3(1024), 0, 0, p); }, reps);
            printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", "mem read-only grid=1x", t, n / t / 1e6, gb_r / t * 1e3);
        }
    }

    if (strstr("offsets", filter)) {
        // relative placement inside ONE allocation (physically contiguous when the driver
        // grants hipDeviceMallocContiguous, else plain hipMalloc): tuples at 0, hashes at
        // 12n + a, queues at 16n + a + b; scan a (b = 0) then b (a = 0) in 32 MiB steps
        const size_t MiB = size_t(1) << 20, span = 1024 * MiB;
        const size_t bytes = n * 17 + 2 * span + 64 * MiB;
        for (int kind = 0; kind < 2; ++kind) {
            uint8_t* pool = nullptr;
            if (kind == 0) {
                if (hipExtMallocWithFlags((void**)&pool, bytes, hipDeviceMallocContiguous) != hipSuccess) {
                    (void)hipGetLastError();
                    printf("offsets: contiguous pool refused\n");
                    continue;
                }
            } else {
                CK(hipMalloc(&pool, bytes));
            }
            CK(hipMemcpy(pool, tup, n * 12, hipMemcpyDeviceToDevice));
            CK(hipDeviceSynchronize());
            for (int scan = 0; scan < 2; ++scan)
                for (size_t off = 0; off <= span; off += 32 * MiB) {
                    const size_t a = scan == 0 ? off : 0, b = scan == 0 ? 0 : off;
                    Params pp = p;
                    pp.tuples = (const uint32_t*)pool;
                    pp.hash_out = (uint32_t*)(pool + n * 12 + a);
                    pp.queue_out = (uint32_t*)(pool + n * 16 + a + b);
                    const float ts = time_ms([&] { hipLaunchKernelGGL(mem_ceiling_q8, dim3(g_cus), dim3(1024), 0, 0, pp); }, reps);
                    const float tp = time_ms([&] {
                        if (rss_hash_device(&key, (const rss_tuple4*)pp.tuples, n, H, Q, pp.hash_out,
                                            pp.queue_out, (uint64_t*)c0, RSS_FLAG_QUEUE_U8, nullptr)) exit(1);
                    }, reps);
                    printf("offsets %s pool %p  hash +%4zu MiB  queue +%4zu MiB  stream %.3f  product %.3f ms\n",
                           kind == 0 ? "contig" : "malloc", (void*)pool, a / MiB, b / MiB, ts, tp);
                }
            CK(hipFree(pool));
        }
    }

    if (strstr("shape", filter)) {
        p.hash_out = h1;
        p.queue_out = q1;
        struct SV { const char* name; void (*k)(Params); int wpc; };
        const SV vs[] = {{"shape 0 product access   grid=1x", mem_shape<0>, 1},
                         {"shape 1 contiguous loads grid=1x", mem_shape<1>, 1},
                         {"shape 2 16-B queue store grid=1x", mem_shape<2>, 1},
                         {"shape 0 product access   grid=2x", mem_shape<0>, 2},
                         {"shape 1 contiguous loads grid=2x", mem_shape<1>, 2},
                         {"shape 2 16-B queue store grid=2x", mem_shape<2>, 2}};
        for (int round = 0; round < 2; ++round)
            for (const SV& v : vs) {
                t = time_ms([&] { hipLaunchKernelGGL(v.k, dim3(g_cus * v.wpc), dim3(1024), 0, 0, p); }, reps);
                printf("%-40s %8.3f ms  %6.0f GB/s\n", v.name, t, n * 17e-9 / t * 1e3);
            }
        t = time_ms([&] { prod(true, RSS_FLAG_QUEUE_U8); }, reps);
        printf("product full u8 (again)                    %8.3f ms  %6.0f GB/s\n", t, n * 17e-9 / t * 1e3);
    }

    if (strstr("memq8", filter)) {
        p.hash_out = h1;
        p.queue_out = q1;
        for (int wpc : {1, 2}) {
            t = time_ms([&] { hipLaunchKernelGGL(mem_ceiling_q8, dim3(g_cus * wpc), dim3(1024), 0, 0, p); }, reps);
            printf("mem 12R+5W nt grid=%dx                   %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", wpc, t,
                   n / t / 1e6, n * 17e-9 / t * 1e3);
        }
    }
    if (strstr("memprobe", filter)) {
        p.hash_out = h1;
        p.queue_out = q1;
        const char* names[3] = {"mem 12R+5W plain stores", "mem 12R+4W (hash only, nt)",
                                "mem 12R+5W nt, queue via LDS x4"};
        void (*ks[3])(Params) = {mem_probe<0>, mem_probe<1>, mem_probe<2>};
        const double bytes[3] = {17e-9, 16e-9, 17e-9};
        for (int m = 0; m < 3; ++m) {
            t = time_ms([&] { hipLaunchKernelGGL(ks[m], dim3(g_cus), dim3(1024), 0, 0, p); }, reps);
            printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", names[m], t, n / t / 1e6, n * bytes[m] / t * 1e3);
        }
        t = time_ms([&] { hipLaunchKernelGGL(mem_ceiling_q8, dim3(g_cus), dim3(1024), 0, 0, p); }, reps);
        printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", "mem 12R+5W nt (as product)", t, n / t / 1e6, n * 17e-9 / t * 1e3);
        t = time_ms([&] { hipLaunchKernelGGL(mem_ceiling<false>, dim3(g_cus), dim3(1024), 0, 0, p); }, reps);
        printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", "mem 12R", t, n / t / 1e6, n * 12e-9 / t * 1e3);
    }
    if (strstr("stream", filter)) {
        p.hash_out = h1;
        p.queue_out = q1;
        struct SV { const char* name; void (*k)(Params); double bytes; };
        const SV sv[8] = {
            {"stream 12R plain grid-stride", mem_stream<false, false, false>, 12e-9},
            {"stream 12R nt grid-stride", mem_stream<true, false, false>, 12e-9},
            {"stream 12R plain chunked", mem_stream<false, true, false>, 12e-9},
            {"stream 12R nt chunked", mem_stream<true, true, false>, 12e-9},
            {"stream 12R+5W plain-ld grid-stride", mem_stream<false, false, true>, 17e-9},
            {"stream 12R+5W nt-ld grid-stride", mem_stream<true, false, true>, 17e-9},
            {"stream 12R+5W plain-ld chunked", mem_stream<false, true, true>, 17e-9},
            {"stream 12R+5W nt-ld chunked", mem_stream<true, true, true>, 17e-9}};
        for (int wpc : {1, 2}) {
            for (const SV& v : sv) {
                t = time_ms([&] { hipLaunchKernelGGL(v.k, dim3(g_cus * wpc), dim3(1024), 0, 0, p); }, reps);
                printf("%-36s x%d %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", v.name, wpc, t, n / t / 1e6,
                       n * v.bytes / t * 1e3);
            }
        }
    }
    if (strstr("policy", filter)) {  // store cache policy / XCD mapping / unroll, 12R+5W
        p.hash_out = h1;
        p.queue_out = q1;
        struct PV { const char* name; void (*k)(Params); int wpc; };
        const PV pv[9] = {{"policy nt stores (as product)", mem_policy<0, false, false>, 1},
                          {"policy sc1 stores", mem_policy<1, false, false>, 1},
                          {"policy sc0 sc1 stores", mem_policy<2, false, false>, 1},
                          {"policy sc0 sc1 nt stores", mem_policy<3, false, false>, 1},
                          {"policy plain stores", mem_policy<4, false, false>, 1},
                          {"policy nt, XCD-contiguous eighths", mem_policy<0, true, false>, 1},
                          {"policy nt, 2 iterations of loads first", mem_policy<0, false, true>, 1},
                          {"policy nt, XCD-contiguous, grid 2x", mem_policy<0, true, false>, 2},
                          {"policy nt (as product) again", mem_policy<0, false, false>, 1}};
        for (const PV& v : pv) {
            t = time_ms([&] { hipLaunchKernelGGL(v.k, dim3(g_cus * v.wpc), dim3(1024), 0, 0, p); }, reps);
            printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", v.name, t, n / t / 1e6, n * 17e-9 / t * 1e3);
        }
    }
    if (strstr("dyn", filter)) {  // static grid-stride vs per-wave dynamic chunks
        p.hash_out = h1;
        p.queue_out = q1;
        unsigned* heads;
        CK(hipMalloc(&heads, 8 * sizeof(unsigned)));
        struct SV { const char* name; void (*k)(Params); double bytes; };
        const SV ref[2] = {{"dyn-ref 12R+5W static grid-stride", mem_stream<false, false, true>, 17e-9},
                           {"dyn-ref 12R static grid-stride", mem_stream<false, false, false>, 12e-9}};
        struct DV { const char* name; void (*k)(Params, unsigned*); double bytes; };
        const DV dv[6] = {{"dyn 12R+5W chunk 16 iters", mem_dyn<16, true>, 17e-9},
                          {"dyn 12R+5W chunk 64 iters", mem_dyn<64, true>, 17e-9},
                          {"dyn 12R+5W chunk 256 iters", mem_dyn<256, true>, 17e-9},
                          {"dyn 12R chunk 16 iters", mem_dyn<16, false>, 12e-9},
                          {"dyn 12R chunk 64 iters", mem_dyn<64, false>, 12e-9},
                          {"dyn 12R chunk 256 iters", mem_dyn<256, false>, 12e-9}};
        for (int rep = 0; rep < 2; ++rep) {
            for (const SV& v : ref) {
                t = time_ms([&] { hipLaunchKernelGGL(v.k, dim3(g_cus), dim3(1024), 0, 0, p); }, reps);
                printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", v.name, t, n / t / 1e6, n * v.bytes / t * 1e3);
            }
            for (const DV& v : dv) {
                t = time_ms([&] {
                    CK(hipMemsetAsync(heads, 0, 8 * sizeof(unsigned), 0));
                    hipLaunchKernelGGL(v.k, dim3(g_cus), dim3(1024), 0, 0, p, heads);
                }, reps);
                printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s\n", v.name, t, n / t / 1e6, n * v.bytes / t * 1e3);
            }
        }
        // the dynamic stream must cover every group exactly once: check its hash output
        CK(hipMemset(h1, 0xFF, n * 4));
        CK(hipMemsetAsync(heads, 0, 8 * sizeof(unsigned), 0));
        hipLaunchKernelGGL((mem_dyn<64, true>), dim3(g_cus), dim3(1024), 0, 0, p, heads);
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> th(n), tt(3 * n);
        CK(hipMemcpy(th.data(), h1, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(tt.data(), tup, n * 12, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < n; ++i) bad += th[i] != (tt[3 * i] ^ tt[3 * i + 1] ^ tt[3 * i + 2]);
        printf("dyn coverage check: %llu mismatches\n", (unsigned long long)bad);
        CK(hipFree(heads));
    }
    auto run_variant = [&](const char* name, void (*k)(Params), int block, int wgs_per_cu, bool write,
                           bool q8 = false) {
        if (!strstr(name, filter)) return;
        auto launch = [&] {
            CK(hipMemsetAsync(c1, 0, Q * 8, 0));
            hipLaunchKernelGGL(k, dim3(g_cus * wgs_per_cu), dim3(block), 0, 0, p);
        };
        p.hash_out = write ? h1 : nullptr;
        p.queue_out = write ? q1 : nullptr;
        CK(hipMemset(h1, 0, n * 4));
        launch();
        CK(hipDeviceSynchronize());
        CK(hipGetLastError());
        bool ok = true;
        CK(hipMemcpy(rc1.data(), c1, Q * 8, hipMemcpyDeviceToHost));
        ok = ok && rc1 == rc0;
        if (write) {
            CK(hipMemcpy(rh1.data(), h1, n * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(rq1.data(), q1, n * 4, hipMemcpyDeviceToHost));
            ok = ok && rh1 == rh0;
            if (q8) {
                const uint8_t* b = reinterpret_cast<const uint8_t*>(rq1.data());
                for (uint64_t i = 0; i < n && ok; ++i) ok = b[i] == rq0[i];
            } else {
                ok = ok && rq1 == rq0;
            }
        }
        const float tt = time_ms(launch, reps);
        printf("%-40s %8.3f ms  %7.1f Gt/s  %6.0f GB/s  %s\n", name, tt, n / tt / 1e6,
               (write ? gb_rw : gb_r) / tt * 1e3, ok ? "OK" : "MISMATCH");
    };
#define V(B, R, BL, WPC, PF)                                                                   \
    run_variant("B" #B " R" #R " blk" #BL " x" #WPC " pf" #PF " full", lut_kernel<B, R, BL, true, PF>, BL, WPC, true); \
    run_variant("B" #B " R" #R " blk" #BL " x" #WPC " pf" #PF " counts", lut_kernel<B, R, BL, false, PF>, BL, WPC, false);
    V(4, 32, 1024, 2, false)
    V(6, 32, 1024, 1, false)
    V(8, 1, 1024, 2, false)
    V(8, 2, 1024, 2, false)
    V(8, 8, 1024, 1, false)
    V(12, 1, 1024, 1, false)
    V(8, 1, 512, 4, false)
    V(8, 1, 256, 8, false)
    run_variant("B12 tpl8 q8nt full", lut12_tpl8<true>, 1024, 1, true, true);
    run_variant("B12 R1 blk1024 x1 pf q8nt full", lut_kernel<12, 1, 1024, true, true, true, true>, 1024, 1, true, true);
    run_variant("B12 tpl8 counts", lut12_tpl8<false>, 1024, 1, false);
    run_variant("B12 R1 blk1024 x1 q8nt full", lut_kernel<12, 1, 1024, true, false, true, true>, 1024, 1, true, true);
    run_variant("B8 R1 blk1024 x2 q8 full", lut_kernel<8, 1, 1024, true, false, true>, 1024, 2, true, true);
    run_variant("B8 R1 blk1024 x2 nt full", lut_kernel<8, 1, 1024, true, false, false, true>, 1024, 2, true);
    run_variant("B8 R1 blk1024 x2 q8nt full", lut_kernel<8, 1, 1024, true, false, true, true>, 1024, 2, true, true);
    run_variant("T9 x2 q8nt full", lut9_kernel<true>, 1024, 2, true, true);
    run_variant("T9 x2 counts", lut9_kernel<false>, 1024, 2, false);
    run_variant("T9 x1 q8nt full", lut9_kernel<true>, 1024, 1, true, true);
    run_variant("T9ref B12 R1 blk1024 x1 q8nt full", lut_kernel<12, 1, 1024, true, false, true, true>, 1024, 1, true, true);
    return 0;
}

/*
 * toeplitz_oracle.c -- CPU restatement of the reference's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker; the product
 * (rss_simulator_nvidia_amd/) never links or calls it.
 *
 * Parity pinned: tests/test_oracle.py checks every function here against the
 * golden fixtures generated from the reference itself (tests/golden/make_golden.py):
 * the README example (F1), the Microsoft RSS KAT (F2), 4096 random tuples x 4 keys
 * (F3), one-hot / all-zero / all-ones inputs (F4) and the queue/count sweeps (F5).
 *
 * Algorithm, restated from noamsto/rss_simulator_nvidia v0.0.2:
 *   - window after i key rotations (toeplitz.py:71-81 __key_left_most_32bits,
 *     toeplitz.py:83-98 __shift_key): the key is rotated left one bit per input
 *     bit, so the window XORed for input bit i is key bits [i, i+32) (no wrap:
 *     i + 31 <= 126 < 320);
 *   - hash (toeplitz.py:46-69): for each of the 96 input bits, MSB first, over
 *     src_ip, dst_ip, src_port, dst_port big-endian (toeplitz.py:113-142),
 *     XOR in the current window when the bit is 1;
 *   - queue (simulator.py:94-98): hash % htable % nqueues;
 *   - counts (simulator.py:107-113): value_counts of the queue column.
 * The rotation is simulated literally (a 416-bit key register shifted left one
 * bit per input bit), not via the closed form, so the restatement stays a
 * line-by-line analogue of the reference loop.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_KEY_MAX 256

/* leftmost 32 bits of a byte-array key (toeplitz.py:81) */
static uint32_t key_left_most_32bits(const uint8_t* key) {
    return (uint32_t)key[0] << 24 | (uint32_t)key[1] << 16 | (uint32_t)key[2] << 8 | key[3];
}

/* rotate the whole key left by one bit (toeplitz.py:83-98) */
static void shift_key(uint8_t* key, size_t len) {
    const uint8_t msb = key[0] >> 7;
    for (size_t i = 0; i + 1 < len; ++i) key[i] = (uint8_t)(key[i] << 1 | key[i + 1] >> 7);
    key[len - 1] = (uint8_t)(key[len - 1] << 1 | msb);
}

/* The 96 windows the reference XORs: window[i] = leftmost 32 bits after i shifts. */
int oracle_windows(const uint8_t* key, size_t len, uint32_t* window96) {
    if (len < 4 || len > ORACLE_KEY_MAX) return -22;
    uint8_t k[ORACLE_KEY_MAX];
    memcpy(k, key, len);
    for (int i = 0; i < 96; ++i) {
        window96[i] = key_left_most_32bits(k);
        shift_key(k, len);
    }
    return 0;
}

/* The first nbits windows (any input length, e.g. 288 for IPv6). */
int oracle_windows_n(const uint8_t* key, size_t len, int nbits, uint32_t* window) {
    if (len < 4 || len > ORACLE_KEY_MAX || nbits < 0) return -22;
    uint8_t k[ORACLE_KEY_MAX];
    memcpy(k, key, len);
    for (int i = 0; i < nbits; ++i) {
        window[i] = key_left_most_32bits(k);
        shift_key(k, len);
    }
    return 0;
}

/* 12 big-endian input bytes (toeplitz.py:127-142); ports masked to 16 bits. */
static void prepare_input_bytes(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport,
                                uint8_t* b) {
    b[0] = (uint8_t)(sip >> 24); b[1] = (uint8_t)(sip >> 16); b[2] = (uint8_t)(sip >> 8); b[3] = (uint8_t)sip;
    b[4] = (uint8_t)(dip >> 24); b[5] = (uint8_t)(dip >> 16); b[6] = (uint8_t)(dip >> 8); b[7] = (uint8_t)dip;
    b[8] = (uint8_t)((sport & 0xFF00) >> 8); b[9] = (uint8_t)(sport & 0xFF);
    b[10] = (uint8_t)((dport & 0xFF00) >> 8); b[11] = (uint8_t)(dport & 0xFF);
}

/* compute_hash with the literal rotating key (toeplitz.py:46-69). */
uint32_t oracle_hash_rotating(const uint8_t* key, size_t len, uint32_t sip, uint32_t dip,
                              uint32_t sport, uint32_t dport) {
    uint8_t k[ORACLE_KEY_MAX];
    if (len < 4 || len > ORACLE_KEY_MAX) return 0;
    uint8_t in[12];
    memcpy(k, key, len);
    prepare_input_bytes(sip, dip, sport, dport, in);
    uint32_t result = 0;
    for (int byte = 0; byte < 12; ++byte)
        for (int bit = 7; bit >= 0; --bit) {
            if ((in[byte] >> bit) & 1) result ^= key_left_most_32bits(k);
            shift_key(k, len);
        }
    return result;
}

/*
 * The same literal loop over an arbitrary byte string (field selection and IPv6
 * inputs: the reference's algorithm applied to other inputs; pinned by the
 * Microsoft RSS verification suite's "IPv4 only" and IPv6 vectors).
 */
uint32_t oracle_hash_bytes(const uint8_t* key, size_t len, const uint8_t* data, size_t nbytes) {
    uint8_t k[ORACLE_KEY_MAX];
    if (len < 4 || len > ORACLE_KEY_MAX) return 0;
    memcpy(k, key, len);
    uint32_t result = 0;
    for (size_t byte = 0; byte < nbytes; ++byte)
        for (int bit = 7; bit >= 0; --bit) {
            if ((data[byte] >> bit) & 1) result ^= key_left_most_32bits(k);
            shift_key(k, len);
        }
    return result;
}

/* Same loop with the rotations precomputed as the 96 windows. */
static inline uint32_t hash_windows(const uint32_t* w, uint32_t sip, uint32_t dip, uint32_t ports) {
    const uint32_t words[3] = {sip, dip, ports};
    uint32_t result = 0;
    for (int i = 0; i < 96; ++i)
        if ((words[i >> 5] >> (31 - (i & 31))) & 1) result ^= w[i];
    return result;
}

/*
 * Batch form over packed tuples (uint32 sip, dip, ports per tuple; ports =
 * sport << 16 | dport).  Any output pointer may be NULL.  counts has nqueues
 * entries and is overwritten.  Returns 0 or -22 (EINVAL).
 */
int oracle_run(const uint8_t* key, size_t len, const uint32_t* tuples, size_t n, uint32_t htable,
               uint32_t nqueues, uint32_t* hash_out, uint32_t* queue_out, uint64_t* counts,
               int threads) {
    uint32_t w[96];
    if (oracle_windows(key, len, w)) return -22;
    if (htable < 1 || nqueues < 1) return -22;
    if (counts) memset(counts, 0, sizeof(uint64_t) * nqueues);
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel num_threads(threads)
#endif
    {
        uint64_t* local = NULL;
        uint64_t local_small[256];
        if (counts) {
            if (nqueues <= 256) {
                local = local_small;
                memset(local, 0, sizeof(uint64_t) * nqueues);
            }
        }
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            const uint32_t* t = tuples + 3 * i;
            const uint32_t h = hash_windows(w, t[0], t[1], t[2]);
            const uint32_t q = (h % htable) % nqueues;
            if (hash_out) hash_out[i] = h;
            if (queue_out) queue_out[i] = q;
            if (counts) {
                if (local) {
                    ++local[q];
                } else {
#ifdef _OPENMP
#pragma omp atomic
#endif
                    ++counts[q];
                }
            }
        }
        if (counts && local) {
#ifdef _OPENMP
#pragma omp critical
#endif
            for (uint32_t q = 0; q < nqueues; ++q) counts[q] += local[q];
        }
    }
    return 0;
}

/*
 * The bench's "optimised CPU" line, not a checker: the same batch as
 * oracle_run with the 96 windows pre-summed into twelve 256-entry byte tables (12 KiB,
 * L1-resident; entry v of table j = XOR of the windows of the bits set in input byte j),
 * 12 lookups per tuple, OpenMP over tuples, per-thread histograms.  hash % htable %
 * nqueues as the reference.  tests/test_oracle.py checks it against oracle_run.
 */
int oracle_run_tables(const uint8_t* key, size_t len, const uint32_t* tuples, size_t n,
                      uint32_t htable, uint32_t nqueues, uint32_t* hash_out, uint32_t* queue_out,
                      uint64_t* counts, int threads) {
    uint32_t w[96];
    if (oracle_windows(key, len, w)) return -22;
    if (htable < 1 || nqueues < 1 || (counts && nqueues > 65536)) return -22;
    uint32_t(*T)[256] = malloc(sizeof(uint32_t[12][256]));
    if (!T) return -12;
    for (int j = 0; j < 12; ++j)
        for (int v = 0; v < 256; ++v) {
            uint32_t x = 0;
            for (int b = 0; b < 8; ++b)
                if ((v >> (7 - b)) & 1) x ^= w[8 * j + b];  /* input bit 8j+b is the byte's bit 7-b */
            T[j][v] = x;
        }
    if (counts) memset(counts, 0, sizeof(uint64_t) * nqueues);
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel num_threads(threads)
#endif
    {
        uint64_t* local = counts ? calloc(nqueues, sizeof(uint64_t)) : NULL;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            const uint32_t* t = tuples + 3 * i;
            uint32_t h = 0;
            for (int k = 0; k < 3; ++k) {
                const uint32_t x = t[k];  /* byte 0 of the input is the word's top byte */
                h ^= T[4 * k][x >> 24] ^ T[4 * k + 1][(x >> 16) & 255] ^
                     T[4 * k + 2][(x >> 8) & 255] ^ T[4 * k + 3][x & 255];
            }
            const uint32_t q = (h % htable) % nqueues;
            if (hash_out) hash_out[i] = h;
            if (queue_out) queue_out[i] = q;
            if (local) ++local[q];
        }
        if (local) {
#ifdef _OPENMP
#pragma omp critical
#endif
            for (uint32_t q = 0; q < nqueues; ++q) counts[q] += local[q];
            free(local);
        }
    }
    free(T);
    return 0;
}

/*
 * Batch form over tuples of `nwords` big-endian-valued uint32 words each (the input bytes
 * are the words' big-endian bytes: nwords = 3 is oracle_run's packed IPv4 tuple, 9 the
 * 36-byte IPv6 tuple -- src 16 B, dst 16 B, sport << 16 | dport).  The same literal loop as
 * oracle_hash_bytes, with the rotations precomputed as the 32 * nwords windows
 * (oracle_windows_n); hash % htable % nqueues and the histogram as oracle_run.  Any output
 * may be NULL; counts (nqueues entries) is overwritten.  Returns 0 or -22.
 */
int oracle_run_words(const uint8_t* key, size_t len, const uint32_t* words, int nwords, size_t n,
                     uint32_t htable, uint32_t nqueues, uint32_t* hash_out, uint32_t* queue_out,
                     uint64_t* counts, int threads) {
    if (nwords < 1 || nwords > 16 || htable < 1 || nqueues < 1) return -22;
    uint32_t w[32 * 16];
    if (oracle_windows_n(key, len, 32 * nwords, w)) return -22;
    if (counts) memset(counts, 0, sizeof(uint64_t) * nqueues);
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel num_threads(threads)
#endif
    {
        uint64_t* local = counts ? calloc(nqueues, sizeof(uint64_t)) : NULL;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            const uint32_t* t = words + (size_t)nwords * i;
            uint32_t h = 0;
            for (int b = 0; b < 32 * nwords; ++b)  /* input bit b: MSB first, word by word */
                if ((t[b >> 5] >> (31 - (b & 31))) & 1) h ^= w[b];
            const uint32_t q = (h % htable) % nqueues;
            if (hash_out) hash_out[i] = h;
            if (queue_out) queue_out[i] = q;
            if (local) ++local[q];
        }
        if (local) {
#ifdef _OPENMP
#pragma omp critical
#endif
            for (uint32_t q = 0; q < nqueues; ++q) counts[q] += local[q];
            free(local);
        }
    }
    return 0;
}

/* splitmix64 finaliser; the synthetic generator of include/rss_toeplitz.h. */
static inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void oracle_generate(uint64_t seed, uint64_t first_index, size_t n, uint32_t* tuples) {
    for (size_t i = 0; i < n; ++i) {
        const uint64_t idx = first_index + i;
        const uint64_t r0 = mix64(seed + 2 * idx);
        const uint64_t r1 = mix64(seed + 2 * idx + 1);
        tuples[3 * i + 0] = (uint32_t)(r0 >> 32);
        tuples[3 * i + 1] = (uint32_t)r0;
        tuples[3 * i + 2] = (uint32_t)r1;
    }
}

/* gen_csv.c -- write N canonical 4-tuple CSV rows (splitmix64 stream) for e2e timing.
 * usage: gen_csv N SEED OUT.csv        (tool, not product) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const uint64_t n = strtoull(argv[1], 0, 0), seed = strtoull(argv[2], 0, 0);
    FILE* f = fopen(argv[3], "wb");
    if (!f) return 1;
    static char buf[1 << 20];
    setvbuf(f, buf, _IOFBF, sizeof buf);
    fputs("src_ip,dst_ip,src_port,dst_port\n", f);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t r0 = mix64(seed + 2 * i), r1 = mix64(seed + 2 * i + 1);
        const uint32_t s = (uint32_t)(r0 >> 32), d = (uint32_t)r0, p = (uint32_t)r1;
        fprintf(f, "%u.%u.%u.%u,%u.%u.%u.%u,%u,%u\n", s >> 24, (s >> 16) & 255, (s >> 8) & 255,
                s & 255, d >> 24, (d >> 16) & 255, (d >> 8) & 255, d & 255, p >> 16, p & 0xFFFF);
    }
    return fclose(f) ? 1 : 0;
}

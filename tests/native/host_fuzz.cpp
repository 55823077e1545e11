// host_fuzz.cpp -- sanitizer fuzz driver for the library's host-side parsers (test
// infrastructure; SURVEY.md §5 "Race detection / sanitizers").  Built with
// -fsanitize=address,undefined -fno-sanitize-recover=all together with rss_csv.cpp and
// rss_pcap.cpp by `make -C rss_simulator_nvidia_amd/csrc asan` (g++ only, no HIP).
//
//   rss_host_fuzz SEED ITERATIONS FILE...
//
// Each FILE is a seed image (a pcap, a pcapng or a 4-tuple / IPv6 CSV).  Every iteration
// takes one seed, applies 1-8 random mutations (bit flips, byte overwrites with
// interesting values, truncation, insertion, deletion, duplication of a span, splicing
// in part of another seed), and feeds the result to every parser entry point:
// rss_pcap_parse / rss_pcap_parse6 (count-only, then into exactly-sized buffers),
// rss_csv_parse / rss_csv_parse6 (1 and 4 threads) and, when a CSV parses, the
// formatters rss_csv_format / rss_csv_format6 into exactly-bounded buffers.  Any memory
// error or undefined behaviour aborts the process (sanitizer report on stderr).  Prints
// one summary line of how many images each parser accepted.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "rss_internal.h"
#include "rss_toeplitz.h"

// the library's definition lives in the HIP translation unit; the host parsers only
// need its contract: record a message, return the code
int rss_set_error(int code, const char* fmt, ...) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return code;
}

namespace {

using Bytes = std::vector<uint8_t>;

Bytes read_file(const char* path) {
    std::ifstream f(path, std::ios::binary);
    return Bytes(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

const uint8_t kInteresting[] = {0x00, 0x01, 0x7F, 0x80, 0xFF, 0x0A, 0x0D, ',', '.', ':',
                                '0',  '9',  0x45, 0x60, 0x06, 0x11, 0x84, 0x2C, 0x3A, 0x08};

void mutate(Bytes& b, const std::vector<Bytes>& seeds, std::mt19937_64& rng) {
    const int rounds = 1 + (int)(rng() % 8);
    for (int r = 0; r < rounds; ++r) {
        const size_t n = b.size();
        const size_t pos = n ? rng() % n : 0;
        switch (rng() % 8) {
            case 0:  // bit flip
                if (n) b[pos] ^= (uint8_t)(1u << (rng() % 8));
                break;
            case 1:  // interesting byte
                if (n) b[pos] = kInteresting[rng() % sizeof kInteresting];
                break;
            case 2:  // truncate
                b.resize(n ? rng() % (n + 1) : 0);
                break;
            case 3: {  // insert random bytes
                const size_t k = 1 + rng() % 16;
                Bytes ins(k);
                for (auto& x : ins) x = (uint8_t)rng();
                b.insert(b.begin() + (long)pos, ins.begin(), ins.end());
                break;
            }
            case 4: {  // delete a span
                if (!n) break;
                const size_t k = 1 + rng() % std::min<size_t>(n - pos, 64);
                b.erase(b.begin() + (long)pos, b.begin() + (long)(pos + k));
                break;
            }
            case 5: {  // duplicate a span
                if (!n) break;
                const size_t k = 1 + rng() % std::min<size_t>(n - pos, 128);
                Bytes span(b.begin() + (long)pos, b.begin() + (long)(pos + k));
                b.insert(b.begin() + (long)(rng() % (b.size() + 1)), span.begin(), span.end());
                break;
            }
            case 6: {  // 16/32-bit field overwrite with an extreme value
                if (n < 4) break;
                const uint32_t v[] = {0u, 1u, 0xFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu, 0x80000000u,
                                      (uint32_t)n, (uint32_t)n + 1};
                const uint32_t x = v[rng() % 8];
                memcpy(&b[pos - pos % 4 < n - 4 ? pos - pos % 4 : n - 4], &x, 4);
                break;
            }
            default: {  // splice part of another seed
                const Bytes& o = seeds[rng() % seeds.size()];
                if (o.empty()) break;
                const size_t a = rng() % o.size(), k = 1 + rng() % std::min<size_t>(o.size() - a, 256);
                b.insert(b.begin() + (long)pos, o.begin() + (long)a, o.begin() + (long)(a + k));
                break;
            }
        }
    }
}

struct Stats {
    size_t pcap4 = 0, pcap6 = 0, csv4 = 0, csv6 = 0, dotted = 0, ipv6 = 0;
};

void run_one(const Bytes& img, Stats& st) {
    // exact-size heap copy: any read past the image is a sanitizer report
    uint8_t* data = static_cast<uint8_t*>(malloc(img.size() ? img.size() : 1));
    if (!img.empty()) memcpy(data, img.data(), img.size());
    const size_t len = img.size();

    size_t n = 0, skipped = 0;
    if (rss_pcap_parse(data, len, nullptr, nullptr, 0, &n, &skipped) == RSS_OK) {
        std::vector<rss_tuple4> t(n ? n : 1);
        std::vector<uint8_t> pr(n ? n : 1);
        size_t n2 = 0;
        if (rss_pcap_parse(data, len, t.data(), pr.data(), n, &n2, &skipped) != RSS_OK || n2 != n)
            abort();
        ++st.pcap4;
    }
    if (rss_pcap_parse6(data, len, nullptr, nullptr, 0, &n, &skipped) == RSS_OK) {
        std::vector<rss_tuple6> t(n ? n : 1);
        std::vector<uint8_t> pr(n ? n : 1);
        size_t n2 = 0;
        if (rss_pcap_parse6(data, len, t.data(), pr.data(), n, &n2, &skipped) != RSS_OK || n2 != n)
            abort();
        ++st.pcap6;
    }
    const char* text = reinterpret_cast<const char*>(data);
    for (int threads : {1, 4}) {
        rss_csv_layout layout;
        size_t rows = 0;
        const size_t cap = len / 19 + 1;
        std::vector<rss_tuple4> t(cap);
        if (rss_csv_parse(text, len, t.data(), cap, &rows, &layout, threads) == RSS_OK) {
            std::vector<uint32_t> h(rows ? rows : 1), q(rows ? rows : 1);
            for (size_t i = 0; i < rows; ++i) {
                h[i] = t[i].sip ^ t[i].ports;
                q[i] = h[i] % 24u;
            }
            std::vector<uint64_t> counts(24, 0);
            for (size_t i = 0; i < rows; ++i) ++counts[q[i]];
            const size_t bound = rss_csv_format_bound(rows, 24);
            char* out = static_cast<char*>(malloc(bound));
            size_t out_len = 0;
            if (rss_csv_format(t.data(), h.data(), q.data(), rows, counts.data(), 24, &layout, out,
                               bound, &out_len, threads) != RSS_OK || out_len > bound)
                abort();
            free(out);
            if (threads == 1) ++st.csv4;
        }
        const size_t cap6 = len / 9 + 1;
        std::vector<rss_tuple6> t6(cap6);
        std::vector<uint64_t> spans(2 * cap6);
        if (rss_csv_parse6(text, len, t6.data(), spans.data(), cap6, &rows, &layout, threads) ==
            RSS_OK) {
            std::vector<uint32_t> h(rows ? rows : 1, 0xFFFFFFFFu), q(rows ? rows : 1, 7u);
            std::vector<uint64_t> counts(8, 0);
            counts[7] = rows;
            const size_t bound = rss_csv_format6_bound(spans.data(), rows, 8);
            char* out = static_cast<char*>(malloc(bound));
            size_t out_len = 0;
            if (rss_csv_format6(text, spans.data(), h.data(), q.data(), rows, counts.data(), 8,
                                &layout, out, bound, &out_len, threads) != RSS_OK ||
                out_len > bound)
                abort();
            free(out);
            if (threads == 1) ++st.csv6;
        }
    }
    // the DataFrame address-column parsers: the image as '\n'-joined cells
    size_t cells = 1;
    for (size_t i = 0; i < len; ++i) cells += text[i] == '\n';
    std::vector<uint32_t> addr(4 * cells);
    std::vector<uint8_t> ok(cells);
    if (rss_parse_dotted(text, len, cells, addr.data(), ok.data()) != RSS_OK) abort();
    if (rss_parse_dotted(text, len, cells + 1, addr.data(), ok.data()) != RSS_EINVAL) abort();
    for (size_t i = 0, a = 0; i < cells; ++i) {  // a canonical cell is what formatting writes
        size_t b = a;
        while (b < len && text[b] != '\n') ++b;
        if (ok[i] == 2) {
            char buf[16];
            const uint32_t v = addr[i];
            const int k = snprintf(buf, sizeof buf, "%u.%u.%u.%u", v >> 24, (v >> 16) & 255u,
                                   (v >> 8) & 255u, v & 255u);
            if ((size_t)k != b - a || memcmp(buf, text + a, b - a) != 0) abort();
            ++st.dotted;
        }
        a = b + 1;
    }
    if (rss_parse_ipv6(text, len, cells, addr.data(), ok.data()) != RSS_OK) abort();
    for (size_t i = 0; i < cells; ++i) st.ipv6 += ok[i];
    free(data);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s SEED ITERATIONS FILE...\n", argv[0]);
        return 2;
    }
    std::mt19937_64 rng(strtoull(argv[1], nullptr, 0));
    const long iters = strtol(argv[2], nullptr, 0);
    std::vector<Bytes> seeds;
    for (int i = 3; i < argc; ++i) seeds.push_back(read_file(argv[i]));
    Stats st;
    for (const Bytes& s : seeds) run_one(s, st);  // the seeds themselves, unmutated
    for (long it = 0; it < iters; ++it) {
        Bytes b = seeds[rng() % seeds.size()];
        mutate(b, seeds, rng);
        run_one(b, st);
    }
    printf("fuzz ok: %ld images, accepted pcap4 %zu pcap6 %zu csv4 %zu csv6 %zu dotted %zu "
           "ipv6 %zu\n",
           iters + (long)seeds.size(), st.pcap4, st.pcap6, st.csv4, st.csv6, st.dotted, st.ipv6);
    return 0;
}

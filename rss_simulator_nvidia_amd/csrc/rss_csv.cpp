// rss_csv.cpp -- host CSV ingest/egress fast path for the 4-tuple schema.
//
// Replaces, for canonical files, the pandas steps around the hot path:
//   pd.read_csv(csv_path)                       rss_simulator/simulator.py:55
//   value_counts().sort_index().to_csv(output)  rss_simulator/simulator.py:107-114
//   df.to_csv(output, mode="a", index=False)    rss_simulator/simulator.py:115
// A file is canonical when the header is exactly the four input columns in any
// order and every data row holds four unquoted fields: dotted-quad addresses
// with octets 0..255 written without leading zeros and decimal ports 0..65535
// without sign or leading zeros (LF or CRLF line ends, empty lines skipped).
// pandas reads such fields as str / int64 and writes them back unchanged, so
// rebuilding every field from the packed tuple reproduces its bytes exactly.
// Anything else returns RSS_ENOTSUP and the caller takes the pandas path, which
// keeps the reference's parsing rules and error messages.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rss_toeplitz.h"

namespace {

const char* const kColumnNames[4] = {"src_ip", "dst_ip", "src_port", "dst_port"};

int pick_threads(int threads, size_t work_items) {
    if (threads <= 0) {
        const unsigned hw = std::thread::hardware_concurrency();
        threads = (int)std::min(16u, hw ? hw : 1u);  // the GPU box's CPU share is 16
    }
    const size_t useful = work_items / 65536 + 1;  // below ~64K rows one thread is enough
    return (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, useful));
}

// [b, e) without its trailing '\r'
inline const char* trim_cr(const char* b, const char* e) { return (e > b && e[-1] == '\r') ? e - 1 : e; }

bool parse_header(const char* b, const char* e, uint8_t field_column[4]) {
    int seen = 0;
    for (int f = 0; f < 4; ++f) {
        const char* comma = f < 3 ? static_cast<const char*>(memchr(b, ',', e - b)) : e;
        if (!comma) return false;
        const size_t len = comma - b;
        int col = -1;
        for (int c = 0; c < 4; ++c)
            if (len == strlen(kColumnNames[c]) && memcmp(b, kColumnNames[c], len) == 0) col = c;
        if (col < 0 || (seen & (1 << col))) return false;
        seen |= 1 << col;
        field_column[f] = (uint8_t)col;
        b = comma + 1;
    }
    return seen == 15;
}

// canonical unsigned decimal in [b, e): 1..max_digits digits, no leading zero
inline bool parse_uint(const char* b, const char* e, int max_digits, uint32_t max_value, uint32_t& v) {
    const long len = e - b;
    if (len < 1 || len > max_digits || (len > 1 && *b == '0')) return false;
    uint32_t x = 0;
    for (const char* p = b; p < e; ++p) {
        const unsigned d = (unsigned)(*p - '0');
        if (d > 9) return false;
        x = x * 10 + d;
    }
    if (x > max_value) return false;
    v = x;
    return true;
}

inline bool parse_ip(const char* b, const char* e, uint32_t& out) {
    uint32_t ip = 0;
    for (int k = 0; k < 4; ++k) {
        const char* dot = k < 3 ? static_cast<const char*>(memchr(b, '.', e - b)) : e;
        if (!dot) return false;
        uint32_t octet;
        if (!parse_uint(b, dot, 3, 255, octet)) return false;
        ip = ip << 8 | octet;
        b = dot + 1;
    }
    out = ip;
    return true;
}

bool parse_row(const char* b, const char* e, const uint8_t field_column[4], rss_tuple4& t) {
    uint32_t v[4];
    for (int f = 0; f < 4; ++f) {
        const char* comma = f < 3 ? static_cast<const char*>(memchr(b, ',', e - b)) : e;
        if (!comma) return false;
        const int col = field_column[f];
        const bool ok = col < 2 ? parse_ip(b, comma, v[col]) : parse_uint(b, comma, 5, 65535, v[col]);
        if (!ok) return false;  // also rejects a fifth field (',' inside the last one)
        b = comma + 1;
    }
    t.sip = v[0];
    t.dip = v[1];
    t.ports = v[2] << 16 | v[3];
    return true;
}

// Split [b, e) into up to `parts` ranges that start at line starts.
std::vector<const char*> split_lines(const char* b, const char* e, int parts) {
    std::vector<const char*> cuts{b};
    for (int k = 1; k < parts; ++k) {
        const char* p = b + (e - b) * k / parts;
        if (p <= cuts.back()) continue;
        const char* nl = static_cast<const char*>(memchr(p, '\n', e - p));
        if (!nl || nl + 1 >= e) break;
        if (nl + 1 > cuts.back()) cuts.push_back(nl + 1);
    }
    cuts.push_back(e);
    return cuts;
}

// Calls fn(line_begin, line_end_without_cr) for each non-empty line of [b, e).
template <typename F>
bool for_each_line(const char* b, const char* e, F&& fn) {
    while (b < e) {
        const char* nl = static_cast<const char*>(memchr(b, '\n', e - b));
        const char* end = nl ? nl : e;
        const char* t = trim_cr(b, end);
        if (t > b && !fn(b, t)) return false;
        b = nl ? nl + 1 : e;
    }
    return true;
}

inline char* put_uint(char* p, uint64_t v) {
    char tmp[24];
    int n = 0;
    do {
        tmp[n++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    while (n) *p++ = tmp[--n];
    return p;
}

inline char* put_ip(char* p, uint32_t ip) {
    for (int k = 3; k >= 0; --k) {
        p = put_uint(p, (ip >> (8 * k)) & 0xFF);
        if (k) *p++ = '.';
    }
    return p;
}

constexpr size_t kMaxRowBytes = 15 + 1 + 15 + 1 + 5 + 1 + 5 + 1 + 10 + 1 + 10 + 1;

}  // namespace

extern "C" {

size_t rss_csv_format_bound(size_t n, uint32_t nqueues) {
    return 64 + (size_t)nqueues * 32 + 96 + n * kMaxRowBytes;
}

int rss_csv_parse(const char* data, size_t len, rss_tuple4* tuples, size_t cap, size_t* n_rows,
                  rss_csv_layout* layout, int threads) {
    if (!data || !n_rows || !layout) return RSS_EINVAL;
    *n_rows = 0;
    const char* end = data + len;
    const char* nl = static_cast<const char*>(memchr(data, '\n', len));
    const char* hend = trim_cr(data, nl ? nl : end);
    if (!parse_header(data, hend, layout->field_column)) return RSS_ENOTSUP;
    const char* body = nl ? nl + 1 : end;
    if (body >= end) return RSS_ENOTSUP;  // no data rows: the pandas path raises
    for (const char* p = data; p < end; ++p)  // ASCII only: pandas decodes utf-8
        if ((unsigned char)*p >= 0x80) return RSS_ENOTSUP;

    const int nt = pick_threads(threads, (end - body) / 32);
    const std::vector<const char*> cuts = split_lines(body, end, nt);
    const int parts = (int)cuts.size() - 1;
    std::vector<size_t> rows(parts + 1, 0);
    std::vector<std::thread> pool;
    for (int k = 0; k < parts; ++k)
        pool.emplace_back([&, k] {
            size_t c = 0;
            for_each_line(cuts[k], cuts[k + 1], [&](const char*, const char*) { ++c; return true; });
            rows[k + 1] = c;
        });
    for (auto& t : pool) t.join();
    pool.clear();
    for (int k = 0; k < parts; ++k) rows[k + 1] += rows[k];
    if (rows[parts] == 0) return RSS_ENOTSUP;
    if (rows[parts] > cap || !tuples) {
        *n_rows = rows[parts];
        return RSS_EINVAL;  // caller's buffer is too small; *n_rows says how many
    }
    std::atomic<bool> ok{true};
    for (int k = 0; k < parts; ++k)
        pool.emplace_back([&, k] {
            rss_tuple4* out = tuples + rows[k];
            const bool good = for_each_line(cuts[k], cuts[k + 1], [&](const char* b, const char* e) {
                return ok.load(std::memory_order_relaxed) && parse_row(b, e, layout->field_column, *out++);
            });
            if (!good) ok = false;
        });
    for (auto& t : pool) t.join();
    if (!ok) return RSS_ENOTSUP;
    *n_rows = rows[parts];
    return RSS_OK;
}

int rss_csv_format(const rss_tuple4* tuples, const uint32_t* hash, const uint32_t* queue, size_t n,
                   const uint64_t* counts, uint32_t nqueues, const rss_csv_layout* layout, char* out,
                   size_t cap, size_t* out_len, int threads) {
    if ((n && (!tuples || !hash || !queue)) || !counts || !layout || !out || !out_len)
        return RSS_EINVAL;
    if (cap < rss_csv_format_bound(n, nqueues)) return RSS_EINVAL;
    for (int f = 0; f < 4; ++f)
        if (layout->field_column[f] > 3) return RSS_EINVAL;
    char* p = out;
    // per-queue counts of the non-empty queues, ascending (value_counts().sort_index())
    memcpy(p, "queue_number,counts\n", 20);
    p += 20;
    for (uint32_t q = 0; q < nqueues; ++q)
        if (counts[q]) {
            p = put_uint(p, q);
            *p++ = ',';
            p = put_uint(p, counts[q]);
            *p++ = '\n';
        }
    for (int f = 0; f < 4; ++f) {
        const char* name = kColumnNames[layout->field_column[f]];
        memcpy(p, name, strlen(name));
        p += strlen(name);
        *p++ = ',';
    }
    memcpy(p, "hash_result,queue_number\n", 25);
    p += 25;

    const int nt = pick_threads(threads, n);
    std::vector<std::string> parts(nt);
    std::vector<std::thread> pool;
    for (int k = 0; k < nt; ++k)
        pool.emplace_back([&, k] {
            const size_t a = n * k / nt, b = n * (k + 1) / nt;
            std::string& s = parts[k];
            s.resize((b - a) * kMaxRowBytes);
            char* w = &s[0];
            for (size_t i = a; i < b; ++i) {
                const rss_tuple4& t = tuples[i];
                const uint32_t col[4] = {t.sip, t.dip, t.ports >> 16, t.ports & 0xFFFF};
                for (int f = 0; f < 4; ++f) {
                    const int c = layout->field_column[f];
                    w = c < 2 ? put_ip(w, col[c]) : put_uint(w, col[c]);
                    *w++ = ',';
                }
                w = put_uint(w, hash[i]);
                *w++ = ',';
                w = put_uint(w, queue[i]);
                *w++ = '\n';
            }
            s.resize(w - &s[0]);
        });
    for (auto& t : pool) t.join();
    pool.clear();
    std::vector<size_t> off(nt + 1, (size_t)(p - out));
    for (int k = 0; k < nt; ++k) off[k + 1] = off[k] + parts[k].size();
    for (int k = 0; k < nt; ++k)
        pool.emplace_back([&, k] { memcpy(out + off[k], parts[k].data(), parts[k].size()); });
    for (auto& t : pool) t.join();
    *out_len = off[nt];
    return RSS_OK;
}

}  // extern "C"

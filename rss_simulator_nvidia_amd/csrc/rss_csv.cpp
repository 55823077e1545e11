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
#include <thread>
#include <vector>

#include "rss_internal.h"
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

inline bool is_digit(const char* p, const char* e) { return p < e && (unsigned)(*p - '0') <= 9; }

// Canonical unsigned decimal at p (1..kMaxDigits digits, no leading zero, <= kMax);
// advances p past it.
template <int kMaxDigits, uint32_t kMax>
inline bool scan_uint(const char*& p, const char* e, uint32_t& v) {
    if (!is_digit(p, e)) return false;
    uint32_t x = (uint32_t)(*p++ - '0');
    if (x == 0) {
        v = 0;
        return !is_digit(p, e);
    }
    for (int k = 1; k < kMaxDigits && is_digit(p, e); ++k) x = x * 10 + (uint32_t)(*p++ - '0');
    if (is_digit(p, e) || x > kMax) return false;
    v = x;
    return true;
}

inline bool scan_ip(const char*& p, const char* e, uint32_t& out) {
    uint32_t ip = 0;
    for (int k = 0; k < 4; ++k) {
        uint32_t octet;
        if (!scan_uint<3, 255>(p, e, octet)) return false;
        ip = ip << 8 | octet;
        if (k < 3) {
            if (p >= e || *p != '.') return false;
            ++p;
        }
    }
    out = ip;
    return true;
}

// One data row starting at p; on success p points past its line end ("\n", "\r\n"
// or end of input).
inline bool scan_row(const char*& p, const char* e, const uint8_t field_column[4], rss_tuple4& t) {
    uint32_t v[4];
    for (int f = 0; f < 4; ++f) {
        const int col = field_column[f];
        if (!(col < 2 ? scan_ip(p, e, v[col]) : scan_uint<5, 65535>(p, e, v[col]))) return false;
        if (f < 3) {
            if (p >= e || *p != ',') return false;
            ++p;
        }
    }
    if (p < e && *p == '\r') ++p;
    if (p < e) {
        if (*p != '\n') return false;
        ++p;
    }
    t.sip = v[0];
    t.dip = v[1];
    t.ports = v[2] << 16 | v[3];
    return true;
}

// If p starts an empty line ("\n", "\r\n", or a final "\r"), skip it.
inline bool skip_empty_line(const char*& p, const char* e) {
    if (*p == '\n') {
        ++p;
        return true;
    }
    if (*p == '\r' && (p + 1 == e || p[1] == '\n')) {
        p += (p + 1 == e) ? 1 : 2;
        return true;
    }
    return false;
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

const char kDigits2[201] =
    "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
    "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
    "8081828384858687888990919293949596979899";

inline size_t uint_len(uint64_t v);

inline char* put_uint(char* p, uint64_t v) {
    const size_t len = uint_len(v);
    char* w = p + len;
    while (v >= 100) {
        const unsigned r = (unsigned)(v % 100);
        v /= 100;
        w -= 2;
        memcpy(w, kDigits2 + 2 * r, 2);
    }
    if (v >= 10) {
        w -= 2;
        memcpy(w, kDigits2 + 2 * v, 2);
    } else {
        *--w = (char)('0' + v);
    }
    return p + len;
}

inline size_t uint_len(uint64_t v) {
    size_t n = 1;
    while (v >= 10000) {
        v /= 10000;
        n += 4;
    }
    return n + (v >= 10) + (v >= 100) + (v >= 1000);
}

inline size_t octet_len(uint32_t v) { return v >= 100 ? 3 : (v >= 10 ? 2 : 1); }

inline size_t ip_len(uint32_t ip) {
    return octet_len(ip >> 24) + octet_len((ip >> 16) & 0xFF) + octet_len((ip >> 8) & 0xFF) +
           octet_len(ip & 0xFF) + 3;
}

inline char* put_ip(char* p, uint32_t ip) {
    for (int k = 3; k >= 0; --k) {
        p = put_uint(p, (ip >> (8 * k)) & 0xFF);
        if (k) *p++ = '.';
    }
    return p;
}

constexpr size_t kMaxRowBytes = 15 + 1 + 15 + 1 + 5 + 1 + 5 + 1 + 10 + 1 + 10 + 1;

// ---- IPv6 rows (SURVEY.md §8f row 4 input through the row-1 fast path) ----
// A canonical IPv6 address is RFC 4291 text without an embedded IPv4 part or zone:
// 1-4 hex digits per group, ':' between groups, at most one '::' standing for one or
// more zero groups, 8 groups without it and at most 7 with it.  ipaddress.IPv6Address
// (the pandas path's parser, ingest.py) reads every such text to the same 128 bits;
// pandas keeps it as a str and writes it back verbatim, so the output row is the
// input line's text plus the two new columns.
// character classes of the IPv6 scanner: 0..15 hex digit, kColon, kEnd (',' '\r' '\n'),
// kBad (anything else)
enum : int8_t { kColon = 16, kEnd = 17, kBad = -1 };
struct Hex6Table {
    int8_t v[256];
    constexpr Hex6Table() : v() {
        for (int c = 0; c < 256; ++c)
            v[c] = (c >= '0' && c <= '9') ? (int8_t)(c - '0')
                 : (c >= 'a' && c <= 'f') ? (int8_t)(c - 'a' + 10)
                 : (c >= 'A' && c <= 'F') ? (int8_t)(c - 'A' + 10)
                 : c == ':'                ? (int8_t)kColon
                 : (c == ',' || c == '\r' || c == '\n') ? (int8_t)kEnd
                                                         : (int8_t)kBad;
    }
};
constexpr Hex6Table kHex6{};

inline int char_class(const char* p, const char* e) {
    return p < e ? (int)kHex6.v[(unsigned char)*p] : (int)kEnd;
}

inline int hex_value(char c) {
    const int v = kHex6.v[(unsigned char)c];
    return v < 16 ? v : -1;
}

inline bool field_end(const char* p, const char* e) { return char_class(p, e) == kEnd; }

inline bool scan_ip6(const char*& p, const char* e, uint32_t out[4]) {
    uint32_t g[8];
    int ng = 0, gap = -1;
    if (p + 1 < e && p[0] == ':' && p[1] == ':') {
        gap = 0;
        p += 2;
    }
    while (!(gap >= 0 && field_end(p, e))) {
        uint32_t v = 0;
        int digits = 0, h;
        while ((h = char_class(p, e)) >= 0 && h < 16 && digits < 4) {
            v = v << 4 | (uint32_t)h;
            ++digits;
            ++p;
        }
        if (digits == 0 || (h >= 0 && h < 16) || ng == 8) return false;
        g[ng++] = v;
        if (h == kEnd) break;
        if (h != kColon) return false;
        if (p + 1 < e && p[1] == ':') {
            if (gap >= 0) return false;
            gap = ng;
            p += 2;
        } else {
            ++p;  // a single ':' must be followed by another group
        }
    }
    if (gap < 0 ? ng != 8 : ng > 7) return false;
    uint32_t full[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int tail = gap < 0 ? 0 : ng - gap;
    for (int k = 0; k < ng; ++k) full[(gap < 0 || k < gap) ? k : 8 - tail + (k - gap)] = g[k];
    for (int k = 0; k < 4; ++k) out[k] = full[2 * k] << 16 | full[2 * k + 1];
    return true;
}

// One IPv6 data row at p: tuple + the byte span of its text (without the line end).
inline bool scan_row6(const char*& p, const char* e, const uint8_t field_column[4], rss_tuple6& t,
                      const char*& text_end) {
    uint32_t addr[2][4], port[2];
    for (int f = 0; f < 4; ++f) {
        const int col = field_column[f];
        if (!(col < 2 ? scan_ip6(p, e, addr[col]) : scan_uint<5, 65535>(p, e, port[col - 2])))
            return false;
        if (f < 3) {
            if (p >= e || *p != ',') return false;
            ++p;
        }
    }
    text_end = p;
    if (p < e && *p == '\r') ++p;
    if (p < e) {
        if (*p != '\n') return false;
        ++p;
    }
    for (int k = 0; k < 4; ++k) {
        t.w[k] = addr[0][k];
        t.w[4 + k] = addr[1][k];
    }
    t.w[8] = port[0] << 16 | port[1];
    return true;
}

constexpr size_t kMaxRow6Extra = 1 + 10 + 1 + 10 + 1;  // ",hash,queue\n"

}  // namespace

bool rss_csv_header(const char* data, size_t len, rss_csv_layout* layout, size_t* body_offset) {
    const char* end = data + len;
    const char* nl = static_cast<const char*>(memchr(data, '\n', len));
    const char* hend = trim_cr(data, nl ? nl : end);
    if (!parse_header(data, hend, layout->field_column)) return false;
    const char* body = nl ? nl + 1 : end;
    if (body >= end) return false;  // no data rows: the pandas path raises
    *body_offset = (size_t)(body - data);
    return true;
}

size_t rss_csv_prefix_bound(uint32_t nqueues) { return 64 + (size_t)nqueues * 32 + 96; }

size_t rss_csv_format_prefix(const uint64_t* counts, uint32_t nqueues,
                             const rss_csv_layout* layout, char* out) {
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
    return (size_t)(p - out);
}

extern "C" {

int rss_parse_dotted(const char* text, size_t len, size_t n, uint32_t* out, uint8_t* ok) {
    if ((n && (!out || !ok)) || (len && !text)) return RSS_EINVAL;
    const char* p = text;
    const char* const end = text + len;
    for (size_t i = 0; i < n; ++i) {
        const char* eol = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
        if (i + 1 < n ? !eol : eol != nullptr) return RSS_EINVAL;  // exactly n cells
        const char* const cell_end = eol ? eol : end;
        uint64_t value = 0;
        int octets = 0, digits = 0;
        uint32_t octet = 0;
        bool good = true, canonical = true;
        for (const char* c = p; c < cell_end && good; ++c) {
            if (*c >= '0' && *c <= '9') {
                canonical = canonical && !(digits == 1 && octet == 0);  // no leading zero
                octet = octet * 10 + (uint32_t)(*c - '0');
                good = ++digits <= 3;
            } else if (*c == '.') {
                good = digits > 0 && octets < 3;
                canonical = canonical && octet <= 255;
                value |= (uint64_t)octet << (24 - 8 * octets);  // (no range check: OR)
                ++octets;
                octet = 0;
                digits = 0;
            } else {
                good = false;
            }
        }
        good = good && octets == 3 && digits > 0;
        canonical = good && canonical && octet <= 255;
        ok[i] = canonical ? 2 : (good ? 1 : 0);
        out[i] = good ? (uint32_t)(value | octet) : 0u;
        p = eol ? eol + 1 : end;
    }
    return RSS_OK;
}

int rss_parse_ipv6(const char* text, size_t len, size_t n, uint32_t* out, uint8_t* ok) {
    if ((n && (!out || !ok)) || (len && !text)) return RSS_EINVAL;
    const char* p = text;
    const char* const end = text + len;
    for (size_t i = 0; i < n; ++i) {
        const char* eol = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
        if (i + 1 < n ? !eol : eol != nullptr) return RSS_EINVAL;  // exactly n cells
        const char* const cell_end = eol ? eol : end;
        const char* q = p;
        // the row scanner's address rules (scan_ip6), and nothing after the address
        const bool good = q < cell_end && scan_ip6(q, cell_end, out + 4 * i) && q == cell_end;
        ok[i] = good ? 1 : 0;
        if (!good) memset(out + 4 * i, 0, 16);
        p = eol ? eol + 1 : end;
    }
    return RSS_OK;
}

size_t rss_csv_format_bound(size_t n, uint32_t nqueues) {
    return rss_csv_prefix_bound(nqueues) + n * kMaxRowBytes;
}

int rss_csv_parse(const char* data, size_t len, rss_tuple4* tuples, size_t cap, size_t* n_rows,
                  rss_csv_layout* layout, int threads) {
    if (!data || !n_rows || !layout) return RSS_EINVAL;
    *n_rows = 0;
    const char* end = data + len;
    size_t body_offset;
    if (!rss_csv_header(data, len, layout, &body_offset)) return RSS_ENOTSUP;
    const char* body = data + body_offset;
    // (no separate ASCII check: rows accept only digits . , \r \n, the header only
    // the four column names, so any non-ASCII byte already fails the scan)

    const int nt = pick_threads(threads, (end - body) / 32);
    const std::vector<const char*> cuts = split_lines(body, end, nt);
    const int parts = (int)cuts.size() - 1;
    // one scanning pass per range into a local buffer, then a parallel gather
    std::vector<std::vector<rss_tuple4>> local(parts);
    std::atomic<bool> ok{true};
    std::vector<std::thread> pool;
    for (int k = 0; k < parts; ++k)
        pool.emplace_back([&, k] {
            const char* p = cuts[k];
            const char* e = cuts[k + 1];
            std::vector<rss_tuple4>& out = local[k];
            out.reserve((size_t)std::count(p, e, '\n') + 1);
            rss_tuple4 t;
            while (p < e) {
                if (skip_empty_line(p, e)) continue;
                if (!scan_row(p, e, layout->field_column, t)) {
                    ok = false;
                    return;
                }
                out.push_back(t);
                if ((out.size() & 4095) == 0 && !ok.load(std::memory_order_relaxed)) return;
            }
        });
    for (auto& t : pool) t.join();
    pool.clear();
    if (!ok) return RSS_ENOTSUP;
    std::vector<size_t> off(parts + 1, 0);
    for (int k = 0; k < parts; ++k) off[k + 1] = off[k] + local[k].size();
    *n_rows = off[parts];
    if (off[parts] == 0) return RSS_ENOTSUP;
    if (off[parts] > cap || !tuples) return RSS_EINVAL;  // *n_rows says how many are needed
    for (int k = 0; k < parts; ++k)
        pool.emplace_back([&, k] {
            if (!local[k].empty())
                memcpy(tuples + off[k], local[k].data(), local[k].size() * sizeof(rss_tuple4));
        });
    for (auto& t : pool) t.join();
    return RSS_OK;
}

int rss_csv_parse6(const char* data, size_t len, rss_tuple6* tuples, uint64_t* spans, size_t cap,
                   size_t* n_rows, rss_csv_layout* layout, int threads) {
    if (!data || !n_rows || !layout) return RSS_EINVAL;
    *n_rows = 0;
    const char* end = data + len;
    size_t body_offset;
    if (!rss_csv_header(data, len, layout, &body_offset)) return RSS_ENOTSUP;
    const char* body = data + body_offset;
    const int nt = pick_threads(threads, (end - body) / 64);
    const std::vector<const char*> cuts = split_lines(body, end, nt);
    const int parts = (int)cuts.size() - 1;
    struct Row {
        rss_tuple6 t;
        uint64_t b, e;
    };
    std::vector<std::vector<Row>> local(parts);
    std::atomic<bool> ok{true};
    std::vector<std::thread> pool;
    for (int k = 0; k < parts; ++k)
        pool.emplace_back([&, k] {
            const char* p = cuts[k];
            const char* e = cuts[k + 1];
            std::vector<Row>& out = local[k];
            out.reserve((size_t)std::count(p, e, '\n') + 1);
            Row r;
            while (p < e) {
                if (skip_empty_line(p, e)) continue;
                const char* b = p;
                const char* te;
                if (!scan_row6(p, e, layout->field_column, r.t, te)) {
                    ok = false;
                    return;
                }
                r.b = (uint64_t)(b - data);
                r.e = (uint64_t)(te - data);
                out.push_back(r);
                if ((out.size() & 4095) == 0 && !ok.load(std::memory_order_relaxed)) return;
            }
        });
    for (auto& t : pool) t.join();
    pool.clear();
    if (!ok) return RSS_ENOTSUP;
    std::vector<size_t> off(parts + 1, 0);
    for (int k = 0; k < parts; ++k) off[k + 1] = off[k] + local[k].size();
    *n_rows = off[parts];
    if (off[parts] == 0) return RSS_ENOTSUP;
    if (off[parts] > cap || !tuples || !spans) return RSS_EINVAL;
    for (int k = 0; k < parts; ++k)
        pool.emplace_back([&, k] {
            for (size_t i = 0; i < local[k].size(); ++i) {
                const Row& r = local[k][i];
                tuples[off[k] + i] = r.t;
                spans[2 * (off[k] + i)] = r.b;
                spans[2 * (off[k] + i) + 1] = r.e;
            }
        });
    for (auto& t : pool) t.join();
    return RSS_OK;
}

size_t rss_csv_format6_bound(const uint64_t* spans, size_t n, uint32_t nqueues) {
    size_t text = 0;
    for (size_t i = 0; i < n; ++i) text += (size_t)(spans[2 * i + 1] - spans[2 * i]);
    return rss_csv_prefix_bound(nqueues) + text + n * kMaxRow6Extra;
}

int rss_csv_format6(const char* data, const uint64_t* spans, const uint32_t* hash,
                    const uint32_t* queue, size_t n, const uint64_t* counts, uint32_t nqueues,
                    const rss_csv_layout* layout, char* out, size_t cap, size_t* out_len,
                    int threads) {
    if ((n && (!data || !spans || !hash || !queue)) || !counts || !layout || !out || !out_len)
        return RSS_EINVAL;
    if (cap < rss_csv_format6_bound(spans, n, nqueues)) return RSS_EINVAL;
    for (int f = 0; f < 4; ++f)
        if (layout->field_column[f] > 3) return RSS_EINVAL;
    char* p = out + rss_csv_format_prefix(counts, nqueues, layout, out);
    const int nt = pick_threads(threads, n);
    std::vector<size_t> off(nt + 1, 0);
    std::vector<std::thread> pool;
    for (int k = 0; k < nt; ++k)
        pool.emplace_back([&, k] {
            const size_t a = n * k / nt, b = n * (k + 1) / nt;
            size_t bytes = 0;
            for (size_t i = a; i < b; ++i)
                bytes += (size_t)(spans[2 * i + 1] - spans[2 * i]) + uint_len(hash[i]) +
                         uint_len(queue[i]) + 3;
            off[k + 1] = bytes;
        });
    for (auto& t : pool) t.join();
    pool.clear();
    off[0] = (size_t)(p - out);
    for (int k = 0; k < nt; ++k) off[k + 1] += off[k];
    for (int k = 0; k < nt; ++k)
        pool.emplace_back([&, k] {
            const size_t a = n * k / nt, b = n * (k + 1) / nt;
            char* w = out + off[k];
            for (size_t i = a; i < b; ++i) {
                const size_t len = (size_t)(spans[2 * i + 1] - spans[2 * i]);
                memcpy(w, data + spans[2 * i], len);
                w += len;
                *w++ = ',';
                w = put_uint(w, hash[i]);
                *w++ = ',';
                w = put_uint(w, queue[i]);
                *w++ = '\n';
            }
        });
    for (auto& t : pool) t.join();
    *out_len = off[nt];
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
    char* p = out + rss_csv_format_prefix(counts, nqueues, layout, out);

    // two passes over row ranges: exact byte count per range, then every thread
    // formats straight into its slice of `out` (no staging copy)
    const int nt = pick_threads(threads, n);
    std::vector<size_t> off(nt + 1, 0);
    auto row_fields = [&](size_t i, uint32_t col[4]) {
        const rss_tuple4& t = tuples[i];
        col[0] = t.sip;
        col[1] = t.dip;
        col[2] = t.ports >> 16;
        col[3] = t.ports & 0xFFFF;
    };
    std::vector<std::thread> pool;
    for (int k = 0; k < nt; ++k)
        pool.emplace_back([&, k] {
            const size_t a = n * k / nt, b = n * (k + 1) / nt;
            size_t bytes = 0;
            for (size_t i = a; i < b; ++i) {
                uint32_t col[4];
                row_fields(i, col);
                bytes += ip_len(col[0]) + ip_len(col[1]) + uint_len(col[2]) + uint_len(col[3]) +
                         uint_len(hash[i]) + uint_len(queue[i]) + 6;
            }
            off[k + 1] = bytes;
        });
    for (auto& t : pool) t.join();
    pool.clear();
    off[0] = (size_t)(p - out);
    for (int k = 0; k < nt; ++k) off[k + 1] += off[k];
    for (int k = 0; k < nt; ++k)
        pool.emplace_back([&, k] {
            const size_t a = n * k / nt, b = n * (k + 1) / nt;
            char* w = out + off[k];
            for (size_t i = a; i < b; ++i) {
                uint32_t col[4];
                row_fields(i, col);
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
        });
    for (auto& t : pool) t.join();
    *out_len = off[nt];
    return RSS_OK;
}

}  // extern "C"

// rss_pcap.cpp -- packet-capture input (the reference's planned
// "Use pcap as input", docs/rss_general_explaination.md:19).
//
// Reads a classic libpcap file image (either byte order, microsecond or nanosecond
// timestamps) or a pcapng image (Wireshark's default format: any number of sections of
// either byte order, per-interface link types, enhanced / simple / obsolete packet
// blocks, every other block skipped) and emits one packed IPv4 4-tuple per IPv4 packet,
// as a NIC's RSS unit would see it: TCP / UDP / SCTP packets contribute their ports,
// everything else (other protocols, and every fragment of a fragmented datagram)
// contributes ports 0, i.e. the 2-tuple hash.  Link types: Ethernet (with 802.1Q /
// 802.1ad tags), Linux cooked capture v1, raw IPv4.  Non-IPv4 and truncated packets,
// and packets of interfaces with other link types, are skipped and counted.
#include <cstring>
#include <vector>

#include "rss_toeplitz.h"

namespace {

inline uint16_t be16(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }
inline uint32_t be32(const uint8_t* p) {
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

struct FileHeader {
    bool swap = false;
    uint32_t linktype = 0;
};

inline uint32_t rd32(const uint8_t* p, bool swap) {
    uint32_t v;
    memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}

enum { DLT_EN10MB = 1, DLT_RAW = 101, DLT_LINUX_SLL = 113, DLT_IPV4 = 228, DLT_IPV6 = 229 };

// Offset of the network-layer header and its ethertype; false if not parseable.
bool link_payload(const uint8_t* pkt, uint32_t caplen, uint32_t linktype, uint32_t* off,
                  uint16_t* ethertype) {
    switch (linktype) {
        case DLT_EN10MB: {
            if (caplen < 14) return false;
            uint32_t o = 12;
            uint16_t et = be16(pkt + o);
            while ((et == 0x8100 || et == 0x88A8 || et == 0x9100) && o + 6 <= caplen) {
                o += 4;  // VLAN / QinQ tag
                et = be16(pkt + o);
            }
            *off = o + 2;
            *ethertype = et;
            return *off <= caplen;
        }
        case DLT_LINUX_SLL:
            if (caplen < 16) return false;
            *off = 16;
            *ethertype = be16(pkt + 14);
            return true;
        case DLT_RAW:
        case DLT_IPV4:
        case DLT_IPV6:
            if (caplen < 1) return false;
            *off = 0;
            *ethertype = (pkt[0] >> 4) == 4 ? 0x0800 : 0x86DD;
            return true;
        default:
            return false;
    }
}

inline uint16_t rd16(const uint8_t* p, bool swap) {
    uint16_t v;
    memcpy(&v, p, 2);
    return swap ? __builtin_bswap16(v) : v;
}

bool supported_linktype(uint32_t lt) {
    return lt == DLT_EN10MB || lt == DLT_RAW || lt == DLT_LINUX_SLL || lt == DLT_IPV4 ||
           lt == DLT_IPV6;
}

bool l4_has_ports(uint8_t proto) { return proto == 6 || proto == 17 || proto == 132; }

// Collects the tuples of a capture: one per IPv4 packet (tuples) or per IPv6 packet
// (tuples6); `skip` counts the rest.
struct TupleSink {
    rss_tuple4* tuples;
    uint8_t* protocols;
    size_t cap;
    rss_tuple6* tuples6 = nullptr;
    bool v6 = false;
    size_t n = 0, skip = 0;

    void packet(const uint8_t* pkt, uint32_t caplen, uint32_t linktype) {
        uint32_t off;
        uint16_t et;
        if (!supported_linktype(linktype) || !link_payload(pkt, caplen, linktype, &off, &et)) {
            ++skip;
            return;
        }
        if (v6) {
            packet6(pkt, caplen, off, et);
            return;
        }
        if (et != 0x0800 || off + 20 > caplen || (pkt[off] >> 4) != 4) {
            ++skip;
            return;
        }
        const uint8_t* ip = pkt + off;
        const uint32_t ihl = (uint32_t)(ip[0] & 15) * 4;
        if (ihl < 20 || off + ihl > caplen) {
            ++skip;
            return;
        }
        const uint8_t proto = ip[9];
        const uint16_t frag = be16(ip + 6);
        const bool fragment = (frag & 0x2000) || (frag & 0x1FFF);  // MF or offset
        uint32_t ports = 0;
        if (!fragment && l4_has_ports(proto)) {
            if (off + ihl + 4 > caplen) {
                ++skip;
                return;
            }
            ports = be32(ip + ihl);  // src port << 16 | dst port
        }
        if (tuples && n < cap) {
            tuples[n].sip = be32(ip + 12);
            tuples[n].dip = be32(ip + 16);
            tuples[n].ports = ports;
            if (protocols) protocols[n] = proto;
        }
        ++n;
    }

    // IPv6: the fixed header's addresses; the extension-header chain (hop-by-hop,
    // routing, destination options, AH, fragment) is walked to the upper layer, whose
    // ports count for TCP / UDP / SCTP.  Fragments (offset or M flag set), ESP and
    // no-next-header packets hash with ports 0, as IPv4 fragments do.
    void packet6(const uint8_t* pkt, uint32_t caplen, uint32_t off, uint16_t et) {
        if (et != 0x86DD || off + 40 > caplen || (pkt[off] >> 4) != 6) {
            ++skip;
            return;
        }
        const uint8_t* ip = pkt + off;
        uint8_t next = ip[6];
        uint32_t pos = off + 40;
        bool fragment = false, truncated = false;
        for (int hops = 0; hops < 16; ++hops) {
            if (next != 0 && next != 43 && next != 60 && next != 51 && next != 44) break;
            if (pos + 8 > caplen) {
                truncated = true;
                break;
            }
            uint32_t hlen;
            if (next == 51) {  // authentication header: length in 4-octet units, minus 2
                hlen = (pkt[pos + 1] + 2u) * 4;
            } else if (next == 44) {  // fragment header: offset or M flag -> a fragment
                const uint16_t fo = be16(pkt + pos + 2);
                fragment = fragment || (fo & 0xFFF8) || (fo & 1);
                hlen = 8;
            } else {  // hop-by-hop, routing, destination options: 8-octet units, minus 1
                hlen = (pkt[pos + 1] + 1u) * 8;
            }
            next = pkt[pos];
            pos += hlen;
        }
        uint32_t ports = 0;
        if (!truncated && !fragment && l4_has_ports(next)) {
            if (pos + 4 > caplen) truncated = true;
            else ports = be32(pkt + pos);
        }
        if (truncated) {
            ++skip;
            return;
        }
        if (tuples6 && n < cap) {
            for (int k = 0; k < 4; ++k) {
                tuples6[n].w[k] = be32(ip + 8 + 4 * k);
                tuples6[n].w[4 + k] = be32(ip + 24 + 4 * k);
            }
            tuples6[n].w[8] = ports;
            if (protocols) protocols[n] = next;
        }
        ++n;
    }
};

int parse_classic(const uint8_t* data, size_t len, TupleSink* sink) {
    FileHeader fh;
    uint32_t magic;
    memcpy(&magic, data, 4);
    if (magic == 0xA1B2C3D4u || magic == 0xA1B23C4Du) {
        fh.swap = false;
    } else if (magic == 0xD4C3B2A1u || magic == 0x4D3CB2A1u) {
        fh.swap = true;
    } else {
        return RSS_ENOTSUP;
    }
    fh.linktype = rd32(data + 20, fh.swap) & 0x0FFFFFFF;
    if (!supported_linktype(fh.linktype)) return RSS_ENOTSUP;
    size_t pos = 24;
    while (pos + 16 <= len) {
        const uint32_t caplen = rd32(data + pos + 8, fh.swap);
        pos += 16;
        if (caplen > len - pos) break;  // truncated file: stop at the last whole record
        sink->packet(data + pos, caplen, fh.linktype);
        pos += caplen;
    }
    return RSS_OK;
}

// pcapng (IETF draft-ietf-opsawg-pcapng): blocks of [type u32][total length u32][body]
// [total length u32], byte order fixed per section by the Section Header Block's magic.
enum : uint32_t {
    PCAPNG_SHB = 0x0A0D0D0Au, PCAPNG_IDB = 1, PCAPNG_OPB = 2, PCAPNG_SPB = 3, PCAPNG_EPB = 6
};

int parse_pcapng(const uint8_t* data, size_t len, TupleSink* sink) {
    bool swap = false;
    std::vector<uint32_t> linktype, snaplen;  // per interface of the current section
    size_t pos = 0;
    bool first = true;
    while (pos + 12 <= len) {
        uint32_t type;
        memcpy(&type, data + pos, 4);  // the SHB type reads the same in both byte orders
        if (type == PCAPNG_SHB) {
            if (pos + 28 > len) break;
            uint32_t bom;
            memcpy(&bom, data + pos + 8, 4);
            if (bom == 0x1A2B3C4Du) swap = false;
            else if (bom == 0x4D3C2B1Au) swap = true;
            else return first ? RSS_ENOTSUP : RSS_OK;  // corrupt section: keep what we have
            linktype.clear();
            snaplen.clear();
        } else if (first) {
            return RSS_ENOTSUP;  // a pcapng image starts with a section header
        } else {
            type = rd32(data + pos, swap);
        }
        first = false;
        const uint32_t blen = rd32(data + pos + 4, swap);
        if (blen < 12 || (blen & 3) || blen > len - pos) break;  // truncated / corrupt: stop
        const uint8_t* body = data + pos + 8;
        const uint32_t body_len = blen - 12;
        if (type == PCAPNG_IDB) {
            if (body_len >= 8) {
                linktype.push_back(rd16(body, swap));
                snaplen.push_back(rd32(body + 4, swap));
            }
        } else if (type == PCAPNG_EPB || type == PCAPNG_OPB) {
            // EPB: if_id u32, ts u32 x2, caplen, origlen; OPB: if_id u16, drops u16, ...
            if (body_len >= 20) {
                const uint32_t ifc = type == PCAPNG_EPB ? rd32(body, swap) : rd16(body, swap);
                const uint32_t caplen = rd32(body + 12, swap);
                if (caplen > body_len - 20 || ifc >= linktype.size())
                    ++sink->skip;
                else
                    sink->packet(body + 20, caplen, linktype[ifc]);
            } else {
                ++sink->skip;
            }
        } else if (type == PCAPNG_SPB) {
            // original length u32, then the packet cut to interface 0's snap length
            if (body_len >= 4 && !linktype.empty()) {
                uint32_t caplen = rd32(body, swap);
                if (snaplen[0] && caplen > snaplen[0]) caplen = snaplen[0];
                if (caplen > body_len - 4) caplen = body_len - 4;
                sink->packet(body + 4, caplen, linktype[0]);
            } else {
                ++sink->skip;
            }
        }  // every other block (name resolution, statistics, custom, ...) is skipped
        pos += blen;
    }
    return RSS_OK;
}

}  // namespace

extern "C" {

int rss_pcap_parse(const uint8_t* data, size_t len, rss_tuple4* tuples, uint8_t* protocols,
                   size_t cap, size_t* n_out, size_t* skipped) {
    if (!data || !n_out) return RSS_EINVAL;
    *n_out = 0;
    if (skipped) *skipped = 0;
    if (len < 24) return RSS_ENOTSUP;
    TupleSink sink{tuples, protocols, cap};
    uint32_t magic;
    memcpy(&magic, data, 4);
    const int rc = magic == PCAPNG_SHB ? parse_pcapng(data, len, &sink)
                                       : parse_classic(data, len, &sink);
    if (rc) return rc;
    *n_out = sink.n;
    if (skipped) *skipped = sink.skip;
    return (tuples && sink.n > cap) ? RSS_EINVAL : RSS_OK;
}

int rss_pcap_parse6(const uint8_t* data, size_t len, rss_tuple6* tuples, uint8_t* protocols,
                    size_t cap, size_t* n_out, size_t* skipped) {
    if (!data || !n_out) return RSS_EINVAL;
    *n_out = 0;
    if (skipped) *skipped = 0;
    if (len < 24) return RSS_ENOTSUP;
    TupleSink sink{nullptr, protocols, cap};
    sink.tuples6 = tuples;
    sink.v6 = true;
    uint32_t magic;
    memcpy(&magic, data, 4);
    const int rc = magic == PCAPNG_SHB ? parse_pcapng(data, len, &sink)
                                       : parse_classic(data, len, &sink);
    if (rc) return rc;
    *n_out = sink.n;
    if (skipped) *skipped = sink.skip;
    return (tuples && sink.n > cap) ? RSS_EINVAL : RSS_OK;
}

}  // extern "C"

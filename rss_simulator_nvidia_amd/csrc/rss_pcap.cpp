// rss_pcap.cpp -- packet-capture input (the reference's planned
// "Use pcap as input", docs/rss_general_explaination.md:19).
//
// Reads a classic libpcap file image (either byte order, microsecond or nanosecond
// timestamps) and emits one packed IPv4 4-tuple per IPv4 packet, as a NIC's RSS unit
// would see it: TCP / UDP / SCTP packets contribute their ports, everything else
// (other protocols, and every fragment of a fragmented datagram) contributes ports 0,
// i.e. the 2-tuple hash.  Link types: Ethernet (with 802.1Q / 802.1ad tags), Linux
// cooked capture v1, raw IPv4.  Non-IPv4 and truncated packets are skipped and counted.
#include <cstring>

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

enum { DLT_EN10MB = 1, DLT_RAW = 101, DLT_LINUX_SLL = 113, DLT_IPV4 = 228 };

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
            if (caplen < 1) return false;
            *off = 0;
            *ethertype = (pkt[0] >> 4) == 4 ? 0x0800 : 0x86DD;
            return true;
        default:
            return false;
    }
}

}  // namespace

extern "C" {

int rss_pcap_parse(const uint8_t* data, size_t len, rss_tuple4* tuples, uint8_t* protocols,
                   size_t cap, size_t* n_out, size_t* skipped) {
    if (!data || !n_out) return RSS_EINVAL;
    *n_out = 0;
    if (skipped) *skipped = 0;
    if (len < 24) return RSS_ENOTSUP;
    FileHeader fh;
    uint32_t magic;
    memcpy(&magic, data, 4);
    if (magic == 0xA1B2C3D4u || magic == 0xA1B23C4Du) {
        fh.swap = false;
    } else if (magic == 0xD4C3B2A1u || magic == 0x4D3CB2A1u) {
        fh.swap = true;
    } else {
        return RSS_ENOTSUP;  // not a classic pcap file (pcapng is not supported)
    }
    fh.linktype = rd32(data + 20, fh.swap) & 0x0FFFFFFF;
    if (fh.linktype != DLT_EN10MB && fh.linktype != DLT_RAW && fh.linktype != DLT_LINUX_SLL &&
        fh.linktype != DLT_IPV4)
        return RSS_ENOTSUP;
    size_t pos = 24, n = 0, skip = 0;
    while (pos + 16 <= len) {
        const uint32_t caplen = rd32(data + pos + 8, fh.swap);
        pos += 16;
        if (caplen > len - pos) break;  // truncated file: stop at the last whole record
        const uint8_t* pkt = data + pos;
        pos += caplen;
        uint32_t off;
        uint16_t et;
        if (!link_payload(pkt, caplen, fh.linktype, &off, &et) || et != 0x0800 ||
            off + 20 > caplen || (pkt[off] >> 4) != 4) {
            ++skip;
            continue;
        }
        const uint8_t* ip = pkt + off;
        const uint32_t ihl = (uint32_t)(ip[0] & 15) * 4;
        if (ihl < 20 || off + ihl > caplen) {
            ++skip;
            continue;
        }
        const uint8_t proto = ip[9];
        const uint16_t frag = be16(ip + 6);
        const bool fragment = (frag & 0x2000) || (frag & 0x1FFF);  // MF or offset
        uint32_t ports = 0;
        if (!fragment && (proto == 6 || proto == 17 || proto == 132)) {
            if (off + ihl + 4 > caplen) {
                ++skip;
                continue;
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
    *n_out = n;
    if (skipped) *skipped = skip;
    return (tuples && n > cap) ? RSS_EINVAL : RSS_OK;
}

}  // extern "C"

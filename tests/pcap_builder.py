"""Synthetic classic-pcap and pcapng captures for the pcap tests (test infrastructure),
plus the expected tuples computed independently of the native parser."""
import struct

ETH_SRC, ETH_DST = b"\x02\x00\x00\x00\x00\x01", b"\x02\x00\x00\x00\x00\x02"


def ipv4(src, dst, proto, payload, frag=0, ihl_words=5):
    opts = b"\x01" * (4 * (ihl_words - 5))
    total = 4 * ihl_words + len(payload)
    hdr = struct.pack("!BBHHHBBH4s4s", 0x40 | ihl_words, 0, total, 1, frag, 64, proto, 0,
                      bytes(src), bytes(dst))
    return hdr + opts + payload


def ipv6(src, dst, next_header, payload, ext=()):
    """IPv6 packet: 16-byte addresses, optional extension headers ``ext`` = [(type, body)]
    (each body padded to the header's length unit), then ``payload``."""
    chain = [t for t, _ in ext] + [next_header]
    hdrs = b""
    for i, (t, body) in enumerate(ext):
        nxt = chain[i + 1]
        if t == 44:  # fragment header: fixed 8 bytes, body = (offset << 3 | M) as u16
            hdrs += struct.pack("!BBH4s", nxt, 0, body, b"\x00\x00\x00\x01")
        elif t == 51:  # AH: length in 4-octet units minus 2
            body += b"\x00" * (-(len(body) + 2) % 4)
            hdrs += struct.pack("!BB", nxt, (len(body) + 2) // 4 - 2) + body
        else:  # hop-by-hop / routing / destination options: 8-octet units minus 1
            body += b"\x00" * (-(len(body) + 2) % 8)
            hdrs += struct.pack("!BB", nxt, (len(body) + 2) // 8 - 1) + body
    first = chain[0]
    return struct.pack("!IHBB16s16s", 0x60000000, len(hdrs) + len(payload), first, 64,
                       bytes(src), bytes(dst)) + hdrs + payload


def l4(sport, dport, extra=16):
    return struct.pack("!HH", sport, dport) + b"\x00" * extra


def ether(payload, ethertype=0x0800, vlans=()):
    tags = b"".join(struct.pack("!HH", tpid, vid) for tpid, vid in vlans)
    return ETH_DST + ETH_SRC + tags + struct.pack("!H", ethertype) + payload


def sll(payload, ethertype=0x0800):
    return struct.pack("!HHH8sH", 0, 1, 6, b"\x02" * 8, ethertype) + payload


def pcap_file(packets, linktype=1, big_endian=False, nanos=False, truncate_last=0):
    e = ">" if big_endian else "<"
    magic = 0xA1B23C4D if nanos else 0xA1B2C3D4
    out = struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, 65535, linktype)
    for i, p in enumerate(packets):
        out += struct.pack(e + "IIII", i, 0, len(p), len(p)) + p
    return out[:len(out) - truncate_last] if truncate_last else out


def _block(e, btype, body):
    body += b"\x00" * (-len(body) % 4)
    total = 12 + len(body)
    return struct.pack(e + "II", btype, total) + body + struct.pack(e + "I", total)


def pcapng_section(packets, interfaces=((1, 65535),), big_endian=False, kinds=None,
                   extra_blocks=True):
    """One pcapng section: SHB, an IDB per (linktype, snaplen), then one packet block per
    entry of ``packets`` -- (interface, bytes) pairs or plain bytes for interface 0.
    ``kinds`` picks the block per packet: "epb" (default), "spb" or "opb"."""
    e = ">" if big_endian else "<"
    out = _block(e, 0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
    for lt, snap in interfaces:
        out += _block(e, 1, struct.pack(e + "HHI", lt, 0, snap))
    if extra_blocks:  # name resolution block + a custom block: both skipped
        out += _block(e, 4, struct.pack(e + "HH", 0, 0))
        out += _block(e, 0x00000BAD, b"\x01\x02\x03\x04\x05")
    for i, p in enumerate(packets):
        ifc, data = p if isinstance(p, tuple) else (0, p)
        kind = kinds[i] if kinds else "epb"
        if kind == "epb":
            out += _block(e, 6, struct.pack(e + "IIIII", ifc, 0, i, len(data), len(data)) + data)
        elif kind == "opb":
            out += _block(e, 2, struct.pack(e + "HHIIII", ifc, 0, 0, i, len(data), len(data)) + data)
        else:
            out += _block(e, 3, struct.pack(e + "I", len(data)) + data)
    if extra_blocks:  # interface statistics block after the packets
        out += _block(e, 5, struct.pack(e + "III", 0, 0, 0))
    return out

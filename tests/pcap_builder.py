"""Synthetic classic-pcap captures for the pcap tests (test infrastructure), plus the
expected tuples computed independently of the native parser."""
import struct

ETH_SRC, ETH_DST = b"\x02\x00\x00\x00\x00\x01", b"\x02\x00\x00\x00\x00\x02"


def ipv4(src, dst, proto, payload, frag=0, ihl_words=5):
    opts = b"\x01" * (4 * (ihl_words - 5))
    total = 4 * ihl_words + len(payload)
    hdr = struct.pack("!BBHHHBBH4s4s", 0x40 | ihl_words, 0, total, 1, frag, 64, proto, 0,
                      bytes(src), bytes(dst))
    return hdr + opts + payload


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

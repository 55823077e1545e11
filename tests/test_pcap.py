"""pcap input (row f4), host side: the native parser against captures built by
tests/pcap_builder.py with known tuples; flow de-duplication; L4 selection; the CLI
(device call replaced by the oracle).  The capture format is new to this build (the
reference only plans it), so parsing parity is against the constructed expectations;
the hashes of the extracted tuples are pinned like every other input."""
import os

import pytest

from oracle import oracle as o
from pcap_builder import ether, ipv4, l4, pcap_file, pcapng_section, sll
from rss_simulator_nvidia_amd import _native, pcap
from rss_simulator_nvidia_amd.main import main
from test_cli_host import OracleContext

A, B, C = (10, 0, 0, 1), (192, 168, 1, 20), (8, 8, 8, 8)


def u32(ip):
    return ip[0] << 24 | ip[1] << 16 | ip[2] << 8 | ip[3]


def packets_and_expected():
    pk, want = [], []
    pk.append(ether(ipv4(A, B, 6, l4(1234, 80))))                      # TCP
    want.append((u32(A), u32(B), 1234 << 16 | 80, 6))
    pk.append(ether(ipv4(B, A, 17, l4(53, 40000)), vlans=[(0x8100, 7)]))  # UDP, VLAN
    want.append((u32(B), u32(A), 53 << 16 | 40000, 17))
    pk.append(ether(ipv4(A, C, 1, b"\x08\x00" + b"\x00" * 30)))        # ICMP: ports 0
    want.append((u32(A), u32(C), 0, 1))
    pk.append(ether(ipv4(A, B, 17, l4(1, 2), frag=0x2000)))            # first fragment
    want.append((u32(A), u32(B), 0, 17))
    pk.append(ether(ipv4(A, B, 17, b"\x00" * 8, frag=0x0010)))         # later fragment
    want.append((u32(A), u32(B), 0, 17))
    pk.append(ether(ipv4(C, A, 132, l4(9, 10)), vlans=[(0x88A8, 1), (0x8100, 2)]))  # SCTP QinQ
    want.append((u32(C), u32(A), 9 << 16 | 10, 132))
    pk.append(ether(ipv4(A, B, 6, l4(5, 6), ihl_words=7)))             # IP options
    want.append((u32(A), u32(B), 5 << 16 | 6, 6))
    pk.append(ether(b"\x60" + b"\x00" * 60, ethertype=0x86DD))         # IPv6: skipped
    pk.append(ether(b"\x00" * 28, ethertype=0x0806))                   # ARP: skipped
    pk.append(ether(ipv4(A, B, 6, b"\x00\x01")))                       # truncated TCP: skipped
    pk.append(ether(ipv4(A, B, 6, l4(1234, 80))))                      # duplicate flow
    want.append((u32(A), u32(B), 1234 << 16 | 80, 6))
    return pk, want, 3


def as_rows(tuples, protos):
    return [(int(t["sip"]), int(t["dip"]), int(t["ports"]), int(p)) for t, p in zip(tuples, protos)]


@pytest.mark.parametrize("big_endian,nanos", [(False, False), (True, False), (False, True)])
def test_parse_ethernet(big_endian, nanos):
    pk, want, skipped = packets_and_expected()
    got = _native.pcap_parse(pcap_file(pk, big_endian=big_endian, nanos=nanos))
    assert got is not None
    assert as_rows(got[0], got[1]) == want and got[2] == skipped


def test_parse_cooked_and_raw():
    pk = [sll(ipv4(A, B, 17, l4(7, 8))), sll(b"\x00" * 40, ethertype=0x86DD)]
    t, p, s = _native.pcap_parse(pcap_file(pk, linktype=113))
    assert as_rows(t, p) == [(u32(A), u32(B), 7 << 16 | 8, 17)] and s == 1
    for lt in (101, 228):
        t, p, s = _native.pcap_parse(pcap_file([ipv4(C, B, 6, l4(1, 2))], linktype=lt))
        assert as_rows(t, p) == [(u32(C), u32(B), 1 << 16 | 2, 6)] and s == 0


def test_truncated_file_and_non_pcap():
    pk, want, _ = packets_and_expected()
    t, p, _ = _native.pcap_parse(pcap_file(pk, truncate_last=5))
    assert as_rows(t, p) == want[:-1]
    assert _native.pcap_parse(b"src_ip,dst_ip,src_port,dst_port\n" * 3) is None
    assert _native.pcap_parse(b"\x0a\x0d\x0d\x0a" + b"\x00" * 40) is None  # bad pcapng magic
    assert _native.pcap_parse(pcap_file(pk, linktype=147)) is None


def test_read_flows_unique_and_l4(tmp_path):
    pk, want, _ = packets_and_expected()
    path = tmp_path / "c.pcap"
    path.write_bytes(pcap_file(pk))
    t, p, s = pcap.read_flows(str(path))
    uniq = []
    for w in want:
        if w[:3] not in [u[:3] for u in uniq]:
            uniq.append(w)
    assert [r[:3] for r in as_rows(t, p)] == [u[:3] for u in uniq]
    t, p, _ = pcap.read_flows(str(path), "udp")
    rows = as_rows(t, p)
    assert all(r[2] == 0 for r in rows if r[3] != 17)
    assert (u32(B), u32(A), 53 << 16 | 40000, 17) in rows
    with pytest.raises(ValueError):
        pcap.parse_l4("icmp")


@pytest.mark.parametrize("fields", ["sdfn", "sd"])
def test_cli_pcap_csv(fields, tmp_path, monkeypatch, oracle_lib, golden_dir, capsys):
    monkeypatch.setattr(_native, "default_context", lambda: OracleContext(oracle_lib))
    pk, _, _ = packets_and_expected()
    path = tmp_path / "c.pcap"
    path.write_bytes(pcap_file(pk))
    out = tmp_path / "out.csv"
    key_file = os.path.join(golden_dir, "example_input", "hash_key.txt")
    main(["--key-file", key_file, "--ips-file", str(path), "--pcap", "--htable-size", "128",
          "--num-queues", "24", "--csv", str(out), "--hash-fields", fields])
    assert capsys.readouterr().out == "Wrote statistics to %s.\n" % out
    key = [int(x, 16) for x in open(key_file).read().split(":")]
    t, _, _ = pcap.read_flows(str(path))
    mask = _native.parse_fields(fields)
    want_h = [oracle_lib.hash_bytes(key, o.select_fields_bytes(r["sip"], r["dip"], r["ports"], mask))
              for r in t]
    lines = out.read_text().splitlines()
    body = lines[lines.index("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number") + 1:]
    assert [int(x.split(",")[4]) for x in body] == want_h
    assert [int(x.split(",")[5]) for x in body] == [h % 128 % 24 for h in want_h]
    assert body[0].startswith("10.0.0.1,192.168.1.20,1234,80,")


@pytest.mark.parametrize("big_endian", [False, True])
def test_pcapng_matches_classic(big_endian):
    """The same packets as enhanced packet blocks of a pcapng section (with name-resolution,
    custom and statistics blocks to skip) parse exactly as the classic capture does."""
    pk, want, skipped = packets_and_expected()
    got = _native.pcap_parse(pcapng_section(pk, big_endian=big_endian))
    assert got is not None
    assert as_rows(got[0], got[1]) == want and got[2] == skipped


def test_pcapng_interfaces_blocks_and_sections():
    """Per-interface link types (Ethernet, cooked, raw, and an unsupported one whose
    packets are skipped), simple / obsolete packet blocks, SPB cut to the snap length,
    a second section of the other byte order, and a truncated last block."""
    p_eth = ether(ipv4(A, B, 6, l4(1, 2)))
    p_sll = sll(ipv4(B, C, 17, l4(3, 4)))
    p_raw = ipv4(C, A, 6, l4(5, 6))
    ifaces = ((1, 65535), (113, 65535), (101, 65535), (147, 65535))
    sec1 = pcapng_section([(0, p_eth), (1, p_sll), (2, p_raw), (3, p_eth), (9, p_eth)],
                          interfaces=ifaces)
    want1 = [(u32(A), u32(B), 1 << 16 | 2, 6), (u32(B), u32(C), 3 << 16 | 4, 17),
             (u32(C), u32(A), 5 << 16 | 6, 6)]
    # section 2 (big endian): SPB + OPB on one Ethernet interface; snap length 34 cuts
    # the SPB packet inside its TCP header (ports unreadable -> skipped)
    sec2 = pcapng_section([p_eth, p_eth, p_eth], interfaces=((1, 34),), big_endian=True,
                          kinds=["spb", "opb", "epb"])
    got = _native.pcap_parse(sec1 + sec2)
    assert as_rows(got[0], got[1]) == want1 + [(u32(A), u32(B), 1 << 16 | 2, 6)] * 2
    assert got[2] == 3  # unsupported link type, unknown interface 9, cut SPB packet
    sec2_bare = pcapng_section([p_eth, p_eth, p_eth], interfaces=((1, 34),), big_endian=True,
                               kinds=["spb", "opb", "epb"], extra_blocks=False)
    cut = _native.pcap_parse(sec1 + sec2_bare[:-7])  # last packet block truncated: dropped
    assert as_rows(cut[0], cut[1]) == want1 + [(u32(A), u32(B), 1 << 16 | 2, 6)]


def test_read_flows_pcapng(tmp_path):
    pk, want, _ = packets_and_expected()
    path = tmp_path / "c.pcapng"
    path.write_bytes(pcapng_section(pk))
    tuples, protos, skipped = pcap.read_flows(str(path))
    assert len(tuples) == len(set(want)) and skipped == 3


S6 = bytes.fromhex("20010db8000000000000000000000001")
D6 = bytes.fromhex("20010db8000000000000000000000002")
E6 = bytes.fromhex("fe800000000000000211223344556677")


def w6(addr):
    return tuple(int.from_bytes(addr[i:i + 4], "big") for i in range(0, 16, 4))


def packets6_and_expected():
    """IPv6 packets with extension-header chains and the tuples a NIC's RSS unit hashes."""
    from pcap_builder import ipv6
    pk, want = [], []

    def add(pkt, src, dst, ports, proto):
        pk.append(pkt)
        if src is not None:
            want.append(w6(src) + w6(dst) + (ports, proto))

    add(ether(ipv6(S6, D6, 6, l4(1000, 443)), ethertype=0x86DD), S6, D6, 1000 << 16 | 443, 6)
    add(ether(ipv6(D6, S6, 17, l4(53, 5353), ext=[(0, b"\x01\x00" * 2), (60, b"\x00" * 10)]),
              ethertype=0x86DD), D6, S6, 53 << 16 | 5353, 17)                    # HBH + dst opts
    add(ether(ipv6(S6, E6, 6, l4(7, 8), ext=[(43, b"\x00" * 22)]), ethertype=0x86DD),
        S6, E6, 7 << 16 | 8, 6)                                                  # routing header
    add(ether(ipv6(S6, D6, 17, l4(1, 2), ext=[(44, 0x0001)]), ethertype=0x86DD),
        S6, D6, 0, 17)                                                           # first fragment
    add(ether(ipv6(S6, D6, 17, b"\x00" * 16, ext=[(44, 185 << 3)]), ethertype=0x86DD),
        S6, D6, 0, 17)                                                           # later fragment
    add(ether(ipv6(E6, D6, 6, l4(9, 10), ext=[(44, 0)]), ethertype=0x86DD),
        E6, D6, 9 << 16 | 10, 6)                                                 # atomic fragment
    add(ether(ipv6(S6, D6, 132, l4(11, 12), ext=[(51, b"\x00" * 10)]), ethertype=0x86DD),
        S6, D6, 11 << 16 | 12, 132)                                              # AH + SCTP
    add(ether(ipv6(S6, D6, 50, b"\x00" * 24), ethertype=0x86DD), S6, D6, 0, 50)  # ESP
    add(ether(ipv6(D6, E6, 58, b"\x80\x00" + b"\x00" * 10), ethertype=0x86DD),
        D6, E6, 0, 58)                                                           # ICMPv6
    add(ether(ipv6(S6, D6, 17, l4(3, 4)), ethertype=0x86DD, vlans=[(0x8100, 9)]),
        S6, D6, 3 << 16 | 4, 17)                                                 # VLAN
    add(ether(ipv4(A, B, 6, l4(1234, 80))), None, None, 0, 0)                    # IPv4: skipped
    add(ether(ipv6(S6, D6, 6, b"\x00\x01"), ethertype=0x86DD), None, None, 0, 0)  # cut TCP: skip
    add(ether(ipv6(S6, D6, 6, l4(1, 2), ext=[(0, b"\x00" * 40)])[:60], ethertype=0x86DD),
        None, None, 0, 0)                                                        # cut ext hdr
    add(ether(ipv6(S6, D6, 6, l4(1000, 443)), ethertype=0x86DD), S6, D6, 1000 << 16 | 443, 6)
    return pk, want, 3


def as_rows6(tuples, protos):
    return [tuple(int(x) for x in t["sip"]) + tuple(int(x) for x in t["dip"]) +
            (int(t["ports"]), int(p)) for t, p in zip(tuples, protos)]


@pytest.mark.parametrize("fmt", ["pcap", "pcapng", "pcapng_be"])
def test_parse_ipv6(fmt):
    pk, want, skipped = packets6_and_expected()
    img = pcap_file(pk) if fmt == "pcap" else pcapng_section(pk, big_endian=fmt == "pcapng_be")
    t, p, s = _native.pcap_parse(img, ipv6=True)
    assert as_rows6(t, p) == want and s == skipped
    # the IPv4 view of the same capture sees only the one IPv4 packet
    t4, _, s4 = _native.pcap_parse(img)
    assert len(t4) == 1 and s4 == len(pk) - 1


def test_parse_ipv6_raw_link_types():
    from pcap_builder import ipv6
    pkt = ipv6(S6, D6, 17, l4(5, 6))
    for lt in (101, 229):
        t, p, s = _native.pcap_parse(pcap_file([pkt, ipv4(A, B, 6, l4(1, 2))], linktype=lt),
                                     ipv6=True)
        assert as_rows6(t, p) == [w6(S6) + w6(D6) + (5 << 16 | 6, 17)] and s == 1


def test_cli_pcap_ipv6_csv(tmp_path, monkeypatch, oracle_lib, golden_dir, capsys):
    """--pcap --ipv6: unique IPv6 flows hashed with the 36-byte input; the CSV carries
    RFC 5952 addresses; hashes follow the oracle's literal loop over the 36 bytes."""
    monkeypatch.setattr(_native, "default_context", lambda: OracleContext(oracle_lib))
    pk, want, _ = packets6_and_expected()
    path = tmp_path / "c6.pcapng"
    path.write_bytes(pcapng_section(pk))
    out = tmp_path / "out6.csv"
    key_file = os.path.join(golden_dir, "example_input", "hash_key.txt")
    main(["--key-file", key_file, "--ips-file", str(path), "--pcap", "--ipv6",
          "--htable-size", "128", "--num-queues", "24", "--csv", str(out)])
    assert capsys.readouterr().out == "Wrote statistics to %s.\n" % out
    key = [int(x, 16) for x in open(key_file).read().split(":")]
    uniq = list(dict.fromkeys(r[:9] for r in want))
    want_h = [oracle_lib.hash_bytes(key, b"".join(int(w).to_bytes(4, "big") for w in r))
              for r in uniq]
    lines = out.read_text().splitlines()
    body = lines[lines.index("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number") + 1:]
    assert [int(x.split(",")[4]) for x in body] == want_h
    assert [int(x.split(",")[5]) for x in body] == [h % 128 % 24 for h in want_h]
    assert body[0] == "2001:db8::1,2001:db8::2,1000,443,%d,%d" % (want_h[0], want_h[0] % 128 % 24)
    counts = {}
    for h in want_h:
        counts[h % 128 % 24] = counts.get(h % 128 % 24, 0) + 1
    assert lines[1:1 + len(counts)] == ["%d,%d" % (q, counts[q]) for q in sorted(counts)]

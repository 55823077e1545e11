"""pcap input (the reference's planned "Use pcap as input",
``docs/rss_general_explaination.md:19``).

``read_flows`` turns a capture into the flow list the simulator hashes: one 4-tuple
per IPv4 packet (``rss_pcap_parse``), optionally restricted to the L4 protocols whose
ports take part in the hash (ethtool ``rx-flow-hash`` style: e.g. only UDP -- the
reference's "Only on UDPs"), then de-duplicated to unique flows in first-seen
order, the unit the reference's histogram counts ("Number of Unique Flows per
Queue", ``simulator.py:152``).
"""
import ipaddress

import numpy as np

from rss_simulator_nvidia_amd import _native
from rss_simulator_nvidia_amd.exceptions import ParseException

PROTOCOLS = {"tcp": 6, "udp": 17, "sctp": 132}


def parse_l4(spec):
    """'tcp,udp' -> {6, 17}; 'none' -> set()."""
    if spec in (None, "", "all"):
        return set(PROTOCOLS.values())
    if spec == "none":
        return set()
    try:
        return {PROTOCOLS[p] for p in spec.split(",")}
    except KeyError:
        raise ValueError("L4 protocols must be a comma list of tcp, udp, sctp (or none)")


def read_flows(path, l4=None, unique=True, ipv6=False):
    """Packed tuples of a capture's IPv4 packets (``TUPLE_DTYPE``), or with ``ipv6`` of its
    IPv6 packets (``TUPLE6_DTYPE``) -> (tuples, protocols, skipped packets)."""
    try:
        data = np.fromfile(path, dtype=np.uint8)
    except OSError as err:
        raise ParseException("Couldn't read pcap file %s: %s" % (path, err))
    parsed = _native.pcap_parse(data, ipv6=ipv6)
    if parsed is None:
        raise ParseException("%s is not a pcap or pcapng file" % path)
    tuples, protos, skipped = parsed
    keep = parse_l4(l4)
    if keep != set(PROTOCOLS.values()):
        tuples = tuples.copy()
        tuples["ports"][~np.isin(protos, list(keep))] = 0
    if unique and len(tuples):
        raw = np.ascontiguousarray(tuples).view(np.dtype((np.void, tuples.dtype.itemsize)))
        _, first = np.unique(raw, return_index=True)
        order = np.sort(first)
        tuples, protos = tuples[order], protos[order]
    return tuples, protos, skipped


def _ip6_text(words):
    """Four host-order words (big-endian-valued) -> RFC 5952 text (``ipaddress``)."""
    return str(ipaddress.IPv6Address(b"".join(int(w).to_bytes(4, "big") for w in words)))


def format_statistics6(tuples6, hashes, queues, counts):
    """``write_statistics``' file (``simulator.py:100-116``) for IPv6 flows: the
    ``queue_number,counts`` rows of the non-empty queues, then the table with the
    addresses in RFC 5952 text."""
    lines = ["queue_number,counts"]
    lines += ["%d,%d" % (q, c) for q, c in enumerate(counts) if c]
    lines.append("src_ip,dst_ip,src_port,dst_port,hash_result,queue_number")
    for t, h, q in zip(tuples6, hashes, queues):
        p = int(t["ports"])
        lines.append("%s,%s,%d,%d,%d,%d" % (_ip6_text(t["sip"]), _ip6_text(t["dip"]), p >> 16,
                                            p & 0xFFFF, h, q))
    return "\n".join(lines) + "\n"

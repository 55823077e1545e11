"""``rss-simulator`` command line -- drop-in for ``rss_simulator/main.py``.

Same five flags, metavars, help texts, validation and exit codes as the
reference (``main.py:10-64``): ``--key-file`` is parsed eagerly (bad key ->
argparse error, exit 2), ``--htable-size`` / ``--num-queues`` must be >= 1,
``--csv PATH`` writes statistics, otherwise the histogram is shown.  Canonical CSVs
take the native parse/format fast path (``fastcsv.py``); everything else the
pandas path of ``Simulator``.
"""
import argparse
from argparse import ArgumentParser

from rss_simulator_nvidia_amd import _native, fastcsv, histogram, pcap, reta
from rss_simulator_nvidia_amd.arg_parse_types import PositiveInt
from rss_simulator_nvidia_amd.arg_parse_types import arg_parse_type_decorator as apt_decorator
from rss_simulator_nvidia_amd.exceptions import ParseException
from rss_simulator_nvidia_amd.hash_key import HashKey

# simulator.py (pandas, ~0.4 s to import) is imported only when the pandas path runs:
# canonical files never need it


def _key_str(key):
    """``Toeplitz.hash_key_str()`` (toeplitz.py:37-44) without importing the pandas path."""
    return ":".join("{:02x}".format(b) for b in key)


def _fields_arg(text):
    _native.parse_fields(text)
    return text


def _l4_arg(text):
    pcap.parse_l4(text)
    return text


def indirection_table(args):
    """The --reta-weights / --reta-file table, validated, or None (reference mapping).
    Raises ValueError (``main`` reports it as a usage error, exit status 2)."""
    if args.reta_weights is not None and args.reta_file is not None:
        raise ValueError("give either --reta-weights or --reta-file")
    if args.reta_weights is None and args.reta_file is None:
        return None
    if args.htable_size > reta.MAX_ENTRIES:  # before a table of htable entries is built
        raise ValueError("indirection tables hold at most %d entries, --htable-size is %d"
                         % (reta.MAX_ENTRIES, args.htable_size))
    if args.reta_weights is not None:
        if len(args.reta_weights) != args.num_queues:
            raise ValueError("--reta-weights needs one weight per queue (%d)" % args.num_queues)
        table = reta.weights(args.htable_size, args.reta_weights)
    elif args.reta_file is not None:
        table = args.reta_file
    else:
        return None
    return reta.validate(table, args.htable_size, args.num_queues)


def run_pcap(args, table):
    """--pcap: unique IPv4 (or, with --ipv6, IPv6) flows of a capture -> the same kernels
    -> CSV or histogram."""
    tuples, _, _ = pcap.read_flows(args.ips_file, args.pcap_l4, ipv6=args.ipv6)
    if len(tuples) == 0:
        raise ParseException("%s holds no %s packets" % (args.ips_file,
                                                          "IPv6" if args.ipv6 else "IPv4"))
    ctx = _native.default_context()
    if args.ipv6:
        key6 = _native.prepare_key6(args.key, args.hash_fields)
        h, q, c = ctx.hash6(key6, tuples, args.htable_size, args.num_queues, reta=table)
    else:
        key = _native.prepare_key(args.key, args.hash_fields)
        h, q, c = ctx.hash(key, tuples, args.htable_size, args.num_queues, reta=table)
    key_str = _key_str(args.key)
    if args.csv:
        if args.ipv6:
            with open(args.csv, "w") as f:
                f.write(pcap.format_statistics6(tuples, h, q, c))
        else:
            out = _native.csv_format(tuples, h, q, c, _native.RssCsvLayout((0, 1, 2, 3)))
            out.tofile(args.csv)
        print("Wrote statistics to {csv}.".format(csv=args.csv))
    else:
        histogram.show(c, key_str, args.htable_size, args.num_queues, args.histogram_png)


def build_parser():
    """The reference's ArgumentParser (``main.py:17-50``)."""
    parser = ArgumentParser(
        prog="rss-simulator",
        description="Simulate Nvidia's NIC RSS queue's distribution for Toeplitz hash function.",
    )
    parser.add_argument("--key-file", metavar="PATH", dest="key",
                        type=apt_decorator(HashKey.from_file), required=True,
                        help="File containing 40B hash key.")
    parser.add_argument("--ips-file", metavar="PATH", required=True,
                        help="csv containing source/destination IP and source/destination ports "
                             "4 tupels entries.")
    parser.add_argument("--htable-size", metavar="NUM", type=PositiveInt.parse, required=True,
                        help="Positive number representing the hash-table size.")
    parser.add_argument("--num-queues", metavar="NUM", type=PositiveInt.parse, required=True,
                        help="Positive number representing number of queues.")
    parser.add_argument("--csv", metavar="PATH", help="Write output to csv file.")
    # Additive options (not in the reference).  They are
    # kept out of usage/--help so the reference's argparse messages stay byte-identical:
    #   --histogram-png PATH  save the histogram instead of opening a window
    #   --hash-fields FIELDS  hashed fields, ethtool letters: s src ip, d dst ip,
    #                         f src port, n dst port (default sdfn = whole 4-tuple)
    #   --ipv6                address columns hold IPv6 addresses (36-byte input)
    parser.add_argument("--histogram-png", metavar="PATH", help=argparse.SUPPRESS)
    parser.add_argument("--hash-fields", metavar="FIELDS", default="sdfn",
                        type=apt_decorator(_fields_arg), help=argparse.SUPPRESS)
    parser.add_argument("--ipv6", action="store_true", help=argparse.SUPPRESS)
    #   --pcap                --ips-file is a pcap / pcapng capture (unique IPv4 flows;
    #                         with --ipv6 its unique IPv6 flows)
    #   --pcap-l4 LIST        protocols whose ports are hashed (tcp,udp,sctp | none)
    parser.add_argument("--pcap", action="store_true", help=argparse.SUPPRESS)
    parser.add_argument("--pcap-l4", metavar="LIST", default="all",
                        type=apt_decorator(_l4_arg), help=argparse.SUPPRESS)
    #   --reta-weights W,..   ethtool -X weight table over --htable-size buckets
    #   --reta-file PATH      explicit indirection table (one queue id per bucket)
    parser.add_argument("--reta-weights", metavar="W,...", type=apt_decorator(reta.parse_weights),
                        help=argparse.SUPPRESS)
    parser.add_argument("--reta-file", metavar="PATH", type=apt_decorator(reta.load),
                        help=argparse.SUPPRESS)
    return parser


def parse_args(argv=None):
    """Parse script arguments (``main.py:10-51``)."""
    return build_parser().parse_args(argv)


def main(argv=None):
    """Invoke the RSS simulator (``main.py:54-64``)."""
    parser = build_parser()
    args = parser.parse_args(argv)
    try:
        table = indirection_table(args)
        # --csv with htable and num-queues both >= 2**32: queue = hash (simulator.py:97), the
        # Simulator path counts those queues sparsely; histogram mode would need 2**32+ bins
        hashes_are_queues = args.csv and _native.queues_are_hashes(args.htable_size,
                                                                   args.num_queues, table)
        if not hashes_are_queues:
            _native.queue_modulus(args.htable_size, args.num_queues, table is not None)
    except ValueError as err:
        parser.error(str(err))
    if args.pcap:
        return run_pcap(args, table)
    fast = fastcsv.enabled() and not hashes_are_queues
    run_csv = fastcsv.run_csv6 if args.ipv6 else fastcsv.run_csv
    run_counts = fastcsv.run_counts6 if args.ipv6 else fastcsv.run_counts
    if args.csv and fast and run_csv(args.key, args.ips_file, args.htable_size, args.num_queues,
                                     args.csv, fields=args.hash_fields, reta=table):
        return  # canonical input: native CSV parse/format around the same GPU kernel
    if not args.csv and fast:
        counts = run_counts(args.key, args.ips_file, args.htable_size, args.num_queues,
                            fields=args.hash_fields, reta=table)
        if counts is not None:  # histogram mode needs the per-queue counts only
            histogram.show(counts, _key_str(args.key), args.htable_size,
                           args.num_queues, args.histogram_png)
            return
    from rss_simulator_nvidia_amd.simulator import Simulator
    rss_sim = Simulator(args.key, args.htable_size, args.num_queues, args.hash_fields, args.ipv6,
                        table)
    rss_sim.load_ips_from_csv(args.ips_file)
    rss_sim.calc_hash()
    rss_sim.calc_queue_number()
    if args.csv:
        rss_sim.write_statistics(args.csv)
    else:
        rss_sim.show_histogram(args.histogram_png)

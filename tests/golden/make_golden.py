"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

This script is the only place that touches /root/reference, and it runs only in the
build container (the reference never travels to the GPU box).  It imports the
reference read-only (PYTHONDONTWRITEBYTECODE=1) with one harness-side compat shim:
``rss_simulator/simulator.py:23`` references ``matplotlib.cbook.mplDeprecation``,
which matplotlib >= 3.8 removed, so the shim re-creates that attribute before import.

Fixtures written (all data; no reference source is copied):

* ``example/out_h{H}_q{Q}.csv``  -- the reference CLI's ``--csv`` output on
  ``example_input/`` (F1); ``example/stdout.json`` holds the stdout lines.
* ``ms_kat.json``                -- Microsoft RSS verification-suite IPv4/TCP vectors
  as computed by ``Toeplitz.compute_hash`` (F2).
* ``random_tuples.npz``          -- 4096 random tuples x 4 keys -> hash_result (F3),
  plus queue columns / per-queue counts from ``Simulator`` for the sweep configs (F5).
* ``one_hot.npz``                -- the 96 one-hot inputs + all-zero + all-ones (F4).
* ``edge/*.csv`` + ``edge_cases.json`` -- CLI edge cases (F4): inputs, exit codes,
  stdout, last stderr line and output CSV bytes.
* ``histogram.json``             -- histogram mode (``show_histogram``) with ``plt.show``
  patched out: bar heights / positions, caption text, title and axis labels.

Run:  PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden.py
"""
import json
import os
import random
import subprocess
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

SHIM = (
    "import matplotlib, matplotlib.cbook\n"
    "matplotlib.use('Agg')\n"
    "matplotlib.cbook.mplDeprecation = matplotlib.MatplotlibDeprecationWarning\n"
    "import sys\n"
    "sys.path.insert(0, %r)\n" % REF
)

MS_KEY = "6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa"
MS_VECTORS = [
    ("66.9.149.187", "161.142.100.80", 2794, 1766),
    ("199.92.111.2", "65.69.140.83", 14230, 4739),
    ("24.19.198.95", "12.22.207.184", 12898, 38024),
    ("38.27.205.30", "209.142.163.6", 48228, 2217),
    ("153.39.163.191", "202.188.127.2", 44251, 1303),
]
SWEEP = [(h, q) for h in (128, 512) for q in (8, 16, 24, 64)] + [(100, 7), (1000, 3), (1, 1), (65536, 1000)]


def assert_reference_module(mod, ref=REF):
    """Refuse to generate anything unless ``mod`` was imported from the reference tree.

    This repository ships its own ``rss_simulator`` import shim (a re-export of the build):
    a path mishap that imported it instead would make every fixture a self-comparison."""
    path = os.path.realpath(getattr(mod, "__file__", "") or "")
    root = os.path.realpath(ref) + os.sep
    if not path.startswith(root):
        raise RuntimeError("golden generator: %s was imported from %r, not from the reference "
                           "tree %r; refusing to generate fixtures" % (mod.__name__, path, root))
    return path


# the same check inside every CLI subprocess (run_cli), before the reference's main runs
GUARD_EXIT = 97
CLI_GUARD = ("import os, rss_simulator\n"
             "if not os.path.realpath(rss_simulator.__file__).startswith("
             "os.path.realpath(%r) + os.sep):\n"
             "    sys.stderr.write('golden generator guard: rss_simulator from %%s\\n' %% "
             "rss_simulator.__file__)\n"
             "    sys.exit(%d)\n" % (REF, GUARD_EXIT))


def import_reference():
    env_ns = {}
    exec(SHIM, env_ns)
    import rss_simulator  # noqa: E402
    from rss_simulator import hash_key, simulator, toeplitz  # noqa: E402
    for mod in (rss_simulator, toeplitz, simulator, hash_key):
        assert_reference_module(mod)
    return toeplitz.Toeplitz, simulator.Simulator, hash_key.HashKey


def ip_str(n):
    return "%d.%d.%d.%d" % ((n >> 24) & 255, (n >> 16) & 255, (n >> 8) & 255, n & 255)


def key_text(kb):
    return ":".join("%02x" % b for b in kb)


def run_cli(args, cwd):
    code = (SHIM + CLI_GUARD +
            "sys.argv = ['rss-simulator'] + %r\nfrom rss_simulator import main\nmain()\n" % (args,))
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg")
    p = subprocess.run([sys.executable, "-c", code], cwd=cwd, capture_output=True, text=True, env=env)
    if p.returncode == GUARD_EXIT and "golden generator guard" in p.stderr:
        raise RuntimeError(p.stderr.strip())
    if "Traceback" not in p.stderr:
        return p.returncode, p.stdout, p.stderr  # argparse usage errors: keep them whole
    err_lines = [ln for ln in p.stderr.strip().splitlines() if ln.strip()]
    return p.returncode, p.stdout, err_lines[-1]


def gen_example():
    outdir = os.path.join(HERE, "example")
    os.makedirs(outdir, exist_ok=True)
    stdout = {}
    for h, q in [(128, 24), (100, 7)] + [(h, q) for h in (128, 512) for q in (8, 16, 24, 64)]:
        name = "out_h%d_q%d.csv" % (h, q)
        out = os.path.join(outdir, name)
        if os.path.exists(out):
            os.remove(out)
        rc, so, err = run_cli(["--key-file", os.path.join(HERE, "example_input/hash_key.txt"),
                               "--ips-file", os.path.join(HERE, "example_input/ips.csv"),
                               "--htable-size", str(h), "--num-queues", str(q), "--csv", out], HERE)
        assert rc == 0, (rc, err)
        stdout[name] = so.replace(out, "{csv}")
    with open(os.path.join(outdir, "stdout.json"), "w") as f:
        json.dump(stdout, f, indent=1, sort_keys=True)


def gen_kat(Toeplitz):
    key = [int(MS_KEY[i:i + 2], 16) for i in range(0, 80, 2)]
    t = Toeplitz(key)
    vecs = []
    for s, d, sp, dp in MS_VECTORS:
        # "hash_ip_only": the reference with both ports 0 = the 8-byte (src, dst) input,
        # the verification suite's "IPv4 only" column
        vecs.append({"src_ip": s, "dst_ip": d, "src_port": sp, "dst_port": dp,
                     "hash": t.compute_hash(s, d, sp, dp),
                     "hash_ip_only": t.compute_hash(s, d, 0, 0)})
    with open(os.path.join(HERE, "ms_kat.json"), "w") as f:
        json.dump({"key": key_text(key), "vectors": vecs}, f, indent=1)


def gen_random(Toeplitz, Simulator):
    rng = random.Random(0x5EED)
    n = 4096
    sip = np.array([rng.getrandbits(32) for _ in range(n)], dtype=np.uint32)
    dip = np.array([rng.getrandbits(32) for _ in range(n)], dtype=np.uint32)
    # ports drawn from 17 bits so that the reference's 16-bit truncation is exercised
    sport = np.array([rng.getrandbits(17) for _ in range(n)], dtype=np.int64)
    dport = np.array([rng.getrandbits(17) for _ in range(n)], dtype=np.int64)
    ex_key = [int(x, 16) for x in open(os.path.join(HERE, "example_input/hash_key.txt")).read().split(":")]
    ms_key = [int(MS_KEY[i:i + 2], 16) for i in range(0, 80, 2)]
    rnd_key = rng.sample(range(256), 40)  # the shape HashKey.random_hash_key() produces
    long_key = [rng.getrandbits(8) for _ in range(52)]
    keys = [ex_key, ms_key, rnd_key, long_key]
    key_arr = np.zeros((4, 52), dtype=np.uint8)
    key_len = np.zeros(4, dtype=np.int32)
    hashes = np.zeros((4, n), dtype=np.uint32)
    for k, key in enumerate(keys):
        key_arr[k, :len(key)] = key
        key_len[k] = len(key)
        t = Toeplitz(list(key))
        for i in range(n):
            hashes[k, i] = t.compute_hash(ip_str(int(sip[i])), ip_str(int(dip[i])), int(sport[i]), int(dport[i]))
        print("key", k, "done", flush=True)

    # F5: queue columns + per-queue counts through the reference Simulator (pandas path)
    csv_path = "/tmp/_golden_random.csv"
    with open(csv_path, "w") as f:
        f.write("src_ip,dst_ip,src_port,dst_port\n")
        for i in range(n):
            f.write("%s,%s,%d,%d\n" % (ip_str(int(sip[i])), ip_str(int(dip[i])), sport[i], dport[i]))
    sim = Simulator(list(ex_key), 128, 24)
    sim.load_ips_from_csv(csv_path)
    sim.calc_hash()
    df = sim._Simulator__ip_df
    assert (df["hash_result"].to_numpy().astype(np.uint32) == hashes[0]).all()
    sweep_q = np.zeros((len(SWEEP), n), dtype=np.uint32)
    sweep_counts = {}
    for j, (h, q) in enumerate(SWEEP):
        sim._Simulator__hash_table_size = h
        sim._Simulator__queue_num = q
        sim.calc_queue_number()
        sweep_q[j] = df["queue_number"].to_numpy()
        vc = df["queue_number"].value_counts().sort_index()
        sweep_counts["%d,%d" % (h, q)] = [[int(a), int(b)] for a, b in vc.items()]
    np.savez(os.path.join(HERE, "random_tuples.npz"), sip=sip, dip=dip, sport=sport, dport=dport,
             keys=key_arr, key_len=key_len, hashes=hashes,
             sweep=np.array(SWEEP, dtype=np.int64), sweep_queue=sweep_q)
    with open(os.path.join(HERE, "sweep_counts.json"), "w") as f:
        json.dump(sweep_counts, f, indent=0, sort_keys=True)


def gen_one_hot(Toeplitz):
    ex_key = [int(x, 16) for x in open(os.path.join(HERE, "example_input/hash_key.txt")).read().split(":")]
    ms_key = [int(MS_KEY[i:i + 2], 16) for i in range(0, 80, 2)]
    rows = []
    for i in range(96):
        v = 1 << (95 - i)  # input bit i (MSB-first over the 96-bit string)
        rows.append(((v >> 64) & 0xFFFFFFFF, (v >> 32) & 0xFFFFFFFF, (v >> 16) & 0xFFFF, v & 0xFFFF))
    rows.append((0, 0, 0, 0))
    rows.append((0xFFFFFFFF, 0xFFFFFFFF, 0xFFFF, 0xFFFF))
    rows = np.array(rows, dtype=np.int64)
    out = np.zeros((2, len(rows)), dtype=np.uint32)
    for k, key in enumerate([ex_key, ms_key]):
        t = Toeplitz(list(key))
        for i, (s, d, sp, dp) in enumerate(rows):
            out[k, i] = t.compute_hash(ip_str(int(s)), ip_str(int(d)), int(sp), int(dp))
    np.savez(os.path.join(HERE, "one_hot.npz"), tuples=rows, hashes=out)


EDGE_CSVS = {
    "ports_wide.csv": "src_ip,dst_ip,src_port,dst_port\r\n1.2.3.4,5.6.7.8,65536,70000\r\n1.2.3.4,5.6.7.8,131071,0\r\n10.0.0.1,10.0.0.2,-1,-65536\r\n",
    "octet_overflow.csv": "src_ip,dst_ip,src_port,dst_port\n3.3.3.300,3.3.3.2,5201,5001\n256.256.256.256,1.1.1.1,1,1\n4294967296.0.0.1,0.0.0.0,0,0\n1.2.3.4.5,9.9.9.9,7,7\n",
    "whitespace.csv": "src_ip,dst_ip,src_port,dst_port\n 3.3.3.1,3.3.3.2 ,5201,5001\n3. 3.3.1,3.3.3.2,5202,5001\n010.001.1.1,3.3.3.2,5203,5001\n",
    "extra_reordered.csv": "dst_port,note,src_ip,vlan,dst_ip,src_port\n5001,a,3.3.3.1,7,3.3.3.2,5201\n5001,\"b,c\",3.3.3.1,8,3.3.3.2,5202\n5001,,3.3.3.1,9,3.3.3.2,5203\n",
    "missing_col.csv": "src_ip,dst_ip,src_port\n3.3.3.1,3.3.3.2,5201\n",
    "header_only.csv": "src_ip,dst_ip,src_port,dst_port\n",
    "single_row.csv": "src_ip,dst_ip,src_port,dst_port\n192.168.1.1,10.0.0.1,443,51234\n",
    "not_csv.csv": "\xff\xfe\x00garbage\n",
}
EDGE_RUNS = [
    # (name, csv, key file, htable, queues)
    ("ports_wide", "ports_wide.csv", "ex", "128", "24"),
    ("octet_overflow", "octet_overflow.csv", "ex", "128", "24"),
    ("whitespace", "whitespace.csv", "ex", "128", "24"),
    ("extra_reordered", "extra_reordered.csv", "ex", "512", "16"),
    ("missing_col", "missing_col.csv", "ex", "128", "24"),
    ("header_only", "header_only.csv", "ex", "128", "24"),
    ("single_row", "single_row.csv", "ex", "7", "3"),
    ("not_csv", "not_csv.csv", "ex", "128", "24"),
    ("no_such_file", "does_not_exist.csv", "ex", "128", "24"),
    ("key52", "single_row.csv", "key52", "128", "24"),
    ("key_trailing_nl", "single_row.csv", "key_nl", "128", "24"),
    ("key_crlf", "single_row.csv", "key_crlf", "128", "24"),
    ("key_bad", "single_row.csv", "key_bad", "128", "24"),
    ("key_41", "single_row.csv", "key_41", "128", "24"),
    ("htable_zero", "single_row.csv", "ex", "0", "24"),
    ("queues_neg", "single_row.csv", "ex", "128", "-3"),
    ("htable_text", "single_row.csv", "ex", "abc", "24"),
    ("htable_plus", "single_row.csv", "ex", "+128", "24"),
]


def gen_edge():
    edir = os.path.join(HERE, "edge")
    os.makedirs(edir, exist_ok=True)
    for name, text in EDGE_CSVS.items():
        with open(os.path.join(edir, name), "w", encoding="latin-1", newline="") as f:
            f.write(text)
    ex = open(os.path.join(HERE, "example_input/hash_key.txt")).read()
    rng = random.Random(7)
    k52 = ex + ":" + ":".join("%02x" % rng.getrandbits(8) for _ in range(12))
    keys = {"ex": ex, "key52": k52, "key_nl": ex + "\n", "key_crlf": ex + "\r\n",
            "key_bad": ex.replace("23:", "zz:", 1), "key_41": ex + ":00"}
    for kname, ktext in keys.items():
        with open(os.path.join(edir, "key_%s.txt" % kname), "w", newline="") as f:
            f.write(ktext)
    results = {}
    for name, csv, kname, h, q in EDGE_RUNS:
        out = os.path.join(edir, "out_%s.csv" % name)
        if os.path.exists(out):
            os.remove(out)
        args = ["--key-file", "key_%s.txt" % kname, "--ips-file", csv,
                "--htable-size", h, "--num-queues", q, "--csv", "out_%s.csv" % name]
        rc, so, err = run_cli(args, edir)
        res = {"args": args, "returncode": rc, "stdout": so, "stderr": err,
               "output": ("out_%s.csv" % name) if os.path.exists(out) else None}
        results[name] = res
        print(name, rc, err[:100], flush=True)
    with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
        json.dump(results, f, indent=1, sort_keys=True)


def gen_histogram(Simulator):
    """Histogram mode (simulator.py:118-172) with plt.show patched out: the figure's bar
    heights, bin edges, caption text, title and axis labels for a few configs."""
    import matplotlib.pyplot as plt
    ex_key = [int(x, 16) for x in open(os.path.join(HERE, "example_input/hash_key.txt")).read().split(":")]
    out = {}
    plt.show = lambda *a, **k: None
    for h, q in [(128, 24), (100, 7), (512, 64), (128, 1)]:
        plt.close("all")
        sim = Simulator(list(ex_key), h, q)
        sim.load_ips_from_csv(os.path.join(HERE, "example_input/ips.csv"))
        sim.calc_hash()
        sim.calc_queue_number()
        sim.show_histogram()
        fig = plt.gcf()
        ax = fig.axes[0]
        bars = [p for p in ax.patches]
        out["%d,%d" % (h, q)] = {
            "heights": [float(b.get_height()) for b in bars],
            "lefts": [float(b.get_x()) for b in bars],
            "caption": [t.get_text() for t in fig.texts],
            "title": ax.get_title(), "xlabel": ax.get_xlabel(), "ylabel": ax.get_ylabel(),
        }
    with open(os.path.join(HERE, "histogram.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def main(parts):
    Toeplitz, Simulator, _ = import_reference()
    if "example" in parts:
        gen_example()
    if "kat" in parts:
        gen_kat(Toeplitz)
    if "one_hot" in parts:
        gen_one_hot(Toeplitz)
    if "edge" in parts:
        gen_edge()
    if "random" in parts:
        gen_random(Toeplitz, Simulator)
    if "histogram" in parts:
        gen_histogram(Simulator)


if __name__ == "__main__":
    main(sys.argv[1:] or ["example", "kat", "one_hot", "edge", "random", "histogram"])

"""Pin the CPU oracle to the reference's own outputs (golden fixtures F1-F5).

The fixtures were produced by running noamsto/rss_simulator_nvidia itself
(tests/golden/make_golden.py); nothing here imports the reference.
"""
import json
import os

import numpy as np
import pandas as pd

from oracle import oracle as o


def test_ms_kat_all_paths(golden_dir, oracle_lib):
    with open(os.path.join(golden_dir, "ms_kat.json")) as f:
        kat = json.load(f)
    key = [int(x, 16) for x in kat["key"].split(":")]
    for v in kat["vectors"]:
        want = v["hash"]
        assert o.compute_hash_port(key, v["src_ip"], v["dst_ip"], v["src_port"], v["dst_port"]) == want
        sip, dip = o.ip_to_u32(v["src_ip"]), o.ip_to_u32(v["dst_ip"])
        assert oracle_lib.hash_rotating(key, sip, dip, v["src_port"], v["dst_port"]) == want
        tup = np.array([[sip, dip, o.pack_ports(v["src_port"], v["dst_port"])]], dtype=np.uint32)
        assert o.hash_batch_np(key, tup)[0] == want
        h, _, _ = oracle_lib.run(key, tup, 1, 1)
        assert h[0] == want


def test_random_tuples_four_keys(random_golden, oracle_lib):
    g = random_golden
    for k, key in enumerate(g["key_list"]):
        want = g["hashes"][k]
        np.testing.assert_array_equal(o.hash_batch_np(key, g["tuples"]), want)
        h, _, _ = oracle_lib.run(key, g["tuples"], 1, 1, threads=4)
        np.testing.assert_array_equal(h, want)


def test_port_restatement_on_subset(random_golden):
    # the slow literal port (the CPU-baseline code) on a slice, incl. ports > 65535
    g = random_golden
    key = g["key_list"][2]
    for i in range(0, 4096, 257):
        ip_s = "%d.%d.%d.%d" % tuple((int(g["sip"][i]) >> s) & 255 for s in (24, 16, 8, 0))
        ip_d = "%d.%d.%d.%d" % tuple((int(g["dip"][i]) >> s) & 255 for s in (24, 16, 8, 0))
        got = o.compute_hash_port(key, ip_s, ip_d, int(g["sport"][i]), int(g["dport"][i]))
        assert got == g["hashes"][2][i]


def test_one_hot_pins_every_window(golden_dir, oracle_lib, example_key):
    d = np.load(os.path.join(golden_dir, "one_hot.npz"), allow_pickle=False)
    rows, want = d["tuples"], d["hashes"]
    ports = ((rows[:, 2] & 0xFFFF) << 16 | (rows[:, 3] & 0xFFFF)).astype(np.uint32)
    tup = np.stack([rows[:, 0], rows[:, 1], ports], axis=1).astype(np.uint32)
    with open(os.path.join(golden_dir, "ms_kat.json")) as f:
        ms_key = [int(x, 16) for x in json.load(f)["key"].split(":")]
    for k, key in enumerate([example_key, ms_key]):
        np.testing.assert_array_equal(o.hash_batch_np(key, tup), want[k])
        # one-hot input i selects exactly window i
        np.testing.assert_array_equal(want[k][:96], oracle_lib.windows(key))
        np.testing.assert_array_equal(o.windows(key), oracle_lib.windows(key))
    assert want[0][96] == 0  # all-zero input


def test_sweep_queues_and_counts(random_golden):
    g = random_golden
    for j, (h, q) in enumerate(g["sweep"]):
        queue, counts = o.queue_and_counts(g["hashes"][0], int(h), int(q))
        np.testing.assert_array_equal(queue, g["sweep_queue"][j])
        ref = g["sweep_counts"]["%d,%d" % (h, q)]
        assert [[int(a), int(counts[a])] for a in np.flatnonzero(counts)] == ref


def test_oracle_lib_queue_counts_match_numpy(random_golden, oracle_lib):
    g = random_golden
    for h, q in [(128, 24), (100, 7), (1, 1), (65536, 1000), (512, 300)]:
        hh, qq, cc = oracle_lib.run(g["key_list"][0], g["tuples"], h, q, threads=3)
        q_np, c_np = o.queue_and_counts(hh, h, q)
        np.testing.assert_array_equal(qq, q_np)
        np.testing.assert_array_equal(cc, c_np)


def test_example_readme_counts(golden_dir, example_key):
    # README.md:82-107 counts reproduced through the oracle on example_input/ips.csv
    df = pd.read_csv(os.path.join(golden_dir, "example_input", "ips.csv"))
    tup = np.array([[o.ip_to_u32(s), o.ip_to_u32(d), o.pack_ports(sp, dp)]
                    for s, d, sp, dp in zip(df.src_ip, df.dst_ip, df.src_port, df.dst_port)],
                   dtype=np.uint32)
    _, counts = o.queue_and_counts(o.hash_batch_np(example_key, tup), 128, 24)
    readme = [4, 3, 3, 4, 3, 4, 3, 2, 8, 7, 7, 7, 2, 2, 2, 2, 2, 2, 2, 2, 7, 7, 8, 7]
    assert counts.tolist() == readme


def test_generator_np_matches_c(oracle_lib):
    for seed, first, n in [(0x5EED, 0, 1000), (0, 123456789, 777), (2**64 - 1, 2**40, 100)]:
        np.testing.assert_array_equal(o.generate_np(seed, first, n), oracle_lib.generate(seed, first, n))


def test_short_keys_wrap_like_the_rotation(oracle_lib):
    # Toeplitz(list) accepts any key >= 4 bytes; below 16 bytes the rotation wraps.
    # Literal pure-Python rotation vs the C restatement's literal rotation.
    rng = np.random.default_rng(3)
    for length in (4, 5, 8, 15, 16, 17, 40, 52, 64):
        key = [int(x) for x in rng.integers(0, 256, length)]
        k, want = list(key), []
        for _ in range(96):
            want.append(k[0] << 24 | k[1] << 16 | k[2] << 8 | k[3])
            k = o._rotate_key_left(k)
        np.testing.assert_array_equal(oracle_lib.windows(key), np.array(want, dtype=np.uint32))
        if length >= 16:
            np.testing.assert_array_equal(o.windows(key), np.array(want, dtype=np.uint32))


def test_table_form_equals_window_form(random_golden, oracle_lib):
    """oracle_run_tables (the bench's optimised-CPU line) == oracle_run == the reference's
    F3 hashes, for every key and a few (H, Q) incl. non-powers of two and Q > 256."""
    g = random_golden
    for k, key in enumerate(g["key_list"]):
        for H, Q in ((128, 24), (100, 7), (512, 64), (1 << 20, 1000)):
            a = oracle_lib.run(key, g["tuples"], H, Q, threads=4, fn="oracle_run_tables")
            b = oracle_lib.run(key, g["tuples"], H, Q, threads=4)
            np.testing.assert_array_equal(a[0], g["hashes"][k])
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y)


def test_word_tuple_batch_pinned(random_golden, golden_dir, oracle_lib):
    """oracle_run_words (the IPv6 checker of tests/test_gpu_ipv6_oracle.py): with 3 words per
    tuple it is oracle_run on the reference-made F3 hashes, all four keys; with 9 words it is
    the literal rotating loop over the 36 input bytes (oracle_hash_bytes) and the Microsoft
    IPv6 KAT."""
    tup = random_golden["tuples"]
    for k, key in enumerate(random_golden["key_list"]):
        h, q, c = oracle_lib.run_words(key, tup, 128, 24)
        np.testing.assert_array_equal(h, random_golden["hashes"][k].astype(np.uint32))
        ho, qo, co = oracle_lib.run(key, tup, 128, 24)
        np.testing.assert_array_equal(q, qo)
        np.testing.assert_array_equal(c, co)
    rng = np.random.default_rng(9)
    for key in random_golden["key_list"]:
        words = rng.integers(0, 2**32, (300, 9), dtype=np.uint64).astype(np.uint32)
        h, q, c = oracle_lib.run_words(key, words, 1000, 77)
        want = np.array([oracle_lib.hash_bytes(key, o.words_to_bytes(r)) for r in words],
                        dtype=np.uint32)
        np.testing.assert_array_equal(h, want)
        np.testing.assert_array_equal(q, want % 1000 % 77)
        np.testing.assert_array_equal(c, np.bincount(q, minlength=77).astype(np.uint64))
    from rss_simulator_nvidia_amd.ingest import ipv6_words
    kat = json.load(open(os.path.join(golden_dir, "ms_kat_ipv6.json")))
    key = [int(x, 16) for x in kat["key"].split(":")]
    words = np.array([ipv6_words(v["src_ip"]) + ipv6_words(v["dst_ip"]) +
                      [(v["src_port"] << 16) | v["dst_port"]] for v in kat["vectors"]],
                     dtype=np.uint32)
    h, _, _ = oracle_lib.run_words(key, words, 1, 1)
    assert [int(x) for x in h] == [int(v["hash_hex"], 16) for v in kat["vectors"]]

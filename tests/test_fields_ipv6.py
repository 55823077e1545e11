"""Field selection and IPv6, host side: the field-remapped and
IPv6 key windows reproduce the literal rotating-key loop over the selected bytes, the
Microsoft verification-suite "IPv4 only" vectors (produced by the reference itself with
zero ports, tests/golden/ms_kat.json) and its IPv6 vectors (tests/golden/ms_kat_ipv6.json)."""
import ipaddress
import json
import os

import numpy as np
import pandas as pd
import pytest

from oracle import oracle as o
from rss_simulator_nvidia_amd import _native
from rss_simulator_nvidia_amd.ingest import ipv6_words, pack_frame6

MASKS = list(range(1, 16))


def _key(text):
    return [int(x, 16) for x in text.split(":")]


def test_ipv4_only_kat_from_reference(golden_dir, oracle_lib):
    kat = json.load(open(os.path.join(golden_dir, "ms_kat.json")))
    key = _key(kat["key"])
    w = np.ctypeslib.as_array(_native.prepare_key(key, "sd").window)
    for v in kat["vectors"]:
        sip, dip = o.ip_to_u32(v["src_ip"]), o.ip_to_u32(v["dst_ip"])
        data = sip.to_bytes(4, "big") + dip.to_bytes(4, "big")
        assert oracle_lib.hash_bytes(key, data) == v["hash_ip_only"]
        # the remapped windows hash the full tuple (ports included) to the 8-byte hash
        tup = np.array([[sip, dip, o.pack_ports(v["src_port"], v["dst_port"])]], dtype=np.uint32)
        assert o.hash_words_np(w, tup)[0] == v["hash_ip_only"]


@pytest.mark.parametrize("mask", MASKS)
def test_field_masks_match_concatenated_bytes(mask, random_golden, oracle_lib):
    g = random_golden
    for key in g["key_list"][:2]:
        w = np.ctypeslib.as_array(_native.prepare_key(key, mask).window)
        got = o.hash_words_np(w, g["tuples"][:300])
        want = [oracle_lib.hash_bytes(key, o.select_fields_bytes(a, b, p, mask))
                for a, b, p in g["tuples"][:300]]
        np.testing.assert_array_equal(got, np.array(want, dtype=np.uint32))


def test_all_fields_is_the_reference_hash(random_golden):
    g = random_golden
    w = np.ctypeslib.as_array(_native.prepare_key(g["key_list"][0], "sdfn").window)
    np.testing.assert_array_equal(o.hash_words_np(w, g["tuples"]), g["hashes"][0])


def test_parse_fields():
    assert _native.parse_fields("sdfn") == 15 and _native.parse_fields("sd") == 3
    assert _native.parse_fields("n") == 8
    for bad in ("", "x", "ss", "sdfnx", None):
        with pytest.raises(ValueError):
            _native.parse_fields(bad)


def _v6_words(v):
    return ipv6_words(v["src_ip"]) + ipv6_words(v["dst_ip"]) + \
        [(v["src_port"] << 16) | v["dst_port"]]


def test_ipv6_kat(golden_dir, oracle_lib):
    kat = json.load(open(os.path.join(golden_dir, "ms_kat_ipv6.json")))
    key = _key(kat["key"])
    np.testing.assert_array_equal(np.ctypeslib.as_array(_native.prepare_key6(key).window),
                                  oracle_lib.windows_n(key, 288))
    w_all = np.ctypeslib.as_array(_native.prepare_key6(key).window)
    w_ip = np.ctypeslib.as_array(_native.prepare_key6(key, "sd").window)
    for v in kat["vectors"]:
        words = np.array([_v6_words(v)], dtype=np.uint32)
        data = o.words_to_bytes(words[0])
        assert oracle_lib.hash_bytes(key, data) == int(v["hash_hex"], 16)
        assert oracle_lib.hash_bytes(key, data[:32]) == int(v["hash_ip_only_hex"], 16)
        assert o.hash_words_np(w_all, words)[0] == int(v["hash_hex"], 16)
        assert o.hash_words_np(w_ip, words)[0] == int(v["hash_ip_only_hex"], 16)


@pytest.mark.parametrize("mask", [1, 2, 3, 4, 8, 12, 5, 10, 15])
def test_ipv6_field_masks(mask, oracle_lib):
    rng = np.random.default_rng(mask)
    key = [int(x) for x in rng.integers(0, 256, 40)]
    words = rng.integers(0, 2**32, (200, 9), dtype=np.uint64).astype(np.uint32)
    w = np.ctypeslib.as_array(_native.prepare_key6(key, mask).window)
    spans = [(1, 0, 16), (2, 16, 16), (4, 32, 2), (8, 34, 2)]
    want = []
    for row in words:
        data = o.words_to_bytes(row)
        want.append(oracle_lib.hash_bytes(key, b"".join(data[a:a + n] for bit, a, n in spans
                                                        if mask & bit)))
    np.testing.assert_array_equal(o.hash_words_np(w, words), np.array(want, dtype=np.uint32))


def test_ipv6_ingest():
    df = pd.DataFrame({"src_ip": ["::1", "3ffe:2501:200:3::1", " fe80::1 "],
                       "dst_ip": ["ff02::1", "::ffff:1.2.3.4", "2001:db8::"],
                       "src_port": [1, 65535, 70000], "dst_port": [0, 2, -1]})
    t = pack_frame6(df)
    for i in range(3):
        assert list(t["sip"][i]) == [int.from_bytes(ipaddress.IPv6Address(
            df.src_ip[i].strip()).packed[4 * k:4 * k + 4], "big") for k in range(4)]
    assert list(t["ports"]) == [(1 << 16) | 0, (65535 << 16) | 2, (4464 << 16) | 0xFFFF]
    with pytest.raises(ValueError):
        pack_frame6(pd.DataFrame({"src_ip": ["1.2.3.4"], "dst_ip": ["::1"], "src_port": [1],
                                  "dst_port": [1]}))

"""Key search: find RSS keys that spread a flow set evenly.

The reference can only draw one random key (``HashKey.random_hash_key``,
``rss_simulator/hash_key.py:53-60``) and show its histogram.  Here thousands of
candidate keys of the same shape (40 distinct random bytes) are evaluated in one
GPU launch (``rss_key_search_device``: one LDS lookup table per key, the flows read
from the on-die cache) and ranked by how close each key's per-queue counts come to
the ideal spread of the hash table: queue q owns ``slots(q) = #{b < H : b % Q == q}``
of the H buckets, so a perfect key gives it ``n * slots(q) / H`` flows.

    python -m rss_simulator_nvidia_amd.keysearch --ips-file flows.csv \\
        --htable-size 128 --num-queues 24 --keys 4096 --top 5 --out best_key.txt
"""
import argparse
import random

import numpy as np
import pandas as pd

from rss_simulator_nvidia_amd import _native
from rss_simulator_nvidia_amd.arg_parse_types import PositiveInt
from rss_simulator_nvidia_amd.arg_parse_types import arg_parse_type_decorator as apt_decorator
from rss_simulator_nvidia_amd.hash_key import HASH_KEY_BYTES_LENGTH, HashKey
from rss_simulator_nvidia_amd.ingest import pack_frame


def random_keys(count, seed=0, length=HASH_KEY_BYTES_LENGTH):
    """``count`` keys shaped like ``random_hash_key()``: ``length`` distinct random bytes."""
    rng = random.Random(seed)
    return [rng.sample(range(256), length) for _ in range(count)]


def key_text(key):
    """Colon-separated hex, the ``--key-file`` format (``hash_key.py:25-28``)."""
    return ":".join("{:02x}".format(b) for b in key)


def slot_share(htable, nqueues, width=None):
    """Fraction of the H buckets each queue owns (bucket b -> queue b % Q), for queues
    ``[0, width)`` (default: all Q)."""
    q = np.arange(nqueues if width is None else min(width, nqueues), dtype=np.int64)
    slots = htable // nqueues + (q < htable % nqueues)
    if nqueues > htable:
        slots = (q < htable).astype(np.int64)
    return slots / float(htable)


def balance(counts, htable, nqueues):
    """Per-key balance metrics for ``counts`` (``[keys, Q]``).

    Returns a dict of arrays: ``max_load`` = max over reachable queues of
    observed / ideal flows (1.0 is perfect), ``chi2`` = sum of (observed - ideal)^2 /
    ideal, and ``used`` = number of non-empty queues.
    """
    counts = np.atleast_2d(np.asarray(counts, dtype=np.float64))
    n = counts.sum(axis=1, keepdims=True)
    # Count rows are min(H, Q) wide (``_native.queue_modulus``): queues >= H own no bucket,
    # so the ideal share is cut to the columns present (nothing is lost).
    ideal = n * slot_share(htable, nqueues, counts.shape[1])[None, :]
    live = ideal[0] > 0
    with np.errstate(divide="ignore", invalid="ignore"):
        rel = np.where(ideal > 0, counts / np.where(ideal > 0, ideal, 1), 0.0)
        chi2 = (((counts - ideal) ** 2) / np.where(ideal > 0, ideal, 1))[:, live].sum(axis=1)
    return {"max_load": rel[:, live].max(axis=1) if live.any() else np.zeros(len(counts)),
            "chi2": chi2, "used": (counts > 0).sum(axis=1)}


def evaluate(keys, tuples, htable, nqueues, ctx=None):
    """uint64 per-queue counts ``[len(keys), Q]`` of packed ``tuples`` under every key (GPU)."""
    ctx = ctx or _native.default_context()
    prepared = [_native.prepare_key(k) for k in keys]
    return ctx.key_search(prepared, tuples, htable, nqueues)


def search(tuples, htable, nqueues, n_keys=1024, seed=0, top=10, extra_keys=()):
    """Rank ``n_keys`` random candidates (plus ``extra_keys``) for ``tuples``.

    Returns a list of dicts (best first): ``key``, ``max_load``, ``chi2``, ``used``, ``counts``.
    """
    keys = [list(k) for k in extra_keys] + random_keys(n_keys, seed)
    counts = evaluate(keys, tuples, htable, nqueues)
    m = balance(counts, htable, nqueues)
    order = np.lexsort((m["chi2"], m["max_load"]))
    return [{"key": keys[i], "max_load": float(m["max_load"][i]), "chi2": float(m["chi2"][i]),
             "used": int(m["used"][i]), "counts": counts[i]} for i in order[:top]]


def load_tuples(ips_file):
    """Packed tuples of a 4-tuple CSV: native fast path, else the pandas ingest."""
    parsed = _native.csv_parse(np.fromfile(ips_file, dtype=np.uint8))
    if parsed is not None:
        return parsed[0]
    return pack_frame(pd.read_csv(ips_file))


def main(argv=None):
    p = argparse.ArgumentParser(prog="rss-keysearch", description=__doc__.splitlines()[0])
    p.add_argument("--ips-file", metavar="PATH", required=True)
    p.add_argument("--htable-size", metavar="NUM", type=PositiveInt.parse, required=True)
    p.add_argument("--num-queues", metavar="NUM", type=PositiveInt.parse, required=True)
    p.add_argument("--keys", metavar="NUM", type=PositiveInt.parse, default=1024,
                   help="random candidate keys to evaluate")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--top", metavar="NUM", type=PositiveInt.parse, default=5)
    p.add_argument("--key-file", metavar="PATH", dest="key",
                   type=apt_decorator(HashKey.from_file),
                   help="also score this key (e.g. the one in use)")
    p.add_argument("--out", metavar="PATH", help="write the best key in --key-file format")
    args = p.parse_args(argv)
    tuples = load_tuples(args.ips_file)
    extra = [args.key] if args.key else []
    ranked = search(tuples, args.htable_size, args.num_queues, args.keys, args.seed, args.top,
                    extra)
    if args.key:
        base = balance(evaluate([args.key], tuples, args.htable_size, args.num_queues),
                       args.htable_size, args.num_queues)
        print("given key: max_load %.4f chi2 %.2f queues used %d"
              % (base["max_load"][0], base["chi2"][0], base["used"][0]))
    for r in ranked:
        print("%s  max_load %.4f chi2 %.2f queues used %d"
              % (key_text(r["key"]), r["max_load"], r["chi2"], r["used"]))
    if args.out:
        with open(args.out, "w") as f:
            f.write(key_text(ranked[0]["key"]))
    return ranked


if __name__ == "__main__":
    main()

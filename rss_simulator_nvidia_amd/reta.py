"""RSS indirection tables (RETA): ``queue = reta[hash % htable]``.

The reference maps buckets to queues with ``hash % htable % num_queues``
(``rss_simulator/simulator.py:96-98``), which is the table :func:`equal` builds --
``ethtool -X <dev> equal N`` -- and its docs point at ``ethtool -X ... weight``
(``docs/rss_general_explaination.md:9-11``), which :func:`weights` reproduces: queue j
gets a contiguous run of buckets proportional to its weight.  Tables are plain
integer lists/arrays; the kernel takes up to 1024 entries (``rss_hash_device_reta``).
"""
import numpy as np

MAX_ENTRIES = 1024


def equal(htable, nqueues, start=0):
    """``ethtool -X equal N [start S]``: bucket b -> start + b % N."""
    return [start + b % nqueues for b in range(htable)]


def weights(htable, weight_list):
    """``ethtool -X weight W0 W1 ...``: contiguous runs proportional to the weights."""
    w = [int(x) for x in weight_list]
    if not w or any(x < 0 for x in w) or sum(w) == 0:
        raise ValueError("weights must be non-negative with a positive sum")
    total, partial, j, table = sum(w), 0, -1, []
    for i in range(htable):
        while i >= htable * partial // total:
            j += 1
            partial += w[j]
        table.append(j)
    return table


def parse_weights(text):
    return [int(x) for x in text.split(",")]


def load(path):
    """Whitespace/comma separated queue ids, one per bucket."""
    with open(path) as f:
        return [int(x) for x in f.read().replace(",", " ").split()]


def validate(table, htable, nqueues):
    t = np.asarray(table, dtype=np.int64)
    if len(t) != htable:
        raise ValueError("indirection table has %d entries, htable is %d" % (len(t), htable))
    if htable > MAX_ENTRIES:
        raise ValueError("indirection tables hold at most %d entries" % MAX_ENTRIES)
    if len(t) and (t.min() < 0 or t.max() >= nqueues):
        raise ValueError("indirection table entries must lie in [0, %d)" % nqueues)
    return t.astype(np.uint32)

"""Generate tests/golden/bench_digest.npz: what bench.py's timed work must produce.

bench.py hashes the splitmix64 stream (seed 0x5EED, ``rss_generate_tuples`` /
``oracle_generate``) under the reference's example key with htable 128, 24 queues: rank r
of the weak-scaling run owns tuples [r * 2^28, (r + 1) * 2^28) (2^31 tuples at N = 8), and
the configs[3] block splits [0, 2^30) over the ranks.  This script runs the C oracle's
literal restatement of the reference loop (``oracle_run``: ``toeplitz.py:46-69`` +
``simulator.py:94-113``) over all 2^31 tuples, in the build container, and records

* per 2^20-tuple block b (2048 blocks): ``hash_xor[b]`` (XOR of the block's hash_result),
  ``hash_wsum[b]`` = sum_j hash[j] * (j + 1) mod 2^64 and ``queue_wsum[b]`` = sum_j
  queue[j] * (j + 1) mod 2^64 (j = index in the block: position-dependent, so a swapped or
  shifted element changes it);
* ``counts[c]`` = the 24 per-queue counts of every 2^27-tuple chunk c (16 chunks): any shard
  of either workload at N in {1, 2, 4, 8} is a union of chunks.

bench.py recomputes the same digests on the device from its resident outputs after the
timed region (``verify``) and exits non-zero on a mismatch.  Data only; no reference code.

Run:  python tests/golden/make_bench_digest.py   (~5 min on 8 threads)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

SEED, H, Q = 0x5EED, 128, 24
TOTAL = 1 << 31
BLOCK = 1 << 20
COUNTS_CHUNK = 1 << 27
STEP = 1 << 26


def block_digests_np(h, q, block=BLOCK):
    """(hash_xor, hash_wsum, queue_wsum) per block of the uint32 hash / queue columns."""
    nb = len(h) // block
    hb = h[:nb * block].reshape(nb, block)
    qb = q[:nb * block].reshape(nb, block).astype(np.uint64)
    w = np.arange(1, block + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        hw = (hb.astype(np.uint64) * w).sum(axis=1, dtype=np.uint64)
        qw = (qb * w).sum(axis=1, dtype=np.uint64)
    return np.bitwise_xor.reduce(hb, axis=1).astype(np.uint32), hw, qw


def main():
    from oracle.oracle import OracleLib
    lib = OracleLib()
    with open(os.path.join(HERE, "example_input", "hash_key.txt")) as f:
        key = [int(x, 16) for x in f.read().split(":")]
    hx, hw, qw = [], [], []
    counts = np.zeros((TOTAL // COUNTS_CHUNK, Q), dtype=np.uint64)
    t0 = time.time()
    for first in range(0, TOTAL, STEP):
        tup = lib.generate(SEED, first, STEP)
        h, q, c = lib.run(key, tup, H, Q, fn="oracle_run")
        a, b, d = block_digests_np(h, q)
        hx.append(a)
        hw.append(b)
        qw.append(d)
        counts[first // COUNTS_CHUNK] += c
        print("%d / %d tuples, %.0f s" % (first + STEP, TOTAL, time.time() - t0), flush=True)
    np.savez(os.path.join(HERE, "bench_digest.npz"), seed=np.uint64(SEED), htable=np.uint32(H),
             queues=np.uint32(Q), key=np.array(key, dtype=np.uint8), total=np.uint64(TOTAL),
             block=np.uint64(BLOCK), counts_chunk=np.uint64(COUNTS_CHUNK),
             hash_xor=np.concatenate(hx), hash_wsum=np.concatenate(hw),
             queue_wsum=np.concatenate(qw), counts=counts)


if __name__ == "__main__":
    main()

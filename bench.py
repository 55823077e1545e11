"""Benchmark: IPv4 4-tuples hashed/s (device-resident) + %HBM roofline on 1..8 MI355X.

One step = one pass of the hot path (Toeplitz hash -> htable index -> queue
modulo -> per-queue histogram, all outputs written) over this rank's resident
shard of synthetic tuples (one ``rss_hash_device_ws`` launch that also writes the step's
counts from zero -- single-pass counts, no zeroing launch; ``--zero-counts`` = a zeroing launch
+ an accumulating one; ``--graph`` replays the launch as a captured HIP graph), followed, under
a launcher, by ONE RCCL all-reduce of that batch's per-queue count vector (``ncclAllReduce`` on
the launch stream; ``--secondary-bucket`` times B batches per collective beside it, labelled).
Weak scaling: every rank owns ``--tuples-per-gpu``
tuples (default 2**28, BASELINE configs[2]) of one global splitmix64 stream.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line (see DESIGN.md §5 for every field).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "IPv4 4-tuples hashed/sec (device-resident) + %HBM roofline, 1/2/4/8 MI355X"
# example_input/hash_key.txt of the reference (the key BASELINE's configs use)
EXAMPLE_KEY = ("23:0d:44:3d:8c:2c:6e:64:d4:1a:f3:44:49:9b:21:74:fd:1a:9d:c1:dd:76:77:37:38:"
               "51:66:85:7b:dc:48:a8:3e:55:08:c1:63:af:01:9d")
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
READ_BYTES = 12                # packed tuple
HASH_BYTES = 4                 # u32 hash_result
QUEUE_BYTES = {"u8": 1, "u16": 2, "u32": 4}
SEED = 0x5EED


def parse_args():
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--tuples-per-gpu", type=int, default=1 << 28)
    p.add_argument("--htable", type=int, default=128)
    p.add_argument("--queues", type=int, default=24)
    p.add_argument("--queue-width", choices=["auto", "u8", "u16", "u32"], default="auto",
                   help="queue_number output dtype; auto = narrowest that holds every queue")
    p.add_argument("--cpu-sample", type=int, default=0,
                   help="tuples for the CPU baseline (default 0 = max(20000, 1500 per process): "
                        "the 20k-tuple subsample of BASELINE.md, >= ~2 s of work per process)")
    p.add_argument("--cpu-procs", type=int, default=0,
                   help="worker processes for the CPU baseline (default 0 = every core this "
                        "process may use: its CPU affinity, capped by a cgroup CPU quota)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the rank-0 secondary lines of the row-f kernels (IPv6 hash, key "
                        "search), timed after the main measurement")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl = RCCL over xGMI; gloo only to rehearse N>1 on one GPU")
    p.add_argument("--zero-counts", action="store_true",
                   help="zero each step's counts with a separate launch (counts.zero_() + an "
                        "accumulating rss_hash_device) instead of single-pass counts")
    p.add_argument("--placement-rounds", type=int, default=4, metavar="R",
                   help="up to R rounds of --placement-probe more output candidates while no "
                        "probed set is clearly faster than the rest (best >= 0.91 x slowest: "
                        "no faster tier found, or only the middle one); at N > 1 the slowest "
                        "rank's placement bounds the job")
    p.add_argument("--allreduce", choices=["overlap", "stream", "rccl"], default="rccl",
                   help="per-step count all-reduce (sharding.CountsPipeline): torch.distributed "
                        "async on its own stream (overlap), torch.distributed stream-ordered "
                        "(stream), or ncclAllReduce through rccl.RcclComm on the launch stream "
                        "(rccl)")
    p.add_argument("--allreduce-bucket", type=int, default=1, metavar="B",
                   help="steps per count all-reduce at N > 1 (default 1: one collective per "
                        "batch, the reference's unit of work -- one histogram per batch, "
                        "simulator.py:100-116); B > 1: each step's uint64[Q] counts are a row "
                        "of a [B, Q] bucket reduced by one collective after its B-th step "
                        "(sharding.CountsPipeline bucket)")
    p.add_argument("--secondary-bucket", type=int, default=8, metavar="B",
                   help="at N > 1, also time the same steps with B steps per collective as the "
                        "labelled secondary block `bucketed` (0 = skip)")
    p.add_argument("--settle-ms", type=float, default=600,
                   help="untimed launches of the step for this long before the warmup steps "
                        "(clock settle; 0 = none)")
    p.add_argument("--graph", action="store_true",
                   help="replay each step as a captured HIP graph (measured: no gain over "
                        "eager launches at 2**28 tuples per step)")
    p.add_argument("--distribution", choices=["uniform", "flow"], default="uniform",
                   help="uniform = splitmix64 over all 96 bits (SURVEY.md 8d); flow = the "
                        "example_input/ips.csv shape: one IP pair, sequential source ports")
    p.add_argument("--placement-probe", type=int, default=12, metavar="K",
                   help="place the resident buffers by timing the kernel on 2 candidate input "
                        "x K candidate output allocations before the timed region and keeping "
                        "the fastest (rss_simulator_nvidia_amd/placement.py); 0 = first "
                        "allocation, as allocated")
    p.add_argument("--secondary-warmup", type=int, default=30,
                   help="untimed launches of each secondary line's own mode before its timed ones")
    p.add_argument("--profile-dir", default=os.path.join(ROOT, "profiles"),
                   help="where committed rocprofv3 PMC summaries (traffic) are looked up")
    p.add_argument("--configs3-tuples", type=int, default=1 << 30, metavar="T",
                   help="BASELINE configs[3]: T global tuples split over the ranks by "
                        "sharding.shard_range, one RCCL all-reduce of the counts per batch "
                        "(the `configs3` block; 0 = skip)")
    p.add_argument("--configs3-steps", type=int, default=0, metavar="K",
                   help="timed configs[3] batches (default 0 = --steps)")
    p.add_argument("--no-verify", action="store_true",
                   help="skip the untimed check of the timed work against "
                        "tests/golden/bench_digest.npz")
    return p.parse_args()


# ---------------------------------------------------------- flow-like input ---
# SURVEY.md 8(d)'s second distribution, shaped like example_input/ips.csv (3.3.3.1 ->
# 3.3.3.2, source ports counting up from 5201, destination port 5001): tuple i has source
# port (5201 + i) mod 2**16 and, so that 2**28 tuples stay distinct, source address
# 3.3.3.1 + i // 2**16.
FLOW_SIP, FLOW_DIP, FLOW_SPORT, FLOW_DPORT = 0x03030301, 0x03030302, 5201, 5001


def flow_np(first, n):
    import numpy as np
    i = np.arange(first, first + n, dtype=np.uint64)
    t = np.empty((n, 3), dtype=np.uint32)
    t[:, 0] = ((FLOW_SIP + (i >> np.uint64(16))) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    t[:, 1] = FLOW_DIP
    t[:, 2] = (((FLOW_SPORT + i) & np.uint64(0xFFFF)) << np.uint64(16)).astype(np.uint32) | FLOW_DPORT
    return t


def flow_device(torch, tuples, first, n, dev):
    """flow_np(first, n) written into the int32 view ``tuples`` on the device (untimed)."""
    t = tuples.view(n, 3)
    chunk = 1 << 26
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        i = torch.arange(first + c0, first + c1, dtype=torch.int64, device=dev)
        t[c0:c1, 0] = ((FLOW_SIP + (i >> 16)) & 0xFFFFFFFF).to(torch.int32)
        t[c0:c1, 1] = FLOW_DIP
        t[c0:c1, 2] = ((((FLOW_SPORT + i) & 0xFFFF) << 16) | FLOW_DPORT).to(torch.int32)


# ------------------------------------------------------------ CPU baseline ----
def _port_worker(args):
    key, rows = args
    from oracle.oracle import compute_hash_port
    return [compute_hash_port(key, s, d, sp, dp) for s, d, sp, dp in rows]


def cpu_share():
    """Cores this process may use: its CPU affinity, capped by a cgroup v2/v1 CPU quota
    (``os.cpu_count()`` is the whole machine, which a container may not own)."""
    try:
        cores = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cores = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                period = int(f.read())
            if q > 0:
                quota = q / period
        except (OSError, ValueError):
            pass
    if quota is not None:
        cores = min(cores, max(1, int(quota)))
    # a scheduler that shares the machine without a quota states the share in
    # OMP_NUM_THREADS (the GPU boxes set it to their CPU share)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp == "1" and int(os.environ.get("LOCAL_WORLD_SIZE", "1")) > 1:
        omp = ""  # torch.distributed.run's own default for nproc > 1, not a CPU share
    if omp.isdigit() and int(omp) > 0:
        cores = min(cores, int(omp))
    return max(1, cores)


def cpu_baseline(key, n_sample, procs, distribution="uniform"):
    """Time the pure-Python restatement of the reference's per-tuple path (``oracle``).

    Runs BEFORE the GPU is touched (fork-safe).  The sample is the first
    ``n_sample`` tuples of the same synthetic stream, as the reference consumes
    them: dotted-quad strings and integer ports.
    """
    import multiprocessing as mp

    from oracle.oracle import generate_np
    tup = generate_np(SEED, 0, n_sample) if distribution == "uniform" else flow_np(0, n_sample)
    dotted = lambda v: "%d.%d.%d.%d" % ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)  # noqa
    rows = [(dotted(int(s)), dotted(int(d)), int(p) >> 16, int(p) & 0xFFFF) for s, d, p in tup]
    procs = max(1, min(procs, n_sample))
    # one core, in this process, as the calibration against the reference was measured
    n1 = min(1000, n_sample)
    t1 = time.perf_counter()
    assert len(_port_worker((key, rows[:n1]))) == n1
    single = n1 / (time.perf_counter() - t1)
    chunks = [rows[i::procs] for i in range(procs)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        out = pool.map(_port_worker, [(key, c) for c in chunks])
    dt = time.perf_counter() - t0
    assert sum(len(o) for o in out) == n_sample
    return {"value": n_sample / dt, "unit": "tuples/s", "cores": procs, "kind": "port",
            "single_core": {"value": single, "unit": "tuples/s", "sample": "first %d tuples, one "
                            "process, no pool" % n1},
            "reference_equivalent": reference_equivalent(n_sample / dt, single_core_rate=single),
            "optimised_c": optimised_c_baseline(key, procs, distribution),
            "procs": procs, "cpu_share": cpu_share(), "host_cores": os.cpu_count(),
            "sample": "first %d tuples of the bench stream, pure-Python restatement of "
                      "toeplitz.py:46-69 (rotating bit-string key) in %d processes (one per "
                      "core of this process's CPU share), %.2f s wall" % (n_sample, procs, dt)}


CALIBRATION_PATH = os.path.join(ROOT, "tests", "golden", "cpu_calibration.json")


def reference_equivalent(port_rate, path=CALIBRATION_PATH, single_core_rate=None):
    """The port's rate expressed in the reference's own: the reference
    cannot run on the GPU box, so tests/golden/make_cpu_calibration.py timed it beside the
    port on one core of the build container, on the same rows, and recorded their ratio
    (cpu_calibration.json, data only).  None when that record is absent.  With
    ``single_core_rate`` (the port timed on one core of this host, in process, as the ratio
    was measured) the line also carries that rate converted the same way: the like-for-like
    figure, one core against one core."""
    try:
        with open(path) as f:
            cal = json.load(f)
    except (OSError, ValueError):
        return None
    ratio = float(cal["port_over_reference"])
    return {"value": port_rate / ratio, "unit": "tuples/s", "port_over_reference": ratio,
            "approximate": True,
            "calibration": "tests/golden/cpu_calibration.json: reference %.0f vs port %.0f "
                           "tuples/s on one build-container core, %d tuples, identical hashes"
                           % (cal["reference_tuples_per_s"], cal["port_tuples_per_s"],
                              cal["tuples"]),
            "mismatch": "the ratio was measured single-core on the build container (its CPU and "
                        "Python build), the port's rate here is a multi-process pool timing on "
                        "the GPU box's host including pool start-up: an approximate conversion, "
                        "not a measurement of the reference",
            "single_core_value": (single_core_rate / ratio if single_core_rate else None)}


def optimised_c_baseline(key, threads, distribution="uniform", n=1 << 24):
    """SURVEY.md 8(d)'s optional "optimised CPU" line: the C byte-table form
    (``oracle_run_tables``: twelve 256-entry tables, hash % H % Q and the histogram, OpenMP
    over ``threads``) on
    ``n`` packed tuples of the same stream, best of three runs.  Reported beside the port,
    never as the baseline."""
    from oracle.oracle import OracleLib, generate_np
    lib = OracleLib()
    tup = generate_np(SEED, 0, n) if distribution == "uniform" else flow_np(0, n)
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        lib.run(key, tup, 128, 24, threads=threads, fn="oracle_run_tables")
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    return {"value": n / best, "unit": "tuples/s", "threads": threads,
            "sample": "%d tuples, hash u32 + queue u32 + counts (H=128, Q=24), oracle/"
                      "toeplitz_oracle.c oracle_run_tables (12 byte tables, 12 lookups per "
                      "tuple, OpenMP), best of 3" % n}


def load_traffic(profile_dir, n, htable, queues, queue_width):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_summarize.py)
    when it was measured on this exact configuration, else None."""
    path = os.path.join(profile_dir, "pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    if (rec.get("tuples"), rec.get("htable"), rec.get("queues"), rec.get("queue_width")) == \
            (n, htable, queues, queue_width):
        return rec.get("hbm_bytes_per_launch")
    return None


# ------------------------------------------------------ output verification --
DIGEST_PATH = os.path.join(ROOT, "tests", "golden", "bench_digest.npz")
DIGEST_BLOCK = 1 << 20   # tuples per digest block (tests/golden/make_bench_digest.py)


def load_digest(path=DIGEST_PATH):
    """The C oracle's digests of the bench stream (tests/golden/make_bench_digest.py), or
    None when the file is absent."""
    import numpy as np
    try:
        with np.load(path, allow_pickle=False) as d:
            return {k: d[k] for k in d.files}
    except OSError:
        return None


def digest_applies(gold, key_bytes, htable, nqueues, distribution):
    return (gold is not None and distribution == "uniform" and htable == int(gold["htable"])
            and nqueues == int(gold["queues"]) and list(gold["key"]) == list(key_bytes))


def block_digests(torch, hashes, queues, nblocks, block=DIGEST_BLOCK, chunk=64):
    """Per ``block``-tuple block of the resident outputs (hash_result int32 view, queue_number
    uint8): ``(hash_xor, hash_wsum, queue_wsum)`` as Python ints -- the XOR of the block's
    hashes, sum_j hash[j] * (j + 1) mod 2^64 and sum_j queue[j] * (j + 1) mod 2^64, exactly
    as tests/golden/make_bench_digest.py computes them with numpy.  Sums are split into
    16-bit halves so no int64 partial sum overflows."""
    dev = hashes.device
    w = torch.arange(1, block + 1, dtype=torch.int64, device=dev)
    hx, hw, qw = [], [], []
    for b0 in range(0, nblocks, chunk):
        nb = min(chunk, nblocks - b0)
        h = hashes[b0 * block:(b0 + nb) * block].view(nb, block)
        x = h
        while x.shape[1] > 1:
            half = x.shape[1] // 2
            x = torch.bitwise_xor(x[:, :half], x[:, half:2 * half])
        hx += [v & 0xFFFFFFFF for v in x[:, 0].tolist()]
        h64 = h.to(torch.int64) & 0xFFFFFFFF
        lo = ((h64 & 0xFFFF) * w).sum(dim=1).tolist()
        hi = ((h64 >> 16) * w).sum(dim=1).tolist()
        hw += [((a << 16) + b) % (1 << 64) for a, b in zip(hi, lo)]
        del h64
        q = queues[b0 * block:(b0 + nb) * block].view(nb, block).to(torch.int64)
        if queues.dtype != torch.uint8:  # int16 / int32 views of u16 / u32 queues
            q &= 0xFFFF if queues.dtype == torch.int16 else 0xFFFFFFFF
        qw += [v % (1 << 64) for v in (q * w).sum(dim=1).tolist()]
    return hx, hw, qw


def verify_outputs(torch, gold, hashes, queues, first, n):
    """Compare the resident outputs of tuples [first, first + n) (the rank's shard of the
    bench stream) with the golden digests; returns a dict with ``ok`` and what was checked
    (``ok`` None when the shard is not made of whole digest blocks inside the golden range)."""
    B = int(gold["block"])
    if first % B or n % B or first + n > int(gold["total"]):
        return {"ok": None, "why": "shard not whole %d-tuple blocks of the golden range" % B}
    b0, nb = first // B, n // B
    hx, hw, qw = block_digests(torch, hashes, queues, nb, B)
    bad = [b0 + i for i in range(nb)
           if (hx[i], hw[i], qw[i]) != (int(gold["hash_xor"][b0 + i]),
                                        int(gold["hash_wsum"][b0 + i]),
                                        int(gold["queue_wsum"][b0 + i]))]
    return {"ok": not bad, "blocks": nb, "first_block": b0, "bad_blocks": bad[:8]}


def golden_counts(gold, first, n):
    """Per-queue counts of tuples [first, first + n) from the golden chunk counts, or None
    when the range is not made of whole chunks."""
    C = int(gold["counts_chunk"])
    if first % C or n % C or first + n > int(gold["total"]):
        return None
    return [int(v) for v in gold["counts"][first // C:(first + n) // C].sum(axis=0)]


def _okcode(v):
    """1 / 0 / -1 for a verification record that passed / failed / could not be checked."""
    if not v or v.get("ok") is None:
        return -1.0
    return 1.0 if v["ok"] and v.get("counts_ok") is not False else 0.0


def gather_rows(torch, dist, row, device, distributed, world):
    """Every rank's ``row`` (floats), in rank order (all_gather; rank-local without a group)."""
    t = torch.tensor(row, dtype=torch.float64, device=device)
    if not distributed:
        return [t.tolist()]
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def max_over_ranks(torch, dist, values, device, distributed):
    """Element-wise max of ``values`` (floats) over the ranks (rank-local without a group)."""
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def verified_of(rows, has_configs3):
    """True: every rank's checks passed; False: any failed; None: nothing was checkable."""
    codes = [r[7] for r in rows] + ([r[8] for r in rows] if has_configs3 else [])
    return False if 0.0 in codes else (True if 1.0 in codes and -1.0 not in codes else None)


def run_bucketed(pipe, launch, steps, warmup, barrier, sync, reduce_max, n, world, Q):
    """The labelled secondary block at N > 1: the main line's steps with B = ``pipe.bucket``
    steps' count rows per collective (CountsPipeline(bucket=B)) -- fewer exchanges than the
    reference's one histogram per batch, so never the ``value``.  ``reduce_max`` = max over
    ranks of a list of floats; the last reduced row must hold n * world tuples."""
    for _ in range(warmup):
        pipe.step(launch)
    pipe.drain()
    barrier()
    sync()
    tb = time.perf_counter()
    for _ in range(steps):
        pipe.step(launch)
    blast = pipe.drain()
    sync()
    barrier()
    b_elapsed = reduce_max([time.perf_counter() - tb])[0]
    if int(blast.sum().item()) != n * world:
        raise SystemExit("bench: bucketed counts sum to %d, expected %d"
                         % (int(blast.sum().item()), n * world))
    return {"steps_per_collective": pipe.bucket,
            "collectives": -(-steps // pipe.bucket),
            "value": n * world * steps / b_elapsed,
            "ms_per_step": b_elapsed * 1e3 / steps,
            "note": "secondary: the main line's steps with %d steps' count rows per "
                    "collective (rows of a [%d, %d] bucket; every row is still its own "
                    "batch's reduced histogram) -- not the reference's one exchange per "
                    "batch, so not `value`" % (pipe.bucket, pipe.bucket, Q)}


def configs3_block(total, world, H, Q, steps, allreduce, distributed, stats_max, qw):
    """The ``configs3`` block from the slowest rank's [elapsed s, step ms, kernel ms, shard
    tuples] (``stats_max``)."""
    elapsed_max, step_max, kernel_max, n3_max = stats_max
    write_bytes = HASH_BYTES + QUEUE_BYTES[qw]
    achieved = n3_max * (READ_BYTES + write_bytes) / (kernel_max / 1e3) / 1e9
    return {
        "workload": "configs[3]: %d global synthetic 4-tuples split over %d rank(s) by "
                    "sharding.shard_range (contiguous shards), htable=%d, queues=%d; one batch "
                    "= one rss_hash_device_ws launch per rank + ONE %s of the batch's uint64[%d] "
                    "counts" % (total, world, H, Q,
                                {"rccl": "ncclAllReduce (rccl.RcclComm, launch stream)",
                                 "overlap": "torch.distributed all-reduce" if distributed
                                 else "local histogram (no process group)",
                                 "stream": "torch.distributed all-reduce"}[allreduce], Q),
        "global_tuples": total,
        "tuples_per_rank_max": int(n3_max),
        "steps": steps,
        "scaling": "strong",
        "ms_per_batch": elapsed_max * 1e3 / steps,
        "tuples_per_s": total * steps / elapsed_max,
        "step_ms_max_rank": step_max,
        "kernel_ms_max_rank": kernel_max,
        "exchange_ms_est": step_max - kernel_max,
        "timing": "ms_per_batch = wall time of the timed batches (barrier + synchronize on "
                  "both sides, slowest rank) / steps; step_ms = one HIP event pair on the "
                  "launch stream around the timed batches (launch + all-reduce); kernel_ms = "
                  "the same number of launches without the collective, after the region",
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "bytes_per_tuple": READ_BYTES + write_bytes},
    }


def run_configs3(args, torch, dist, _native, dev, stream, key, comm, rank, world, distributed,
                 barrier, qw, probe, gold):
    """BASELINE configs[3] as a strong-scaling batch: ``--configs3-tuples`` global tuples of
    the bench stream split over the ranks by ``sharding.shard_range``; one batch = one
    ``rss_hash_device_ws`` launch per rank over its resident shard + ONE all-reduce of the
    batch's counts (``CountsPipeline(bucket=1)``, RCCL on the launch stream under a launcher).
    Returns the ``configs3`` block of the line (+ this rank's values for ``per_rank``)."""
    from rss_simulator_nvidia_amd.resident import ResidentBatch
    from rss_simulator_nvidia_amd.sharding import CountsPipeline, shard_range
    total, H, Q = args.configs3_tuples, args.htable, args.queues
    first, n3 = shard_range(total, rank, world)
    sp = stream.cuda_stream

    def fill(t):
        if args.distribution == "uniform":
            _native.generate_device(SEED, first, n3, t.data_ptr(), sp)
        else:
            flow_device(torch, t, first, n3, dev)

    # placed like the main line's buffers, with fewer candidates (a 2^30-tuple shard's output
    # pair is 5 GiB)
    probe3 = (probe[0], min(8, probe[1]), probe[2]) if len(probe) > 2 else probe
    batch = ResidentBatch(n3, key, H, Q, device=dev, fill=fill, queue_width=qw,
                          placement=probe3, stream=stream)
    allreduce = args.allreduce if distributed else "overlap"
    pipe = CountsPipeline(Q, dev, single_pass=True, htable=H, allreduce=allreduce, comm=comm,
                          bucket=1)
    steps = args.configs3_steps or args.steps

    def launch(c, workspace):
        batch.hash(counts=c, workspace=workspace)

    for _ in range(max(3, args.warmup)):
        pipe.step(launch)
    pipe.drain()
    barrier()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for _ in range(steps):
        pipe.step(launch)
    pipe.flush()
    ev[1].record(stream)
    last = pipe.drain()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    step_ms = ev[0].elapsed_time(ev[1]) / steps  # launch + exchange, on the launch stream
    # the kernel alone (no collective), one event pair around `steps` launches
    local = torch.zeros(batch.counts_len, dtype=torch.int64, device=dev)
    ev[2].record(stream)
    for _ in range(steps):
        batch.hash(counts=local)
    ev[3].record(stream)
    torch.cuda.synchronize()
    kernel_ms = ev[2].elapsed_time(ev[3]) / steps
    stats_max = max_over_ranks(torch, dist, [elapsed, step_ms, kernel_ms, float(n3)],
                               dev if args.dist_backend == "nccl" else "cpu", distributed)
    counts = [int(x) & ((1 << 64) - 1) for x in last.tolist()]
    if sum(counts) != total:
        raise SystemExit("bench: configs[3] counts sum to %d, expected %d" % (sum(counts), total))
    verified = None
    if gold is not None:
        verified = verify_outputs(torch, gold, batch.hashes, batch.queue_view(), first, n3)
        want = golden_counts(gold, 0, total)
        verified["counts_ok"] = None if want is None else counts[:len(want)] == want
    out = configs3_block(total, world, H, Q, steps, allreduce, distributed, stats_max, qw)
    out.update({
        "placement_rank0": dict(batch.report),
        "verified": verified,
        "kernel_ms_rank": kernel_ms,
        "placement_rank": {"chosen_ms": batch.report["chosen_ms"],
                           "first_allocation_ms": batch.report["first_allocation_ms"]},
    })
    del batch, pipe, local
    torch.cuda.empty_cache()
    return out


# ------------------------------------------------------------------- main -----
def relaunch_distributed(n):
    """``--gpus N`` (N > 1) outside a launcher: run this script under torch.distributed.run
    as a child process (nothing has touched the GPU yet) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


CONFIGS4 = [(H, Q) for H in (128, 512) for Q in (8, 16, 24, 64)]


def configs4_block(torch, _native, key, tuples, hashes, queues, n, stream, warm, reps):
    """BASELINE configs[4] timed on this GPU (rank 0, after the main measurement): the same
    resident tuples and output buffers hashed under every (htable, num-queues) of the sweep
    (H in {128, 512} x Q in {8, 16, 24, 64}), full outputs (hash u32 + queue u8 + counts,
    17 B/tuple) and counts only (12 B/tuple), each the mean of `reps` launches bracketed by one
    HIP event pair after `warm` untimed ones.  Its per-queue parity with simulator.py is
    tests/test_gpu_parity.py::test_256M_sweep_counts_and_digest.  The launches carry
    RSS_FLAG_ADDR64 (the 64-bit-offset instance, like the probe and the settle launches), so
    the main step's kernel symbol in a rocprof summary counts the timed step's launches and
    its warmup alone."""
    sp = stream.cuda_stream
    counts = torch.zeros(64, dtype=torch.int64, device=tuples.device)
    acc = _native.FLAG_ACCUMULATE | _native.FLAG_ADDR64

    def timed(fn):
        for _ in range(warm):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    rows = []
    for H, Q in CONFIGS4:
        full = timed(lambda: _native.hash_device(key, tuples.data_ptr(), n, H, Q, hashes.data_ptr(),
                                                 queues.data_ptr(), counts.data_ptr(),
                                                 _native.FLAG_QUEUE_U8 | acc, sp))
        co = timed(lambda: _native.hash_device(key, tuples.data_ptr(), n, H, Q, None, None,
                                               counts.data_ptr(), acc, sp))
        rows.append({"htable": H, "queues": Q, "full_ms": full,
                     "full_tuples_per_s": n / (full / 1e3),
                     "full_frac": n * (READ_BYTES + HASH_BYTES + 1) / (full / 1e3) / 1e9 / HBM_PEAK_GBS,
                     "counts_only_ms": co, "counts_only_tuples_per_s": n / (co / 1e3),
                     "counts_only_read_frac": n * READ_BYTES / (co / 1e3) / 1e9 / HBM_PEAK_GBS})
    return {"tuples": n, "rows": rows,
            "note": "BASELINE configs[4]: the sweep's (H, Q) on the main line's placed buffers "
                    "(uniform input), full outputs (u8 queues) and counts only; mean of %d "
                    "launches after %d untimed ones, one HIP event pair each; 64-bit-offset "
                    "instance (RSS_FLAG_ADDR64)" % (reps, warm)}


def extra_lines(torch, _native, dev, stream, key_bytes):
    """Secondary timings of the row-f kernels on this GPU, after the main measurement
    (DESIGN.md §7-§8): the IPv6 kernel (2^26 uniform 36-byte tuples, u32 hash + u8 queue +
    counts: 36 B read + 5 B written per tuple) and key search (1024 random keys x 2^20 resident
    tuples, H=128, Q=24, counts only).  Mean launch time over one HIP event pair around
    back-to-back launches, after warm launches."""
    from rss_simulator_nvidia_amd import keysearch
    sp = stream.cuda_stream

    def timed(fn, warm=10, reps=20):
        # one pair of HIP events around `reps` back-to-back launches, as the main line's
        # kernel_ms (a pair around every launch costs ~7 us per launch)
        for _ in range(warm):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    out = {}
    n6 = 1 << 26
    words = torch.randint(-2**31, 2**31 - 1, (9 * n6,), dtype=torch.int32, device=dev)
    h6 = torch.empty(n6, dtype=torch.int32, device=dev)
    q6 = torch.empty(n6, dtype=torch.uint8, device=dev)
    c6 = torch.zeros(24, dtype=torch.int64, device=dev)
    k6 = _native.prepare_key6(key_bytes)
    ws6 = torch.zeros(_native.counts_workspace_bytes(128, 24) // 8, dtype=torch.int64, device=dev)
    # the IPv6 step as the IPv4 one: single-pass counts with the balanced tail
    # (rss_hash6_device_ws); beside it the plain launch (static walk, accumulating counts)
    def ipv6_ws():
        _native.hash6_device(k6, words.data_ptr(), n6, 128, 24, h6.data_ptr(), q6.data_ptr(),
                             c6.data_ptr(), _native.FLAG_QUEUE_U8, sp, ws6.data_ptr())

    def ipv6_plain():
        _native.hash6_device(k6, words.data_ptr(), n6, 128, 24, h6.data_ptr(), q6.data_ptr(),
                             c6.data_ptr(), _native.FLAG_QUEUE_U8 | _native.FLAG_ACCUMULATE, sp)

    # alternating, best of two each: right after the IPv4 launches the first IPv6 launches
    # run slow while the clocks settle (as counts-only does), which a single
    # pass would charge to whichever variant went first
    ms, ms_plain = float("inf"), float("inf")
    for _ in range(2):
        ms = min(ms, timed(ipv6_ws, warm=30))
        ms_plain = min(ms_plain, timed(ipv6_plain, warm=30))
    out["ipv6_hash"] = {"tuples": n6, "kernel_ms": ms, "tuples_per_s": n6 / (ms / 1e3),
                        "achieved_GBs": n6 * 41 / (ms / 1e3) / 1e9,
                        "bound": "hbm", "peak_GBs": HBM_PEAK_GBS,
                        "frac": n6 * 41 / (ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                        "bytes_per_tuple": 41, "outputs": "hash u32 + queue u8 + counts",
                        "launch": "rss_hash6_device_ws (single-pass counts, balanced tail)",
                        "plain_launch_ms": ms_plain}
    del words, h6, q6
    nk, nt = 1024, 1 << 20
    keys = keysearch.random_keys(nk, seed=0)
    import numpy as np
    win = np.stack([np.ctypeslib.as_array(_native.prepare_key(k).window) for k in keys])
    windows = torch.from_numpy(win.astype(np.uint32).view(np.int32)).to(dev)
    tup = torch.empty(3 * nt, dtype=torch.int32, device=dev)
    _native.generate_device(1, 0, nt, tup.data_ptr(), sp)
    kc = torch.empty((nk, 24), dtype=torch.int64, device=dev)
    ms = timed(lambda: _native.key_search_device(windows.data_ptr(), nk, tup.data_ptr(), nt, 128,
                                                 24, kc.data_ptr(), sp), warm=3, reps=10)
    rate = nk * nt / (ms / 1e3)
    out["key_search"] = {"keys": nk, "tuples": nt, "kernel_ms": ms,
                         "key_tuple_evals_per_s": rate, "htable": 128, "queues": 24,
                         "bound": "valu", "peak_evals_per_s": KEYSEARCH_VALU_PEAK,
                         "frac": rate / KEYSEARCH_VALU_PEAK,
                         "lds_peak_evals_per_s": KEYSEARCH_LDS_PEAK,
                         "lds_frac": rate / KEYSEARCH_LDS_PEAK,
                         "bound_note": "rss_key_search_packed_kernel on conflict-free tables "
                                       "(PMC, profiles/r04/pmc_keysearch_small/summary.json): per "
                                       "64 tuples x 8 keys 99 VALU (4 cycles each on a SIMD) and "
                                       "29 LDS instructions (58 LDS-array cycles, 0 bank "
                                       "conflicts) -- VALU issue binds; peaks at 2.4 GHz: VALU "
                                       "1024 SIMDs / (4 x 99) per 512 evaluations, LDS 256 CUs / "
                                       "58 per 512"}
    return out


def build_line(args, m):
    """Rank 0's JSON line from the measurements ``m`` (every rank's reduced / gathered
    values, rank 0's secondary timings); DESIGN.md §5 documents every field."""
    n, world, H, Q, qw = m["n"], m["world"], args.htable, args.queues, m["qw"]
    distributed, rows, c3 = m["distributed"], m["rows"], m["c3"]
    kernel_ms_max, launch_ms, bucket = m["kernel_ms_max"], m["launch_ms"], m["bucket"]
    co_ms, u32_ms, flow_ms = m["co_ms"], m["u32_ms"], m["flow_ms"]
    value = n * world * args.steps / m["elapsed"]
    # the slowest rank's mean launch time: at N > 1 the fraction is the worst rank's
    write_bytes = m["write_bytes"]
    achieved = n * (READ_BYTES + write_bytes) / (kernel_ms_max / 1e3) / 1e9
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "tuples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": m["elapsed"] * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": ("synthetic: splitmix64 IPv4 4-tuples generated on device, resident in HBM"
                 if args.distribution == "uniform" else
                 "synthetic flow-like IPv4 4-tuples (example_input/ips.csv shape: one IP "
                 "pair, sequential source ports) generated on device, resident in HBM"),
        "config": {
            "workload": "configs[2]: %d synthetic 4-tuples per GPU (x%d GPUs), key "
                        "example_input/hash_key.txt (40 B), htable=%d, queues=%d; outputs "
                        "hash_result (u32) + queue_number (%s) + per-queue counts (u64)"
                        % (n, world, H, Q, qw),
            "distribution": args.distribution,
            "tuples_per_gpu": n,
            "global_tuples": n * world,
            "htable": H,
            "queues": Q,
            "queue_width": qw,
            "collectives_per_batch": (1.0 / bucket) if distributed else 0,
            "parallelism": ("tuple-sharded x%d, %s all-reduce of every step's uint64[%d] "
                            "counts, %s %s"
                            % (world, "RCCL" if args.dist_backend == "nccl" else "gloo", Q,
                               "one collective per batch" if bucket == 1 else
                               "%d steps per collective (rows of a [%d, %d] bucket)"
                               % (bucket, bucket, Q),
                               {"overlap": "(torch.distributed async, overlapped with the "
                                           "next step)",
                                "stream": "(torch.distributed, stream-ordered after the "
                                          "launch)",
                                "rccl": "(ncclAllReduce via rccl.RcclComm, stream-ordered "
                                        "after the launch)"}[args.allreduce]))
                           if distributed else "single process, one GPU (no process group)",
            "step": ("zero counts + " if args.zero_counts else
                     "single-pass counts (rss_hash_device_ws): ") +
                    ("hash kernel (hipGraph replay)" if m["graph"]
                     else "hash kernel (eager launches)"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": m["traffic"],
            "kernel": "rss_toeplitz_kernel",
            "bytes_per_tuple": READ_BYTES + write_bytes,
            "kernel_ms": kernel_ms_max,
            "kernel_ms_rank0": m["kernel_ms"],
            "kernel_ms_max_rank": kernel_ms_max,
            "kernel_ms_min_max": [launch_ms[0], launch_ms[-1]],
            "kernel_ms_median": launch_ms[len(launch_ms) // 2],
            "kernel_ms_events_mean": sum(launch_ms) / len(launch_ms),
            "timing": "kernel_ms = GPU time per step on the launch stream: one pair of HIP "
                      "events around the %d timed launches (launches + the gaps between "
                      "them), slowest rank (kernel_ms_max_rank); min_max / median / "
                      "events_mean: %d launches each bracketed by HIP events, after the "
                      "timed region (RSS_FLAG_ADDR64: the 64-bit instance, like the probe, "
                      "settle and flow-like launches; the step's 32-bit instance runs only "
                      "the warmup and timed launches)"
                      % (args.steps, args.steps),
        },
        # the HBM-read roofline is the counts-only mode's bound (12 B read
        # per tuple, 666.7 G tuples/s per GPU); the full-output `value` also writes
        # write_bytes per tuple, so its share of that read-only bound understates its
        # HBM use (roofline.frac is its own algorithmic-byte fraction)
        "hbm_read_roofline": {
            "bound_tuples_per_s_per_gpu": HBM_PEAK_GBS * 1e9 / READ_BYTES,
            "counts_only_frac": n / (co_ms / 1e3) / (HBM_PEAK_GBS * 1e9 / READ_BYTES),
            "full_value_frac": value / (world * HBM_PEAK_GBS * 1e9 / READ_BYTES),
            # the same for the full-output kernel alone (slowest rank's mean launch), i.e.
            # without the per-step counts zeroing, event records and launch gaps
            "full_kernel_frac": n / (kernel_ms_max / 1e3) / (HBM_PEAK_GBS * 1e9 / READ_BYTES),
        },
        "counts_only": {
            "kernel_ms": co_ms,
            "input_probe_ms": m["co_probe"],
            "tuples_per_s_per_gpu": n / (co_ms / 1e3),
            "hbm_read_GBs": n * READ_BYTES / (co_ms / 1e3) / 1e9,
            "hbm_read_frac": n * READ_BYTES / (co_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
        },
        "queue_u32": {
            "kernel_ms": u32_ms,
            "queue_buffer_probe_ms": m["u32_probe"],
            "tuples_per_s_per_gpu": n / (u32_ms / 1e3),
            "achieved_GBs": n * 20 / (u32_ms / 1e3) / 1e9,
        },
        "cpu_baseline": m["baseline"],
    }
    line["secondary_min_median_max_ms"] = m["secondary_spread"]
    line["settle"] = {"launches": m["settle_launches"], "s": round(m["settle_s"], 3),
                      "note": "untimed launches of the step before the warmup steps "
                              "(--settle-ms; clock settle, rank-local)"}
    line["placement"] = dict(m["placement"], first_allocation_tuples_per_s_per_gpu=n / (
        m["placement"]["first_allocation_ms"] / 1e3), probe_addr64=True,
        note="resident buffers chosen among the probed candidate allocations before the "
             "timed region (ResidentBatch); first_allocation_* = the unplaced allocation's "
             "kernel-only rate")
    line["per_rank"] = [
        {"rank": int(r[0]), "kernel_ms": r[1], "chosen_ms": r[2], "first_allocation_ms": r[3],
         "configs3_kernel_ms": r[4] if c3 else None,
         "configs3_chosen_ms": r[5] if c3 else None,
         "configs3_first_allocation_ms": r[6] if c3 else None,
         "verified_main": {1.0: True, 0.0: False}.get(r[7]),
         "verified_configs3": {1.0: True, 0.0: False}.get(r[8])} for r in rows]
    if m["bucketed"] is not None:
        line["bucketed"] = m["bucketed"]
    if c3 is not None:
        c3.pop("kernel_ms_rank", None)
        c3.pop("placement_rank", None)
        line["configs3"] = c3
    line["verification"] = dict(m["verified"], source="tests/golden/bench_digest.npz (C oracle, "
                                "tests/golden/make_bench_digest.py): per-2^20-block hash / "
                                "queue digests of every rank's resident outputs + the "
                                "reduced counts, checked after the timed region")
    line["verified"] = m["verified_all"]
    if flow_ms is not None:
        line["flow_like"] = {
            "kernel_ms": flow_ms, "tuples_per_s_per_gpu": n / (flow_ms / 1e3),
            "note": "same outputs on flow-like input (one IP pair, sequential source ports; "
                    "--distribution flow), timed after the uniform run"}
    if m.get("configs4") is not None:
        line["configs4"] = m["configs4"]
    if m["extras"] is not None:
        line["row_f_kernels"] = m["extras"]
    return line


# rss_key_search_packed_kernel's bounds, per wave-step of 64 tuples x 8 keys
# (= 512 evaluations; PMC of the current kernel): 99 VALU instructions at 4 cycles on one of
# 1024 SIMDs, 58 LDS-array cycles on one of 256 CUs; 2.4 GHz
KEYSEARCH_VALU_PEAK = 1024 * 2.4e9 / (4 * 99) * 512
KEYSEARCH_LDS_PEAK = 256 * 2.4e9 / 58 * 512


def main():
    args = parse_args()
    if args.steps < 1 or args.warmup < 0:
        raise SystemExit("bench: --steps must be >= 1 and --warmup >= 0")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args.gpus))
    # under a launcher (torch.distributed.run sets WORLD_SIZE) a process group is created
    # at every world size, so `--nproc-per-node 1` runs the same RCCL calls as N = 8
    distributed = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        print("bench: --gpus %d but WORLD_SIZE=%d; reporting %d" % (args.gpus, world, world),
              file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    key_bytes = [int(x, 16) for x in EXAMPLE_KEY.split(":")]

    # rank 0 times the CPU baseline at every world size, before it (or any rank) joins the
    # process group or touches the GPU: the other ranks wait in the rendezvous meanwhile
    baseline = None
    if rank == 0 and not args.no_cpu_baseline:
        procs = args.cpu_procs or cpu_share()
        baseline = cpu_baseline(key_bytes, args.cpu_sample or max(20000, 1500 * procs), procs,
                                args.distribution)

    import torch
    import torch.distributed as dist

    from rss_simulator_nvidia_amd import _native

    # RSS_BENCH_DEVICE pins every rank to one device (rehearsing N>1 on a 1-GPU box)
    dev_index = int(os.environ.get("RSS_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if distributed:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    def barrier():
        if distributed:
            if args.dist_backend == "nccl":
                dist.barrier(device_ids=[dev_index])
            else:
                dist.barrier()

    n = args.tuples_per_gpu
    H, Q = args.htable, args.queues
    qw = args.queue_width
    if qw == "auto":
        qw = "u8" if Q <= 256 else ("u16" if Q <= 65536 else "u32")
    qflag = {"u8": _native.FLAG_QUEUE_U8, "u16": _native.FLAG_QUEUE_U16, "u32": 0}[qw]
    write_bytes = HASH_BYTES + QUEUE_BYTES[qw]
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    key = _native.prepare_key(key_bytes)
    counts = torch.zeros(Q, dtype=torch.int64, device=dev)

    def fill_input(t):
        if args.distribution == "uniform":
            _native.generate_device(SEED, rank * n, n, t.data_ptr(), sp)
        else:
            flow_device(torch, t, rank * n, n, dev)

    # resident stream buffers, placed by probing candidate allocations with the real kernel
    # (ResidentBatch / placement.py); queue buffers of the queue width (the u32
    # secondary line gets its own buffer after the timed region)
    from rss_simulator_nvidia_amd.resident import ResidentBatch
    probe = ((2, args.placement_probe, args.placement_rounds) if args.placement_probe > 0
             else (1, 1))
    batch = ResidentBatch(n, key, H, Q, device=dev, fill=fill_input, queue_width=qw,
                          placement=probe, stream=stream)
    tuples, hashes, queues = batch.tuples, batch.hashes, batch.queues
    placement = batch.report
    torch.cuda.synchronize()

    # Two count buffers: step i hashes into one while the RCCL all-reduce of step i-1's
    # buffer (async, on the collective stream) overlaps it (sharding.CountsPipeline).
    from rss_simulator_nvidia_amd.sharding import CountsPipeline
    # Single-pass counts (rss_hash_device_ws): the launch writes the step's counts itself, no
    # zeroing launch before it; --zero-counts = counts.zero_() + an accumulating launch
    comm = None
    if distributed and args.allreduce == "rccl" and args.dist_backend != "nccl":
        args.allreduce = "overlap"  # the gloo rehearsal: torch.distributed's exchange
    if distributed and args.allreduce == "rccl":
        from rss_simulator_nvidia_amd.rccl import RcclComm, RcclError
        try:
            comm = RcclComm(dev)
        except RcclError as err:
            if err.stuck:  # an init still blocked inside RCCL: no safe fallback in-process
                raise SystemExit("bench: RcclComm init timed out (%s); exiting instead of "
                                 "falling back to torch.distributed on the same RCCL" % err)
            # a clean failure on every rank: keep the run on torch.distributed's exchange
            print("bench: RcclComm unavailable (%s); --allreduce overlap" % err, file=sys.stderr)
            args.allreduce = "overlap"
    if args.allreduce_bucket < 1:
        raise SystemExit("bench: --allreduce-bucket must be >= 1")
    pipeline = CountsPipeline(Q, dev, single_pass=not args.zero_counts, htable=H,
                              allreduce=args.allreduce if distributed else "overlap", comm=comm,
                              bucket=args.allreduce_bucket if distributed else 1)

    def launch(c, workspace=None, extra_flags=0):
        ws = workspace
        _native.hash_device(key, tuples.data_ptr(), n, H, Q, hashes.data_ptr(), queues.data_ptr(),
                            c.data_ptr(), qflag | extra_flags |
                            (0 if ws is not None else _native.FLAG_ACCUMULATE),
                            torch.cuda.current_stream(dev).cuda_stream,
                            ws.data_ptr() if ws is not None else None)

    graphs = None
    if args.graph:
        try:  # capture one hash launch per count buffer; replay = one graph launch per step
            side = torch.cuda.Stream(dev)
            side.wait_stream(stream)
            with torch.cuda.stream(side):
                launch(pipeline.buffers[0], workspace=pipeline.workspace)
            stream.wait_stream(side)
            graphs = {}
            for c in pipeline.buffers:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    launch(c, workspace=pipeline.workspace)
                graphs[c.data_ptr()] = g
        except Exception as err:  # eager fallback keeps the same work per step
            print("bench: graph capture unavailable (%s); launching eagerly" % err, file=sys.stderr)
            graphs = None

    def step(i, ev=None):
        def timed_launch(c, workspace=None):
            if ev is not None:
                ev[0].record(stream)
            if graphs is not None:
                graphs[c.data_ptr()].replay()
            else:
                launch(c, workspace)
            if ev is not None:
                ev[1].record(stream)
        pipeline.step(timed_launch)

    def drain():
        return pipeline.drain()

    # Clock settle (untimed, rank-local, no collective): the first ~0.4 s of back-to-back
    # launches run ~0.8 % slower than sustained ones, and a box left idle for 0.3 s drops
    # back (tools/drift_probe.py, profiles/r02/drift_probe.jsonl) -- a service hashing batch
    # after batch runs in the settled state, so the timed steps should too.  The settle
    # launches carry RSS_FLAG_ADDR64 (same access shape, 64-bit addressing) like the
    # placement probe's, so a profile's row for the step's 32-bit kernel instance holds the
    # warmup and timed launches alone.
    settle_launches, t_settle = 0, time.perf_counter()
    while args.settle_ms > 0:
        for _ in range(16):
            _native.hash_device(key, tuples.data_ptr(), n, H, Q, hashes.data_ptr(),
                                queues.data_ptr(), counts.data_ptr(),
                                _native.FLAG_ACCUMULATE | _native.FLAG_ADDR64 | qflag, sp)
        settle_launches += 16
        torch.cuda.synchronize()
        if time.perf_counter() - t_settle >= args.settle_ms / 1e3:
            break
    settle_s = time.perf_counter() - t_settle

    for i in range(args.warmup):
        step(i)
    drain()
    barrier()
    torch.cuda.synchronize()
    # One pair of HIP events on the launch stream brackets the K timed launches:
    # roofline.achieved = algorithmic bytes over that GPU time per step (the launches plus
    # the gaps between them -- no per-launch events inside the timed region: a pair around
    # every launch costs ~7 us per step, profiles/r02/drift_probe.jsonl).  The per-launch
    # spread comes from K event-bracketed launches after the timed region.
    region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    region[0].record(stream)
    for i in range(args.steps):
        step(i)
    pipeline.flush()  # a partly filled bucket's collective belongs to the timed steps
    region[1].record(stream)
    last = drain()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0

    # kernel-only timing (HIP events on the launch stream), for roofline.achieved
    def kernel_ms_of(hash_ptr, queue_ptr, flags, reps, tuples_ptr=None):
        """Mean launch time of `reps` launches of one output mode (HIP events on the
        launch stream around each launch), after 30 untimed launches of that mode: right
        after the memory-bound full-output steps, the LDS/VALU-heavier counts-only launches
        run 10-35 % slow for ~20 launches while the clocks settle
        (profiles/r01_runs/mode_switch_probe.json, bench_secondary_warmup.json)."""
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(reps)]
        for i in range(-args.secondary_warmup, reps):
            if i >= 0:
                ev[i][0].record(stream)
            _native.hash_device(key, tuples_ptr or tuples.data_ptr(), n, H, Q, hash_ptr, queue_ptr,
                                counts.data_ptr(), flags | _native.FLAG_ACCUMULATE, sp)
            if i >= 0:
                ev[i][1].record(stream)
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) for a, b in ev)
        secondary_spread.append([t[0], t[len(t) // 2], t[-1]])
        return sum(t) / len(t)

    secondary_spread = []  # [min, median, max] ms of each secondary line, in order

    total = int(last.sum().item())
    if total != n * world:
        raise SystemExit("bench: per-queue counts sum to %d, expected %d" % (total, n * world))
    kernel_ms = region[0].elapsed_time(region[1]) / args.steps
    # per-launch spread: K launches of the same step, each bracketed by its own events --
    # with RSS_FLAG_ADDR64 (same access shape, the 64-bit instance) like every untimed
    # launch of the step, so a profile's row for the step's 32-bit instance holds exactly
    # the W warmup + K timed launches
    spread_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                 for _ in range(args.steps)]
    for e in spread_ev:
        e[0].record(stream)
        launch(counts, workspace=pipeline.workspace, extra_flags=_native.FLAG_ADDR64)
        e[1].record(stream)
    torch.cuda.synchronize()
    launch_ms = sorted(a.elapsed_time(b) for a, b in spread_ev)
    red_dev = dev if args.dist_backend == "nccl" else "cpu"

    def reduce_max(values):
        return max_over_ranks(torch, dist, values, red_dev, distributed)

    elapsed, kernel_ms_max = reduce_max([elapsed, kernel_ms])

    # The timed work itself, checked after the timed region (untimed): the resident outputs
    # of this rank's shard against the C oracle's per-block digests and the reduced counts
    # against the oracle's (tests/golden/make_bench_digest.py; simulator.py:94-113).
    gold = None if args.no_verify else load_digest()
    verify_ok = digest_applies(gold, key_bytes, H, Q, args.distribution)
    verified = {"main": None, "configs3": None}
    if verify_ok:
        v = verify_outputs(torch, gold, hashes, batch.queue_view(), rank * n, n)
        want = golden_counts(gold, 0, n * world)
        v["counts_ok"] = None if want is None else \
            [int(x) & ((1 << 64) - 1) for x in last.tolist()] == want
        verified["main"] = v

    # Labelled secondary block at N > 1: the same steps with B steps' count rows per
    # collective (CountsPipeline(bucket=B)) -- fewer exchanges than the reference's one
    # histogram per batch, so never the `value`
    bucketed = None
    if distributed and args.secondary_bucket > 1:
        bpipe = CountsPipeline(Q, dev, single_pass=not args.zero_counts, htable=H,
                               allreduce=args.allreduce, comm=comm, bucket=args.secondary_bucket)
        bucketed = run_bucketed(bpipe, launch, args.steps, args.warmup, barrier,
                                torch.cuda.synchronize, reduce_max, n, world, Q)
        del bpipe

    # BASELINE configs[3]: 2^30 global tuples split over the ranks (sharding.shard_range),
    # one batch = one rss_hash_device_ws launch per rank + ONE all-reduce of its counts
    # (bucket 1) -- the reference's unit of work, one histogram per batch
    # (simulator.py:100-116) -- strong scaling over N.
    c3 = None
    if args.configs3_tuples > 0:
        c3 = run_configs3(args, torch, dist, _native, dev, stream, key, comm, rank, world,
                          distributed, barrier, qw, probe, gold if verify_ok else None)
        verified["configs3"] = c3.pop("verified")

    # every rank's timings and placement, gathered for the line (rank 0 prints it)
    row = [float(rank), kernel_ms, placement["chosen_ms"], placement["first_allocation_ms"],
           c3["kernel_ms_rank"] if c3 else -1.0, c3["placement_rank"]["chosen_ms"] if c3 else -1.0,
           c3["placement_rank"]["first_allocation_ms"] if c3 else -1.0,
           _okcode(verified["main"]), _okcode(verified["configs3"])]
    rows = gather_rows(torch, dist, row, red_dev, distributed, world)
    verified_all = verified_of(rows, c3 is not None)

    # secondary lines (rank 0, after the timed region): counts-only mode (12 B/tuple,
    # the HBM-read roofline) and u32 queue outputs (20 B/tuple)
    co_ms = u32_ms = flow_ms = configs4 = None
    if rank == 0:
        reps = max(5, args.steps // 2)
        # counts only reads its input alone, and the read rate also depends a little on the
        # input's placement (profiles/r02/co_placed_probe.log): a counts-only deployment places
        # its input for that mode, so the line runs on the input kept by a counts-only probe of
        # the placed input and three copies
        co_input, co_probe = tuples, None
        if args.placement_probe > 0:
            def probe_co(buf, ev):
                if ev is not None:
                    ev[0].record(stream)
                _native.hash_device(key, buf.data_ptr(), n, H, Q, None, None, counts.data_ptr(),
                                    _native.FLAG_ACCUMULATE, sp)
                if ev is not None:
                    ev[1].record(stream)

            cands = [tuples.view(torch.uint8)]
            for _ in range(3):
                cands.append(torch.empty(12 * n, dtype=torch.uint8, device=dev))
                cands[-1].copy_(cands[0])
            times = []
            for b in cands:
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(5)]
                for k in range(-5, 5):
                    probe_co(b, ev[k] if k >= 0 else None)
                torch.cuda.synchronize()
                times.append(sorted(a.elapsed_time(c) for a, c in ev)[2])
            best = min(range(len(cands)), key=times.__getitem__)
            co_input = cands[best]
            co_probe = {"input%d" % i: round(x, 4) for i, x in enumerate(times)}
            co_probe["chosen"] = "input%d" % best
            del cands
        co_ms = kernel_ms_of(None, None, 0, reps, co_input.data_ptr())
        del co_input
        torch.cuda.empty_cache()
        queues32, u32_probe = queues, None
        if queues.numel() < 4 * n:  # the u32 line's queue buffer, placed like the others
            from rss_simulator_nvidia_amd.placement import choose_buffer

            def probe32(buf, ev):
                if ev is not None:
                    ev[0].record(stream)
                _native.hash_device(key, tuples.data_ptr(), n, H, Q, hashes.data_ptr(),
                                    buf.data_ptr(), counts.data_ptr(), _native.FLAG_ACCUMULATE, sp)
                if ev is not None:
                    ev[1].record(stream)
            queues32, u32_probe = choose_buffer(torch, dev, 4 * n, probe32, candidates=4)
        u32_ms = kernel_ms_of(hashes.data_ptr(), queues32.data_ptr(), 0, reps)
        del queues32
        if not args.no_extras and n >= 1 << 20:
            configs4 = configs4_block(torch, _native, key, tuples, hashes, queues, n, stream,
                                      args.secondary_warmup, reps)
        if args.distribution == "uniform":  # same kernel on SURVEY.md 8(d)'s flow-like input
            flow_device(torch, tuples, 0, n, dev)
            flow_ms = kernel_ms_of(hashes.data_ptr(), queues.data_ptr(),
                                   qflag | _native.FLAG_ADDR64, reps)

    extras = None
    if rank == 0 and not args.no_extras:
        extras = extra_lines(torch, _native, dev, stream, key_bytes)

    if rank == 0:
        line = build_line(args, dict(
            n=n, world=world, elapsed=elapsed, kernel_ms=kernel_ms, kernel_ms_max=kernel_ms_max,
            launch_ms=launch_ms, write_bytes=write_bytes, qw=qw, distributed=distributed,
            bucket=pipeline.bucket, graph=graphs is not None, co_ms=co_ms, co_probe=co_probe,
            u32_ms=u32_ms, u32_probe=u32_probe, flow_ms=flow_ms, baseline=baseline,
            secondary_spread=secondary_spread, settle_launches=settle_launches,
            settle_s=settle_s, placement=placement, rows=rows, c3=c3, bucketed=bucketed,
            verified=verified, verified_all=verified_all, extras=extras, configs4=configs4,
            traffic=load_traffic(args.profile_dir, n, H, Q, qw)))
        print(json.dumps(line), flush=True)
    if verified_all is False:
        print("bench: the timed work does not match the oracle's digests (see `verification`)",
              file=sys.stderr)
    if distributed:
        barrier()  # ranks leave together (rank 0 ran the secondary timings alone)
        if comm is not None:
            torch.cuda.synchronize()
            comm.destroy()
        dist.destroy_process_group()
    if verified_all is False:
        sys.exit(3)


if __name__ == "__main__":
    main()

"""Benchmark: IPv4 4-tuples hashed/s (device-resident) + %HBM roofline on 1..8 MI355X.

One step = one pass of the hot path (Toeplitz hash -> htable index -> queue
modulo -> per-queue histogram, all outputs written) over this rank's resident
shard of synthetic tuples, followed by the RCCL all-reduce of the per-queue
count vector when N > 1.  Weak scaling: every rank owns ``--tuples-per-gpu``
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
    p.add_argument("--cpu-sample", type=int, default=12000,
                   help="tuples for the CPU baseline (about 20 CPU-seconds)")
    p.add_argument("--cpu-procs", type=int, default=16,
                   help="worker processes for the CPU baseline (the box's CPU share)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--profile-dir", default=os.path.join(ROOT, "profiles"),
                   help="where committed rocprofv3 PMC summaries (traffic) are looked up")
    return p.parse_args()


# ------------------------------------------------------------ CPU baseline ----
def _port_worker(args):
    key, rows = args
    from oracle.oracle import compute_hash_port
    return [compute_hash_port(key, s, d, sp, dp) for s, d, sp, dp in rows]


def cpu_baseline(key, n_sample, procs):
    """Time the pure-Python restatement of the reference's per-tuple path (``oracle``).

    Runs BEFORE the GPU is touched (fork-safe).  The sample is the first
    ``n_sample`` tuples of the same synthetic stream, as the reference consumes
    them: dotted-quad strings and integer ports.
    """
    import multiprocessing as mp

    from oracle.oracle import generate_np
    tup = generate_np(SEED, 0, n_sample)
    dotted = lambda v: "%d.%d.%d.%d" % ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)  # noqa
    rows = [(dotted(int(s)), dotted(int(d)), int(p) >> 16, int(p) & 0xFFFF) for s, d, p in tup]
    procs = max(1, min(procs, n_sample))
    chunks = [rows[i::procs] for i in range(procs)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        out = pool.map(_port_worker, [(key, c) for c in chunks])
    dt = time.perf_counter() - t0
    assert sum(len(o) for o in out) == n_sample
    return {"value": n_sample / dt, "unit": "tuples/s", "cores": procs, "kind": "port",
            "sample": "first %d tuples of the bench stream, pure-Python restatement of "
                      "toeplitz.py:46-69 (rotating bit-string key) in %d processes, %.2f s wall"
                      % (n_sample, procs, dt)}


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


# ------------------------------------------------------------------- main -----
def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    key_bytes = [int(x, 16) for x in EXAMPLE_KEY.split(":")]

    baseline = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        baseline = cpu_baseline(key_bytes, args.cpu_sample, args.cpu_procs)

    import torch
    import torch.distributed as dist

    from rss_simulator_nvidia_amd import _native

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local_rank])

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
    tuples = torch.empty(3 * n, dtype=torch.int32, device=dev)
    hashes = torch.empty(n, dtype=torch.int32, device=dev)
    queues = torch.empty(n, dtype=torch.int32, device=dev)  # big enough for any width
    counts = torch.zeros(Q, dtype=torch.int64, device=dev)
    _native.generate_device(SEED, rank * n, n, tuples.data_ptr(), sp)
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]

    def step(i=None, hash_ptr=hashes.data_ptr(), queue_ptr=queues.data_ptr(), flags=qflag):
        counts.zero_()
        if i is not None:
            ev[i][0].record(stream)
        _native.hash_device(key, tuples.data_ptr(), n, H, Q, hash_ptr, queue_ptr,
                            counts.data_ptr(), _native.FLAG_ACCUMULATE | flags, sp)
        if i is not None:
            ev[i][1].record(stream)
        if world > 1:
            dist.all_reduce(counts)  # RCCL over xGMI: the one exchange step

    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    stats = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    elapsed, kernel_ms_max = float(stats[0]), float(stats[1])

    total = int(counts.sum().item())
    if total != n * world:
        raise SystemExit("bench: per-queue counts sum to %d, expected %d" % (total, n * world))

    # secondary lines (rank 0, after the timed region): counts-only mode (12 B/tuple,
    # the HBM-read roofline) and u32 queue outputs (20 B/tuple)
    def kernel_ms_of(hash_ptr, queue_ptr, flags):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = max(5, args.steps // 2)
        _native.hash_device(key, tuples.data_ptr(), n, H, Q, hash_ptr, queue_ptr,
                            counts.data_ptr(), flags, sp)
        a.record(stream)
        for _ in range(reps):
            _native.hash_device(key, tuples.data_ptr(), n, H, Q, hash_ptr, queue_ptr,
                                counts.data_ptr(), flags, sp)
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    co_ms = u32_ms = None
    if rank == 0:
        co_ms = kernel_ms_of(None, None, 0)
        u32_ms = kernel_ms_of(hashes.data_ptr(), queues.data_ptr(), 0)

    if rank == 0:
        value = n * world * args.steps / elapsed
        kernel_s = kernel_ms / 1e3
        achieved = n * (READ_BYTES + write_bytes) / kernel_s / 1e9
        traffic = load_traffic(args.profile_dir, n, H, Q, qw)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "tuples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: splitmix64 IPv4 4-tuples generated on device, resident in HBM",
            "config": {
                "workload": "configs[2]: %d synthetic 4-tuples per GPU (x%d GPUs), key "
                            "example_input/hash_key.txt (40 B), htable=%d, queues=%d; outputs "
                            "hash_result (u32) + queue_number (%s) + per-queue counts (u64)"
                            % (n, world, H, Q, qw),
                "tuples_per_gpu": n,
                "global_tuples": n * world,
                "htable": H,
                "queues": Q,
                "queue_width": qw,
                "parallelism": "tuple-sharded x%d, RCCL all-reduce of uint64[%d] counts"
                               % (world, Q),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "rss_toeplitz_kernel",
                "bytes_per_tuple": READ_BYTES + write_bytes,
                "kernel_ms": kernel_ms,
                "kernel_ms_max_rank": kernel_ms_max,
            },
            "hbm_read_roofline_frac": value / (world * HBM_PEAK_GBS * 1e9 / READ_BYTES),
            "counts_only": {
                "kernel_ms": co_ms,
                "tuples_per_s_per_gpu": n / (co_ms / 1e3),
                "hbm_read_GBs": n * READ_BYTES / (co_ms / 1e3) / 1e9,
                "hbm_read_frac": n * READ_BYTES / (co_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
            },
            "queue_u32": {
                "kernel_ms": u32_ms,
                "tuples_per_s_per_gpu": n / (u32_ms / 1e3),
                "achieved_GBs": n * 20 / (u32_ms / 1e3) / 1e9,
            },
            "cpu_baseline": baseline,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

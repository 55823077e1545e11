"""Rehearsal of bench.py's N > 1 path on CPU ranks (gloo) -- test infrastructure, no GPU.

Run as ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...
tests/bench_rehearsal.py OUT``.  Every rank parses bench's own arguments for ``--gpus N
--dist-backend gloo`` with a tiny shard and runs bench's own N > 1 machinery: the main
line's timed steps through ``sharding.CountsPipeline`` (bucket 1: ONE all-reduce per batch,
the reference's one histogram per batch), the labelled bucketed block (``run_bucketed``),
the configs[3] block over ``sharding.shard_range`` shards (``configs3_block``), the
max-over-ranks reductions (``max_over_ranks``), the per-rank gather (``gather_rows``,
``verified_of``) and ``build_line``.  The kernel launch is replaced by a CPU histogram of a
fixed queue sequence (there is no GPU here), so nothing is verified against the digests
(``verified`` is None) and every timing is a CPU timing: the line checks the structure the
driver's N = 8 run produces, never a rate.  Rank 0 writes the line to OUT."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_path = sys.argv[1]
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    sys.argv = ["bench.py", "--gpus", str(world), "--dist-backend", "gloo",
                "--tuples-per-gpu", "4096", "--steps", "10", "--warmup", "2",
                "--configs3-tuples", str(1 << 16), "--configs3-steps", "4",
                "--no-cpu-baseline", "--no-extras"]
    import torch
    import torch.distributed as dist

    import bench
    from rss_simulator_nvidia_amd.sharding import CountsPipeline, shard_range
    args = bench.parse_args()
    dist.init_process_group("gloo")
    # count the all-reduces the pipelines issue (sharding.allreduce_counts calls
    # dist.all_reduce through the module): one per batch is the contract
    issued = {"n": 0}
    all_reduce = dist.all_reduce

    def counting_all_reduce(*a, **k):
        issued["n"] += 1
        return all_reduce(*a, **k)

    dist.all_reduce = counting_all_reduce
    distributed = True
    n, H, Q = args.tuples_per_gpu, args.htable, args.queues
    qw = "u8"

    def histogram(first, count):
        i = torch.arange(first, first + count, dtype=torch.int64)
        return torch.bincount(((i * 2654435761) >> 7) % Q, minlength=Q)

    def launch_of(first, count):
        def launch(c, workspace=None):  # the pipeline zeroed c: accumulate, as the kernel does
            c += histogram(first, count)
        return launch

    def barrier():
        dist.barrier()

    def sync():
        pass

    def reduce_max(values):
        return bench.max_over_ranks(torch, dist, values, "cpu", distributed)

    # the main line: one collective per batch
    issued["n"] = 0
    launch = launch_of(rank * n, n)
    pipeline = CountsPipeline(Q, "cpu", allreduce="overlap", bucket=args.allreduce_bucket)
    for _ in range(args.warmup):
        pipeline.step(launch)
    pipeline.drain()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipeline.step(launch)
    pipeline.flush()
    last = pipeline.drain()
    barrier()
    elapsed = time.perf_counter() - t0
    main_collectives = issued["n"]
    kernel_ms = elapsed * 1e3 / args.steps
    total = int(last.sum().item())
    if total != n * world:
        raise SystemExit("rehearsal: counts sum to %d, expected %d" % (total, n * world))
    want = sum(histogram(r * n, n) for r in range(world))
    assert torch.equal(last, want), "reduced counts differ from the global histogram"
    elapsed, kernel_ms_max = reduce_max([elapsed, kernel_ms])

    bucketed = bench.run_bucketed(
        CountsPipeline(Q, "cpu", allreduce="overlap", bucket=args.secondary_bucket), launch,
        args.steps, args.warmup, barrier, sync, reduce_max, n, world, Q)

    # configs[3]: the global batch split by shard_range, one all-reduce per batch
    first, n3 = shard_range(args.configs3_tuples, rank, world)
    pipe3 = CountsPipeline(Q, "cpu", allreduce="overlap", bucket=1)
    launch3 = launch_of(first, n3)
    issued["n"] = 0
    barrier()
    t3 = time.perf_counter()
    for _ in range(args.configs3_steps):
        pipe3.step(launch3)
    last3 = pipe3.drain()
    barrier()
    e3 = time.perf_counter() - t3
    c3_collectives = issued["n"]
    dist.all_reduce = all_reduce
    shards = [None] * world
    dist.all_gather_object(shards, [first, n3, main_collectives, c3_collectives])
    if int(last3.sum().item()) != args.configs3_tuples:
        raise SystemExit("rehearsal: configs[3] counts sum to %d" % int(last3.sum().item()))
    stats3 = reduce_max([e3, e3 * 1e3 / args.configs3_steps, e3 * 1e3 / args.configs3_steps,
                         float(n3)])
    c3 = bench.configs3_block(args.configs3_tuples, world, H, Q, args.configs3_steps, "overlap",
                              distributed, stats3, qw)
    placement = {"chosen_ms": kernel_ms, "first_allocation_ms": kernel_ms}
    row = [float(rank), kernel_ms, kernel_ms, kernel_ms, stats3[2], kernel_ms, kernel_ms, -1.0, -1.0]
    rows = bench.gather_rows(torch, dist, row, "cpu", distributed, world)
    verified = {"main": None, "configs3": None}
    verified_all = bench.verified_of(rows, True)
    if rank == 0:
        line = bench.build_line(args, dict(
            n=n, world=world, elapsed=elapsed, kernel_ms=kernel_ms, kernel_ms_max=kernel_ms_max,
            launch_ms=[kernel_ms] * args.steps, write_bytes=bench.HASH_BYTES + bench.QUEUE_BYTES[qw],
            qw=qw, distributed=distributed, bucket=pipeline.bucket, graph=False, co_ms=kernel_ms,
            co_probe=None, u32_ms=kernel_ms, u32_probe=None, flow_ms=None, baseline=None,
            secondary_spread=[], settle_launches=0, settle_s=0.0, placement=placement, rows=rows,
            c3=c3, bucketed=bucketed, verified=verified, verified_all=verified_all, extras=None,
            traffic=None))
        line["data"] = "rehearsal: CPU ranks, a CPU histogram in place of the kernel (not a rate)"
        line["rehearsal"] = {
            "main_batches": args.warmup + args.steps,
            "main_collectives": [s[2] for s in shards],
            "configs3_batches": args.configs3_steps,
            "configs3_collectives": [s[3] for s in shards],
            "configs3_shards": [[s[0], s[1]] for s in shards]}
        with open(out_path, "w") as f:
            f.write(json.dumps(line) + "\n")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""bench.py host helpers (no GPU): the flow-like generator's device (torch) and numpy
forms agree and start at example_input/ips.csv's first row; PMC traffic lookup keys."""
import json

import numpy as np
import pytest
import torch

import bench
from rss_simulator_nvidia_amd.ingest import ip_to_u32


def test_flow_generator_forms_agree():
    for first, n in ((0, 1000), (65530, 20), ((1 << 32) - 3, 70000)):
        t = torch.empty(3 * n, dtype=torch.int32)
        bench.flow_device(torch, t, first, n, "cpu")
        np.testing.assert_array_equal(t.numpy().view(np.uint32).reshape(n, 3),
                                      bench.flow_np(first, n))


def test_flow_generator_matches_example_shape(golden_dir):
    t = bench.flow_np(0, 100)
    assert t[0].tolist() == [ip_to_u32("3.3.3.1"), ip_to_u32("3.3.3.2"), 5201 << 16 | 5001]
    assert (t[:, 0] == t[0, 0]).all() and (t[:, 1] == t[0, 1]).all()
    assert ((t[:, 2] >> 16) == np.arange(5201, 5301)).all()
    t = bench.flow_np(65536 - 5201, 1)  # source ports wrap, the source address advances
    assert t[0].tolist() == [ip_to_u32("3.3.3.1"), ip_to_u32("3.3.3.2"), 5001]
    assert bench.flow_np(1 << 16, 1)[0, 0] == ip_to_u32("3.3.3.2")


def test_load_traffic_only_for_matching_config(tmp_path):
    rec = {"tuples": 8, "htable": 128, "queues": 24, "queue_width": "u8",
           "hbm_bytes_per_launch": 136.0}
    (tmp_path / "pmc_traffic.json").write_text(json.dumps(rec))
    assert bench.load_traffic(str(tmp_path), 8, 128, 24, "u8") == 136.0
    assert bench.load_traffic(str(tmp_path), 8, 128, 24, "u32") is None
    assert bench.load_traffic(str(tmp_path / "missing"), 8, 128, 24, "u8") is None


def test_cpu_share_ignores_torchrun_default_omp(monkeypatch):
    """torch.distributed.run sets OMP_NUM_THREADS=1 for nproc > 1 when it is unset: that is
    not the node's CPU share, so the N > 1 baseline is not cut to one core by it."""
    import bench
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    free = bench.cpu_share()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert bench.cpu_share() == 1
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert free == bench.cpu_share()
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert bench.cpu_share() == min(3, free)


def _make_bench_digest():
    import importlib.util
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "make_bench_digest.py")
    spec = importlib.util.spec_from_file_location("make_bench_digest_under_test", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_block_digests_match_the_generator():
    """bench.block_digests (torch, what the GPU run computes) == the generator's numpy form,
    incl. all-ones hashes (the largest partial sums) and u8 / u16 / u32 queue views."""
    gen = _make_bench_digest()
    rng = np.random.default_rng(5)
    B, nb = 1024, 6
    h = rng.integers(0, 1 << 32, B * nb, dtype=np.uint64).astype(np.uint32)
    h[:B] = 0xFFFFFFFF
    for qmax, dt in ((24, torch.uint8), (60000, torch.int16), (3_000_000_000, torch.int32)):
        q = rng.integers(0, qmax, B * nb, dtype=np.uint64).astype(np.uint32)
        q[B:2 * B] = qmax - 1
        want = gen.block_digests_np(h, q, block=B)
        qv = {torch.uint8: q.astype(np.uint8), torch.int16: q.astype(np.uint16).view(np.int16),
              torch.int32: q.view(np.int32)}[dt]
        got = bench.block_digests(torch, torch.from_numpy(h.view(np.int32)),
                                  torch.from_numpy(qv), nb, block=B, chunk=4)
        assert got[0] == [int(x) for x in want[0]]
        assert got[1] == [int(x) for x in want[1]]
        assert got[2] == [int(x) for x in want[2]]


def test_bench_digest_is_pinned_to_the_oracle(oracle_lib, example_key):
    """The committed digests of blocks 0 and 2047 (first and last 2^20 tuples of the 2^31
    stream) recomputed here by the C oracle; verify_outputs accepts them and flags one
    changed hash or queue; the chunk counts cover 2^27 tuples each."""
    gold = bench.load_digest()
    assert gold is not None and bench.digest_applies(gold, example_key, 128, 24, "uniform")
    assert not bench.digest_applies(gold, example_key, 128, 24, "flow")
    B = int(gold["block"])
    for b in (0, int(gold["total"]) // B - 1):
        tup = oracle_lib.generate(bench.SEED, b * B, B)
        h, q, _ = oracle_lib.run(example_key, tup, 128, 24, fn="oracle_run_tables")
        ht = torch.from_numpy(h.view(np.int32).copy())
        qt = torch.from_numpy(q.astype(np.uint8))
        v = bench.verify_outputs(torch, gold, ht, qt, b * B, B)
        assert v["ok"] is True and v["blocks"] == 1, v
        ht[B // 2] ^= 1
        assert bench.verify_outputs(torch, gold, ht, qt, b * B, B)["bad_blocks"] == [b]
        ht[B // 2] ^= 1
        qt[7], qt[8] = qt[8].item(), qt[7].item() + (1 if qt[7] == qt[8] else 0)
        assert bench.verify_outputs(torch, gold, ht, qt, b * B, B)["ok"] is False
    assert (gold["counts"].sum(axis=1) == int(gold["counts_chunk"])).all()
    assert bench.golden_counts(gold, 0, 1 << 28) == \
        [int(x) for x in gold["counts"][:2].sum(axis=0)]
    assert bench.golden_counts(gold, 1 << 20, 1 << 27) is None   # not whole chunks
    assert bench.verify_outputs(torch, gold, ht, qt, 5, B)["ok"] is None


def check_bench_line(line):
    """The fields VERDICT r02 asked every bench line to carry (configs[3] block, per-rank
    timings and placement, the verification of the timed work) are present and coherent."""
    n = line["n_gpus"]
    assert line["verified"] is True, line.get("verification")
    v = line["verification"]
    assert v["main"]["ok"] is True and v["main"]["counts_ok"] is True
    c3 = line["configs3"]
    assert c3["scaling"] == "strong" and c3["global_tuples"] == 1 << 30
    assert c3["tuples_per_rank_max"] == (1 << 30) // n
    assert c3["tuples_per_s"] > 0 and c3["ms_per_batch"] > 0
    assert c3["kernel_ms_max_rank"] <= c3["step_ms_max_rank"] * 1.5
    assert 0 < c3["roofline"]["frac"] < 1
    assert v["configs3"]["ok"] is True and v["configs3"]["counts_ok"] is True
    rows = line["per_rank"]
    assert [r["rank"] for r in rows] == list(range(n))
    for r in rows:
        assert r["kernel_ms"] > 0 and r["chosen_ms"] > 0 and r["first_allocation_ms"] > 0
        assert r["configs3_kernel_ms"] > 0 and r["verified_main"] is True
        assert r["verified_configs3"] is True
    assert line["roofline"]["kernel_ms_max_rank"] == max(r["kernel_ms"] for r in rows)
    return line


def test_default_exchange_is_one_collective_per_batch(monkeypatch):
    """at N > 1 the headline does one all-reduce per batch (the reference's
    unit of work, one histogram per batch, simulator.py:100-116); bucketing is a labelled
    secondary block."""
    import bench
    monkeypatch.setattr("sys.argv", ["bench.py", "--gpus", "8"])
    args = bench.parse_args()
    assert args.allreduce_bucket == 1 and args.secondary_bucket == 8
    assert args.configs3_tuples == 1 << 30


def test_committed_bench_lines_do_one_exchange_per_batch():
    """The world-size-1 RCCL run (torchrun --nproc-per-node 1) and the 8-rank gloo rehearsal
    on one GPU (RSS_BENCH_DEVICE=0), as committed under profiles/r06/: the configs[3] and
    per-rank blocks, ONE all-reduce per batch in the main line (VERDICT r03 item 2:
    simulator.py:100-116 makes one histogram per batch) and the 8-steps-per-collective form
    only as the labelled `bucketed` block."""
    import glob
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    paths = sorted(glob.glob(os.path.join(root, "profiles", "r06", "bench_lines", "*.json")))
    assert paths, "no committed round-6 bench lines"
    seen = set()
    for p in paths:
        with open(p) as f:
            line = check_bench_line(json.loads(f.read().strip().splitlines()[-1]))
        cfg = line["config"]
        assert cfg["collectives_per_batch"] == 1.0, p
        assert "one collective per batch" in cfg["parallelism"], p
        b = line["bucketed"]
        assert b["steps_per_collective"] == 8 and b["value"] > 0
        assert b["collectives"] == -(-line["steps"] // 8)
        assert line["configs3"]["scaling"] == "strong"
        seen.add((line["n_gpus"], "gloo" if "gloo" in cfg["parallelism"] else
                  ("RCCL" if "RCCL" in cfg["parallelism"] else "none")))
    assert (1, "RCCL") in seen and (8, "gloo") in seen, seen


@pytest.mark.parametrize("world", [2, 4, 8])
def test_world_rehearsal_line(tmp_path, world):
    """bench.py's N > 1 machinery at every N of the driver's
    curve but 1 (BASELINE configs[3] "scaling curve 1/2/4/8") on CPU ranks (gloo,
    tests/bench_rehearsal.py): one all-reduce per batch on every rank (counted), N per-rank
    rows in rank order, the configs[3] block over N contiguous shard_range shards that tile
    the global batch, and the labelled bucketed block -- so the driver's multi-GPU runs do not
    meet a path only world size 1 has run."""
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "line.json"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", str(world), "--master-addr", "127.0.0.1",
                        "--master-port", str(port),
                        os.path.join(root, "tests", "bench_rehearsal.py"), str(out)],
                       capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = json.loads(out.read_text())
    assert line["n_gpus"] == world and line["scaling"] == "weak" and line["value"] > 0
    cfg = line["config"]
    assert cfg["collectives_per_batch"] == 1.0 and cfg["global_tuples"] == world * 4096
    assert "one collective per batch" in cfg["parallelism"] and "gloo" in cfg["parallelism"]
    rows = line["per_rank"]
    assert [r["rank"] for r in rows] == list(range(world))
    assert line["roofline"]["kernel_ms_max_rank"] >= max(r["kernel_ms"] for r in rows) * 0.999
    reh = line["rehearsal"]
    assert reh["main_collectives"] == [reh["main_batches"]] * world
    assert reh["configs3_collectives"] == [reh["configs3_batches"]] * world
    c3 = line["configs3"]
    assert c3["scaling"] == "strong" and c3["global_tuples"] == 1 << 16
    shards = reh["configs3_shards"]
    assert shards[0][0] == 0 and sum(n for _, n in shards) == 1 << 16
    assert all(a + n == b for (a, n), (b, _) in zip(shards, shards[1:]))  # contiguous
    assert c3["tuples_per_rank_max"] == max(n for _, n in shards) == -(-(1 << 16) // world)
    b = line["bucketed"]
    assert b["steps_per_collective"] == 8 and b["collectives"] == -(-line["steps"] // 8)
    assert line["verified"] is None and line["verification"]["main"] is None


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_configs3_shards_tile_the_full_batch(world):
    """BASELINE configs[3] at its real size: 2^30 tuples over N ranks, contiguous
    shard_range shards of 2^30 / N (the same ranges rss_hash_host_multi uses)."""
    from rss_simulator_nvidia_amd.sharding import shard_range
    total = 1 << 30
    shards = [shard_range(total, r, world) for r in range(world)]
    assert shards[0][0] == 0 and all(n == total // world for _, n in shards)
    assert all(a + n == b for (a, n), (b, _) in zip(shards, shards[1:]))
    assert sum(n for _, n in shards) == total


def test_relaunch_runs_torchrun_on_loopback(monkeypatch):
    """`bench.py --gpus 8` outside a launcher re-runs itself under torch.distributed.run with
    8 processes on 127.0.0.1, the same arguments, and returns the child's exit code."""
    import subprocess
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return Done()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr("sys.argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    assert bench.relaunch_distributed(8) == 7
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]


def test_cpu_baseline_reference_calibration(tmp_path):
    """the port's GPU-box rate is also reported in the reference's own terms,
    through the ratio tests/golden/make_cpu_calibration.py measured against the reference on
    identical rows (hashes equal); absent record -> None."""
    cal = json.loads(open(bench.CALIBRATION_PATH).read())
    assert cal["hashes_equal"] is True and cal["tuples"] >= 1000
    assert 0.5 < cal["port_over_reference"] < 3.0
    eq = bench.reference_equivalent(1000.0)
    assert abs(eq["value"] * cal["port_over_reference"] - 1000.0) < 1e-6
    assert bench.reference_equivalent(1000.0, str(tmp_path / "none.json")) is None

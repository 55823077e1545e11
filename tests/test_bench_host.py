"""bench.py host helpers (no GPU): the flow-like generator's device (torch) and numpy
forms agree and start at example_input/ips.csv's first row; PMC traffic lookup keys."""
import json

import numpy as np
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

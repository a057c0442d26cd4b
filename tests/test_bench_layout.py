"""bench.py's BIGANN layouts and metric fields, on the CPU.

* configs[3] (BIGANN-100M "sharded across 4 MI355X") is served as 4-rank
  layouts once there are 4 or 8 ranks: ws / 4 replicas, rank r holding shard
  r % 4 of replica r // 4.  configs[4] keeps its 8-way layout (modelled peers
  below 8 ranks).
* The block reports the reference's metric, queries / (online + maintenance at
  the harness's cadence, private-search.go:216-240), beside the region's own
  rate and the online-only rate.
* A gloo world-4 run checks the rank-to-shard mapping and that the replica
  groups (bench.replica_groups) reduce over exactly the ranks of one layout.
"""
import importlib.util
import os
import pathlib
import socket
import tempfile

import torch.multiprocessing as mp

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("pm_bench", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bigann_layout_mapping():
    b = _bench()
    for ws, layout, replicas in ((1, 1, 1), (2, 2, 1), (4, 4, 1), (8, 4, 2)):
        lays = [b.bigann_layout("config3_bigann_100m", ws, r) for r in range(ws)]
        for r, lay in enumerate(lays):
            assert lay["layout"] == layout and lay["replicas"] == replicas, (ws, r, lay)
            assert lay["shard"] == r % layout and lay["replica"] == r // layout
            assert not lay["modelled"]
            assert lay["combine"] == (layout > 1)
            assert r in lay["group_ranks"] and len(lay["group_ranks"]) == (layout if layout > 1 else 1)
        # every (replica, shard) pair exactly once: each replica holds the whole DB
        assert sorted((x["replica"], x["shard"]) for x in lays) == [(q, s) for q in range(replicas) for s in range(layout)]
    for ws in (1, 2, 4):
        lay = b.bigann_layout("config4_bigann_1b", ws, ws - 1)
        assert lay["layout"] == 8 and lay["modelled"] and not lay["combine"] and lay["replicas"] == 1
        assert lay["shard"] == ws - 1
    lay = b.bigann_layout("config4_bigann_1b", 8, 5)
    assert lay["layout"] == 8 and not lay["modelled"] and lay["combine"] and lay["group_ranks"] == list(range(8))


def test_bigann_rates_fields():
    b = _bench()
    # 18 sessions x 36 queries in 0.25 s with no maintenance in the region; one
    # client's preprocessing 0.2 s; SupportBatchNum 19,560 -> a 326-query window
    r = b.bigann_rates(1, 18, 36, 0.25, 0.0, 0.2, 19560)
    assert set(r) == {"private_queries_per_s", "private_queries_per_s_at_maintenance_cadence",
                      "private_queries_per_s_online_only", "maintenance_window_queries"}
    assert r["maintenance_window_queries"] == 326.0
    assert r["private_queries_per_s"] == r["private_queries_per_s_online_only"] == round(18 * 36 / 0.25, 2)
    want = 18 * 36 / (0.25 + 36 * 18 * 0.2 / 326)
    assert abs(r["private_queries_per_s_at_maintenance_cadence"] - want) < 0.01
    assert r["private_queries_per_s_at_maintenance_cadence"] < r["private_queries_per_s"]
    r2 = b.bigann_rates(2, 18, 36, 0.25, 0.0, 0.2, 19560)   # two replicas: twice the job's queries
    assert r2["private_queries_per_s"] == round(2 * 18 * 36 / 0.25, 2)


def test_ip_shards_closed_form():
    """configs[0] sharded by rows (bench.ip_shard_rows / ip_closed_form): the
    shards cover [0, N) once, and their mod-2^32 sums add up to
    TestInnerProduct's 1,178,525,696 at N = 1e8, D = 128."""
    b = _bench()
    assert b.ip_closed_form(0, b.C0_N, b.C0_D) == b.C0_SUM == 1_178_525_696
    for ws in (1, 2, 3, 4, 8):
        spans = [b.ip_shard_rows(b.C0_N, ws, r) for r in range(ws)]
        assert spans[0][0] == 0 and spans[-1][1] == b.C0_N
        assert all(spans[i][1] == spans[i + 1][0] for i in range(ws - 1))
        assert sum(b.ip_closed_form(r0, r1, b.C0_D) for r0, r1 in spans) % (1 << 32) == b.C0_SUM
    # small case against the definition
    assert b.ip_closed_form(3, 11, 8) == sum((i + j) * j for i in range(3, 11) for j in range(8)) % (1 << 32)


def test_step_grid_threads():
    """bench.step_grid_threads restates pm_engine.cpp's k_step launch: the
    configs[2] batch (32 sub-queries over 16 partitions) takes 3 gather helpers
    per sub-query; a 96-sub-query search step has no room for any."""
    b = _bench()
    assert b.step_grid_threads(32, 16) == (64 + 16 + 96) * 1024
    assert b.step_grid_threads(96, 16) == (192 + 16) * 1024
    assert b.step_grid_threads(120, 16) == (240 + 16) * 1024


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _bench()
        lay = b.bigann_layout("config3_bigann_100m", world, rank)
        # the world-4 layout is one 4-way replica; replica groups of 2 ranks
        # rehearse the 8-rank case (two 4-way replicas) on four processes
        groups = b.replica_groups(dist, world, 2)
        g = groups[rank // 2]
        t = torch.tensor([1 << rank], dtype=torch.int64)
        dist.all_reduce(t, group=g)
        # configs[0] over the world: this rank's shard sum, reduced like the bench's gloo path
        r0, r1 = b.ip_shard_rows(b.C0_N, world, rank)
        ip = torch.tensor([b.ip_closed_form(r0, r1, b.C0_D)], dtype=torch.int64)
        dist.all_reduce(ip)
        with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
            f.write(f"{lay['layout']}|{lay['shard']}|{lay['replica']}|{int(t.item())}|{int(ip.item()) & 0xFFFFFFFF}")
    finally:
        dist.destroy_process_group()


def test_replica_groups_gloo_world4():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank, args=(4, _free_port(), d), nprocs=4, join=True)
        res = [open(os.path.join(d, f"r{r}.txt")).read().split("|") for r in range(4)]
    for r in range(4):
        assert res[r][:3] == ["4", str(r), "0"], res
        pair = (1 << (r & ~1)) | (1 << ((r & ~1) + 1))
        assert int(res[r][3]) == pair, res   # the group reduced over its own two ranks only
        assert int(res[r][4]) == 1_178_525_696, res   # configs[0]'s shard sums over the world

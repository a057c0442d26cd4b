"""The N > 1 combine cannot hang or split the ranks:
world-size-2 gloo runs on the CPU.

* agreed_setup: one rank's setup fails at once while the other's takes a
  while and succeeds; both ranks reach the agreement, both raise
  RcclUnavailable, the successful one tears its result down, and both go on
  to the next collective (every rank finishes).
* combiner_with_fallback through the real library: rank 1's pm_rccl_create is
  failed by injection (PM_FAULT_RCCL_CREATE=1, i.e. that rank never joins);
  rank 0's attempt ends within the bound (here: no device, or the
  rccl_timeout_s bound), the ranks agree and both fall back to the gloo
  combine, then complete a sum over the fallback group."""
import os
import socket
import tempfile
import time

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_agree(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pacmann_amd.shard import RcclUnavailable, agreed_setup
        torn = []

        def setup():
            if rank == 1:
                raise RuntimeError("injected: rank 1 cannot create its communicators")
            time.sleep(1.0)   # rank 0 is still inside its (bounded) setup when rank 1 fails
            return "handle0"
        try:
            agreed_setup(setup, teardown=torn.append)
            outcome = "used"
        except RcclUnavailable as e:
            outcome = f"fallback: {e}"
        t = torch.tensor([rank + 1], dtype=torch.int64)
        dist.all_reduce(t)   # the ranks are still in step
        with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
            f.write(f"{outcome}|{torn}|{int(t.item())}")
    finally:
        dist.destroy_process_group()


def test_agreed_setup_one_rank_fails():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_agree, args=(2, _free_port(), d), nprocs=2, join=True)
        res = [open(os.path.join(d, f"r{r}.txt")).read().split("|") for r in range(2)]
    assert res[0][0].startswith("fallback") and "another rank" in res[0][0], res
    assert res[1][0].startswith("fallback") and "injected" in res[1][0], res
    assert res[0][1] == "['handle0']" and res[1][1] == "[]", res   # rank 0 released what it had made
    assert res[0][2] == res[1][2] == "3", res


def _rank_native(rank, world, port, out_dir, fault="PM_FAULT_RCCL_CREATE", bound=10):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if rank == 1:
        # PM_FAULT_RCCL_CREATE: this rank's pm_rccl_create fails at once (it never joins);
        # PM_FAULT_RCCL_BLOCK: its init never settles, the bounded wait runs out
        os.environ[fault] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pacmann_amd as pm
        from pacmann_amd.shard import combiner_with_fallback
        pm.set_option("rccl_timeout_s", bound)
        t0 = time.perf_counter()
        comb, path, note = combiner_with_fallback([1000, 1000], device=0, prefer="native",
                                                  nccl_group_fn=lambda: None)
        dt = time.perf_counter() - t0
        t = torch.tensor([10 * (rank + 1)], dtype=torch.int64)
        dist.all_reduce(t, group=comb.group)   # the fallback combine's group works on every rank
        with open(os.path.join(out_dir, f"n{rank}.txt"), "w") as f:
            f.write(f"{path}|{note}|{int(t.item())}|{dt:.1f}")
    finally:
        dist.destroy_process_group()


def test_native_combine_falls_back_when_a_rank_fails():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_native, args=(2, _free_port(), d), nprocs=2, join=True)
        res = [open(os.path.join(d, f"n{r}.txt")).read().split("|") for r in range(2)]
    for r in range(2):
        assert res[r][0] == "gloo", res
        assert res[r][1].startswith("native RCCL combine unavailable"), res
        assert res[r][2] == "30", res
        assert float(res[r][3]) < 60, res   # bounded: no rank waited for the one that never joined
    assert "injected fault" in res[1][1], res


def test_native_combine_falls_back_when_a_rank_blocks():
    """rank 1's communicator creation BLOCKS (its init never
    settles: PM_FAULT_RCCL_BLOCK) instead of failing.  Its bounded wait ends
    with PM_ETIMEDOUT after rccl_timeout_s (4 s here), rank 0 waits for it at
    the agreement, both ranks fall back to the gloo combine and both processes
    exit -- within the bound plus slack, with no thread left waiting."""
    t0 = time.monotonic()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_native, args=(2, _free_port(), d, "PM_FAULT_RCCL_BLOCK", 4), nprocs=2, join=True)
        res = [open(os.path.join(d, f"n{r}.txt")).read().split("|") for r in range(2)]
    wall = time.monotonic() - t0
    for r in range(2):
        assert res[r][0] == "gloo", res
        assert res[r][1].startswith("native RCCL combine unavailable"), res
        assert res[r][2] == "30", res
    assert "PM_FAULT_RCCL_BLOCK" in res[1][1] and "not ready after 4 s" in res[1][1], res
    assert 3.5 < float(res[1][3]) < 30, res   # the blocked rank waited out its bound, no longer
    assert wall < 90, wall                     # both processes exited (spawn joined them)

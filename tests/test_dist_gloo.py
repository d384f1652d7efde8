"""world_size-2 gloo run of the multi-GPU path (DESIGN.md §0 row e) on CPU: each rank samples its own
seeded shard, solves it (the CPU oracle stands in for the GPU solver here), and the solutions are
gathered to rank 0; rank 0 must hold both shards in rank order, identical to solving the union in one
process, the other rank holds nothing, and the max-over-ranks / sum-over-ranks reductions must be right.
A second test drives bench.py's own timed loop (barriers, max-over-ranks clock) with the solve injected."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import oracle as O
    from nlotrajectories_amd.dist import gather_solutions, max_over_ranks, rank_world, sum_over_ranks
    from nlotrajectories_amd.problem import BENCHMARKS
    from nlotrajectories_amd.sampling import sample_start_goal

    dist.init_process_group("gloo", rank=rank, world_size=world)
    r_, _, w_ = rank_world()
    assert (r_, w_) == (rank, world)
    p = BENCHMARKS["b2"]["problem"]
    sdf = lambda P: np.sqrt(((np.asarray(P) - 0.5) ** 2).sum(1)) - 0.25
    x0, xg = sample_start_goal(p, 2, seed=7, sdf=sdf, lo=(0, 0), hi=(1, 1), rank=rank)
    rc = O.solve_batch(p, x0, xg, threads=1)
    r = {k: torch.as_tensor(np.asarray(rc[k])) for k in ("X", "U", "S", "cost", "status", "iters")}
    r["x0"] = torch.as_tensor(x0)
    g = gather_solutions(r, keys=("X", "U", "S", "cost", "status", "iters", "x0"))
    if rank != 0:
        assert all(v is None for v in g.values())  # gather to rank 0 only
    t = max_over_ranks(float(rank + 1), "cpu")
    n = sum_over_ranks(int((r["status"] == 0).sum()), "cpu")
    if rank == 0:
        torch.save({k: v for k, v in g.items()} | {"t": t, "n": n}, os.path.join(out_dir, "g.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_gather(tmp_path):
    import oracle as O
    from nlotrajectories_amd.problem import BENCHMARKS
    from nlotrajectories_amd.sampling import sample_start_goal

    world, port = 2, _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    g = torch.load(tmp_path / "g.pt", weights_only=True)
    p = BENCHMARKS["b2"]["problem"]
    sdf = lambda P: np.sqrt(((np.asarray(P) - 0.5) ** 2).sum(1)) - 0.25
    shards = [sample_start_goal(p, 2, seed=7, sdf=sdf, lo=(0, 0), hi=(1, 1), rank=r) for r in range(world)]
    x0 = np.concatenate([s[0] for s in shards])
    xg = np.concatenate([s[1] for s in shards])
    assert not np.allclose(shards[0][0], shards[1][0])  # disjoint seeded shards
    np.testing.assert_array_equal(g["x0"].numpy(), x0)  # rank order
    ref = O.solve_batch(p, x0, xg, threads=2)
    np.testing.assert_array_equal(g["status"].numpy(), ref["status"])
    np.testing.assert_allclose(g["X"].numpy(), ref["X"], atol=0, rtol=0)  # same code, same inputs
    assert g["t"] == 2.0 and g["n"] == int((ref["status"] == 0).sum())


def _bench_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import time

    import bench
    import oracle as O
    from nlotrajectories_amd.dist import gather_solutions, sum_over_ranks
    from nlotrajectories_amd.problem import BENCHMARKS
    from nlotrajectories_amd.sampling import sample_start_goal

    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = BENCHMARKS["b2"]["problem"]
    sdf = lambda P: np.sqrt(((np.asarray(P) - 0.5) ** 2).sum(1)) - 0.25
    x0, xg = sample_start_goal(p, 1, seed=3, sdf=sdf, lo=(0, 0), hi=(1, 1), rank=rank)
    calls = []

    def step():  # the injected solve: the oracle on this rank's shard; rank 1 is slower
        rc = O.solve_batch(p, x0, xg, threads=1)
        time.sleep(0.3 * rank)
        calls.append(1)
        r = {k: torch.as_tensor(np.asarray(rc[k])) for k in ("status", "cost")}
        gather_solutions(r, keys=("status", "cost"))
        return r

    res, elapsed = bench.timed_loop(step, 2, 1, world, lambda: None, "cpu")
    solved = sum_over_ranks(sum(int((x["status"] == 0).sum()) for x in res), "cpu")
    torch.save({"elapsed": elapsed, "calls": len(calls), "solved": solved},
               os.path.join(out_dir, f"b{rank}.pt"))
    dist.destroy_process_group()


def test_bench_timed_loop_two_ranks(tmp_path):
    """bench.timed_loop on 2 gloo ranks: warm-up + exactly K timed steps per rank, and the reported time is
    the max over ranks (both ranks see the slow rank's clock)."""
    world, port = 2, _free_port()
    mp.start_processes(_bench_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r0 = torch.load(tmp_path / "b0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "b1.pt", weights_only=True)
    assert r0["calls"] == r1["calls"] == 3  # 1 warm-up + 2 timed
    assert r0["elapsed"] == r1["elapsed"] >= 0.6  # max over ranks: rank 1 sleeps 0.3 s per timed step
    assert r0["solved"] == r1["solved"]


def test_bench_batch_calls():
    """bench.batch_calls: the timed batches per solve call under continuous batching (<= 4 per call, every
    timed batch exactly once) and one call per batch otherwise."""
    import bench

    assert bench.batch_calls(4, True) == (4, [4])
    assert bench.batch_calls(2, True) == (2, [2])
    assert bench.batch_calls(10, True) == (4, [4, 4, 2])
    assert bench.batch_calls(3, False) == (1, [1, 1, 1])
    for k in range(1, 13):
        G, calls = bench.batch_calls(k, True)
        assert sum(calls) == k and max(calls) <= G <= 4

"""bench.py --gpus N runs N ranks, on the CPU: with no launcher around it (WORLD_SIZE unset),
`bench.py --gpus 2` starts two ranks itself through torch.distributed.run as a child process; --launch-check makes each
rank draw its seeded shard and gather it to rank 0 over the process group (gloo here, RCCL on the GPU node) without
solving.  The line must say n_gpus 2, the process group must hold 2 ranks, and the shards must arrive in rank order.
A launcher that starts another number of ranks than --gpus asks for is an error (exit code 2), not a relabelled line."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    env.update(NLOT_DIST_BACKEND="gloo", OMP_NUM_THREADS="1", **kw)
    return env


def test_gpus_2_self_launches_two_ranks():
    import bench

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check", "--batch", "3",
                        "--seed", "5"], env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == 2 and line["process_group_world_size"] == 2 and line["backend"] == "gloo"
    assert line["self_launched"]
    want = np.concatenate([bench.draw_b6(3, 5, rank)[0] for rank in range(2)])
    np.testing.assert_array_equal(np.array(line["x0"]), want)  # both shards, in rank order
    assert not np.allclose(want[:3], want[3:])  # distinct seeded shards


def test_gpus_1_single_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--launch-check", "--batch", "2"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and not line["self_launched"] and len(line["x0"]) == 2


def test_world_size_mismatch_exits_nonzero():
    """A launcher's WORLD_SIZE that differs from --gpus: exit code 2 before anything runs."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--gpus 2 but the launcher started 1 rank" in r.stderr

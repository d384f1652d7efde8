"""RRT initial guesses computed by the REFERENCE's own RRTInitializer (core/trajectory_initialization.py:58-239) —
runs only where /root/reference exists; the output tests/golden/rrt_golden.json is what travels.

The reference module is imported under the numeric casadi / shapely / matplotlib stubs of make_nlp_golden.py and
driven exactly as scripts/run_benchmark.py:116-127 drives it (N = solver.N + 1 points, the YAML's rrt_bounds,
step_size, max_iter, margin, the body's geometry, sdf_func = the scene's exact MultiObstacle.sdf).  Its only
non-reproducible input, Python's global `random` (never seeded by the reference), is replaced in the module's
namespace by the counter-based stream the restatement and the GPU kernel draw from (oracle/rrt_oracle.py u01:
iteration it draws u(it, 0) for the goal bias, then u(it, 1), u(it, 2) for random.uniform of x and y).  Scenes:
the circle / square scenes of benchmarks 1, 2 and 5 (exact SDFs in numpy); polygon and ring scenes need shapely's
exact distance, absent here, so their RRT stays parity-unpinned.

    python tests/golden/make_rrt_golden.py [--reference /root/reference]
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "..", "oracle"))
from make_nlp_golden import write_stubs  # noqa: E402

M64 = (1 << 64) - 1


def mix64(z):  # splitmix64 finaliser (oracle/rrt_oracle.py, csrc/nlot_rrt.hip)
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


class CounterRandom:
    """Stands in for the `random` module: random() opens iteration it (draw 0), uniform() takes draws 1 and 2."""

    def __init__(self, seed, instance):
        self.key = mix64((seed & M64) ^ mix64(instance))
        self.it, self.k = -1, 0

    def _u(self, k):
        return (mix64(self.key ^ (4 * self.it + k)) >> 11) * 2.0 ** -53

    def random(self):
        self.it += 1
        self.k = 1
        return self._u(0)

    def uniform(self, a, b):
        u = self._u(self.k)
        self.k += 1
        return a + (b - a) * u


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "rrt_golden.json"))
    a = ap.parse_args()
    if not os.path.isdir(a.reference):
        print("reference tree absent; nothing to do")
        return 0
    stub_dir = tempfile.mkdtemp(prefix="nlot_casadi_stub_")
    write_stubs(stub_dir)
    sys.path[:0] = [stub_dir, os.path.join(a.reference, "src")]
    import yaml
    from nlotrajectories.core import trajectory_initialization as TI
    from nlotrajectories.core.config import Config

    bdir = os.path.join(a.reference, "src", "nlotrajectories", "benchmarks")
    rng = np.random.default_rng(31)
    cases = []
    for fn in ("benchmark_1_dot_circle.yaml", "benchmark_2_unicycle_circle.yaml", "benchmark_5_ackermann_circle.yaml"):
        with open(os.path.join(bdir, fn)) as f:
            cfg = Config(**yaml.safe_load(f))
        ini = cfg.solver.initializer.choice
        obstacles = cfg.get_obstacles()
        for inst in range(4):
            x0 = np.array(cfg.body.start_state, float)
            xg = np.array(cfg.body.goal_state, float)
            if inst:
                x0[:2] += rng.uniform(-0.05, 0.05, 2)
                xg[:2] += rng.uniform(-0.05, 0.05, 2)
            seed = 1000  # one stream per scene; instance = the batch index (nlot_rrt_init, rrt_oracle.rrt_one)
            TI.random = CounterRandom(seed, inst)
            init = TI.RRTInitializer(N=cfg.solver.N + 1, x0=x0, x_goal=xg, dt=cfg.solver.dt, sdf_func=obstacles.sdf,
                                     bounds=ini.rrt_bounds, geometry=cfg.body.create_geometry(), step_size=ini.step_size,
                                     max_iter=ini.max_iter, margin=ini.margin)
            try:
                X = init.get_initial_guess()
                ok = True
            except RuntimeError:  # "RRT failed to find a path within max_iter."
                X, ok = None, False
            cases.append({"yaml": fn, "instance": inst, "seed": seed, "x0": x0.tolist(), "xg": xg.tolist(),
                          "bounds": np.asarray(ini.rrt_bounds, float).tolist(), "step_size": ini.step_size,
                          "max_iter": ini.max_iter, "margin": ini.margin, "ok": ok,
                          "X_init": None if X is None else np.asarray(X, float).tolist(),
                          "tree_nodes": len(init._last_tree) if init._last_tree else 0})
            print(fn, inst, "ok" if ok else "failed", cases[-1]["tree_nodes"], "tree nodes")
    with open(a.out, "w") as f:
        json.dump({"generator": "tests/golden/make_rrt_golden.py (the reference's RRTInitializer, counter-based draws)",
                   "cases": cases}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

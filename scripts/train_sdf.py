"""Train the learned SDF of a benchmark config the way run_benchmark.py does (nlotrajectories_amd.trainer),
seeded, on the GPU, and write its weights (MlpWeights npz) plus the loss history.

    python scripts/train_sdf.py benchmark_6_ackermann_wave.yaml nlotrajectories_amd/data/b6_mlp128_seed0.npz [seed]

The config is read from tests/golden/nlp_golden.json (the reference's own Config dumps; the YAML files do not
travel to the GPU box) or from a YAML path."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlotrajectories_amd.config import Config  # noqa: E402
from nlotrajectories_amd.nn import MlpWeights  # noqa: E402
from nlotrajectories_amd.trainer import train_for_config  # noqa: E402

name, out = sys.argv[1], sys.argv[2]
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
if os.path.exists(name):
    cfg = Config.load(name)
else:
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = Config.model_validate(json.load(open(os.path.join(root, "tests", "golden", "nlp_golden.json")))["configs"][name])
t = time.time()
model, tr = train_for_config(cfg, seed=seed)
w = MlpWeights.from_module(model)
w.save(out)
log = {"config": name, "seed": seed, "seconds": time.time() - t, "epochs_run": len(tr.history),
       "history": tr.history, "model": cfg.model.model_dump(), "device": str(tr.device)}
json.dump(log, open(os.path.splitext(out)[0] + "_train.json", "w"), indent=1)
print("wrote", out, "in", round(time.time() - t, 1), "s", flush=True)

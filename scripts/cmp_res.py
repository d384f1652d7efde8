"""Compare two step_trace.py result files (status / iterations / cost per instance): exit 1 unless bitwise equal."""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
eq = {k: bool((a[k] == b[k]).all()) for k in ("status", "iters", "cost")}
print(f"{sys.argv[1]} vs {sys.argv[2]}: " + " ".join(f"{k} {'equal' if v else 'DIFFER'}" for k, v in eq.items()) +
      f"; wall {float(a['wall']):.2f} s vs {float(b['wall']):.2f} s")
sys.exit(0 if all(eq.values()) else 1)

cd $GRAFT_REPO_ROOT
timeout -k 10 120 python scripts/latency_probe.py 2>&1 | grep -v amdgpu.ids

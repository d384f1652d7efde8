#!/bin/bash
# Scheduling knobs re-measured on the final tree (product library): speculation in the bulk (NLOT_SPEC_BULK), the
# speculation threshold (NLOT_SPEC_THRESHOLD), the host's run-ahead (NLOT_PIPE), k_ric's attempt cap
# (NLOT_RIC_TRIES); step_trace workload (2 x 32,768); results are bitwise equal across these knobs
OUT=gpurun_out/r05ae
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $OUT
run() {
  local n=$1; shift
  env "$@" timeout -k 10 240 python3 scripts/step_trace.py run 32768 2 32768 $OUT/$n > $OUT/$n.log 2>&1 || exit $?
  echo "$n: $(grep 'traj/s' $OUT/$n.log)"
}
run base X=0
run bulk1 NLOT_SPEC_BULK=1
run bulk3 NLOT_SPEC_BULK=3
run thr4k NLOT_SPEC_THRESHOLD=4096
run thr16k NLOT_SPEC_THRESHOLD=16384
run pipe4 NLOT_PIPE=4
run tries2 NLOT_RIC_TRIES=2
run base2 X=0

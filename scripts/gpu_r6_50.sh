#!/bin/bash
# per-workgroup phases of the assign at small K (D=128 K=64 / 256 against 1024, D=32 K=256):
# where the per-row fixed cost of the sweep's small-K cells goes
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for cfg in "128 64" "128 256" "128 1024" "32 256"; do
  set -- $cfg
  timeout -k 10 200 python -u scripts/assign_timeline.py --n 10000000 --d $1 --k $2 > gpurun_out/r6_50_timeline_d$1_k$2.log 2>&1 || exit $?
done
echo done

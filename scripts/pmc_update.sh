#!/bin/bash
# L2 hit/miss of the headline M-step kernel (counter-only rocprofv3 pass over scripts/kbench.py).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmcu1 gpurun_out/pmcu2
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmcu1 -- python3 scripts/kbench.py --n 20000000 --reps 2 > gpurun_out/pmcu1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/pmcu2 -- python3 scripts/kbench.py --n 20000000 --reps 2 > gpurun_out/pmcu2.log 2>&1 || exit $?
python3 scripts/summarize_prof.py gpurun_out/pmcu1 > gpurun_out/pmcu1.md
python3 scripts/summarize_prof.py gpurun_out/pmcu2 > gpurun_out/pmcu2.md
echo pmc-done

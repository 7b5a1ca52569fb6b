#!/bin/bash
# Round-3 session V: SQ/GRBM counters of the headline step (counter-only pass with the kernel
# trace for durations), N=2e7 rows of the headline shape.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
P="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
rm -rf gpurun_out/pmc_v
timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_v -- \
  python3 bench.py --n 20000000 --steps 3 --warmup 1 --no-also-incremental > gpurun_out/pmc_v.log 2>&1 || exit $?
python3 scripts/summarize_pmc.py gpurun_out/pmc_v > gpurun_out/pmc_v.md && cat gpurun_out/pmc_v.md

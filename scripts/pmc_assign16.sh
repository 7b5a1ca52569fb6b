#!/bin/bash
# A/B of assign16 pipeline variants + PMC counters of the default and the diagnostics.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=${AB_VARIANTS:-16g1v2,16g0v10,16g0v11,16g0v12,16g0v13,32p2}
timeout -k 10 300 python3 scripts/ab_kernels.py --n 20000000 --rounds 5 --variants $V > gpurun_out/ab3.log 2>&1 || exit $?
cat gpurun_out/ab3.log
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_COUNT"
for i in 1 2; do
  eval P=\$P$i
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmca$i -- python3 scripts/ab_kernels.py --n 20000000 --rounds 1 --variants $V > gpurun_out/pmca$i.log 2>&1 || exit $?
done
echo pmc-done

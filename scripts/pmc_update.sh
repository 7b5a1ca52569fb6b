#!/bin/bash
# Update-kernel timing under label patterns + PMC counters (counter-only runs).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 scripts/bench_update.py ${UPD_ARGS:-} > gpurun_out/bench_update.log 2>&1 || exit $?
cat gpurun_out/bench_update.log
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_ADDR_CONFLICT GRBM_COUNT"
P3="SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY"
for i in 1 2 3; do
  eval P=\$P$i
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcu$i -- python3 scripts/bench_update.py --reps 1 --patterns random --n ${UPD_N:-20000000} > gpurun_out/pmcu$i.log 2>&1 || exit $?
done
echo pmc-done

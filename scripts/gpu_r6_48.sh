#!/bin/bash
# counters of the M-step at D = 128 / 384 / 512 (K-split kernel) and 768 (column-slice kernel),
# K=1024 bf16, N=5e6: why the wide widths run at 3.2-3.5 TB/s against 5.5 at D=128
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_COUNT"
P3="FETCH_SIZE"
for d in 128 384 512 768; do
for i in 1 2 3; do
  eval P=\$P$i
  o=gpurun_out/r6_48_pmc_d${d}_$i
  rm -rf $o
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $o -- python3 scripts/assign_sweep.py --n 5000000 --d $d --k 1024 --dtypes bf16 --what mstep > $o.log 2>&1 || exit $?
  python3 scripts/summarize_pmc.py $o --match update > $o.md || exit $?
  rm -rf $o
done
done
echo done

#!/bin/bash
# PMC counters of the assign kernel at one shape (scripts/assign_ab.py, default arm), one
# counter-only rocprofv3 pass per group (--kernel-trace only beside --pmc).
#   pmc_assign.sh <name> <assign_ab args...>  -> gpurun_out/pmca_<name><i>/ and pmca_<name>.md
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
name=$1; shift
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_COUNT"
P3="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
: > gpurun_out/pmca_$name.md
for i in 1 2 3; do
  eval P=\$P$i
  rm -rf gpurun_out/pmca_$name$i
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmca_$name$i -- \
    python3 scripts/assign_ab.py --rounds 1 --reps 3 --arms default "$@" > gpurun_out/pmca_$name$i.log 2>&1 || exit $?
  python3 scripts/summarize_pmc.py gpurun_out/pmca_$name$i --match ${MATCH:-assign16} >> gpurun_out/pmca_$name.md
done
echo pmc-done

#!/bin/bash
# memory-path PMC counters of the assign kernel (TCP/UTCL1/TA), one counter-only rocprofv3
# pass per group:  pmc_assign_mem.sh <name> <assign_ab args...>  -> gpurun_out/pmcm_<name>.md
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
name=$1; shift
P1="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
P2="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_SERIALIZATION_STALL_sum GRBM_GUI_ACTIVE"
P3="TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P4="TA_TA_BUSY_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
P5="TA_FLAT_READ_WAVEFRONTS_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
: > gpurun_out/pmcm_$name.md
for i in ${PASSES:-1 2 3 4 5}; do
  eval P=\$P$i
  rm -rf gpurun_out/pmcm_$name$i
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmcm_$name$i -- \
    python3 scripts/assign_ab.py --rounds 1 --reps 3 --arms default "$@" > gpurun_out/pmcm_$name$i.log 2>&1 || exit $?
  python3 scripts/summarize_pmc.py gpurun_out/pmcm_$name$i --match ${MATCH:-assign16} >> gpurun_out/pmcm_$name.md
done
echo pmc-done

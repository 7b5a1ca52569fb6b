#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_COUNT"
timeout -k 10 300 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc16a -- python3 scripts/ab_kernels.py --n 20000000 --rounds 1 --variants 16g2 > gpurun_out/pmc16a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc16b -- python3 scripts/ab_kernels.py --n 20000000 --rounds 1 --variants 16g2 > gpurun_out/pmc16b.log 2>&1 || exit $?
echo pmc-done

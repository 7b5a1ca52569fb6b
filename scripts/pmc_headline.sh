#!/bin/bash
# PMC counters of the headline Lloyd step's kernels (assign16 + update) on bench data,
# one counter-only rocprofv3 pass per group (no tracing domains with --pmc), N=2e7.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
N=${PMC_N:-20000000}
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_COUNT"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for i in 1 2 3 4; do
  eval P=\$P$i
  rm -rf gpurun_out/pmch$i
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmch$i -- python3 bench.py --n $N --steps 2 --warmup 1 --no-also-incremental --pg auto > gpurun_out/pmch$i.log 2>&1 || exit $?
done
echo pmc-done

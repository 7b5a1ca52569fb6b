#!/bin/bash
# row norms with four loads in flight vs HEAD's kernel, one process
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/ab_ext.py run scripts/abbin/_C_ab_4fd787ba7971.so --what rownorms --n 100000000 --d 128 --rounds 5 --reps 5 > gpurun_out/r6_17_ab_rownorms_d128.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/ab_ext.py run scripts/abbin/_C_ab_4fd787ba7971.so --what rownorms --n 50000000 --d 64 --rounds 5 --reps 5 > gpurun_out/r6_17_ab_rownorms_d64.log 2>&1 || exit $?
echo done

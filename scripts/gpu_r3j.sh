#!/bin/bash
# Round-3 session J: the per-point-offset seed fix (scalar v_add_f32 seeds) against the repro,
# the whole GPU suite, then this tree (PMAJ issue order + one-round-trip prologue) against the
# committed HEAD kernels in one process, and the headline / cfg5 benches.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
REPRO_LAUNCHES=30 run keys_d32_fix 500 python -u scripts/debug/keys_d32_repro.py || exit 1
run pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread || exit 1
AB=scripts/abbin/_C_ab_7868911c10ea.so
run ab_head_d128 200 python -u scripts/ab_ext.py run $AB --n 20000000 --d 128 --k 1024 || exit 1
run ab_head_d256 200 python -u scripts/ab_ext.py run $AB --n 16777216 --d 256 --k 512 || exit 1
run ab_head_d64 200 python -u scripts/ab_ext.py run $AB --n 10000000 --d 64 --k 4096 || exit 1
MIKMEANS_ASSIGN_PMAJ=0 run ab_head_d128_nopmaj 200 python -u scripts/ab_ext.py run $AB --n 20000000 --d 128 --k 1024 || exit 1
MIKMEANS_ASSIGN_PMAJ=0 run ab_head_d256_nopmaj 200 python -u scripts/ab_ext.py run $AB --n 16777216 --d 256 --k 512 || exit 1
run bench 300 python -u bench.py || exit 1
run bench4 300 python -u bench.py --config cfg4 || exit 1
run bench5r 300 python -u bench.py --config cfg5 --resident || exit 1
MIKMEANS_UPDATE_KS=1 run bench5r_ks 300 python -u bench.py --config cfg5 --resident || exit 1
exit 0

cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf1 -- python3 scripts/bench_update.py --reps 1 --patterns random --n 100000000 > gpurun_out/pmcf1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmcf2 -- python3 scripts/bench_update.py --reps 1 --patterns random --n 100000000 > gpurun_out/pmcf2.log 2>&1 || exit $?
echo done

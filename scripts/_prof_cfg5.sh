cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; cd gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d prof5 -o p -- python3 ../bench.py --config cfg5 --steps 5 --warmup 1 > b5.log 2>&1
find prof5 -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} k5.csv
head -6 k5.csv | cut -c1-200

#!/bin/bash
# round 6 (after the packed statistics pass): closing bench lines (headline, cfg2, cfg4, cfg5 streamed / resident) and rocprofv3
# kernel traces of the headline and cfg5 resident
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_15_bench.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --config cfg2 --steps 300 --warmup 30 > gpurun_out/r6_15_bench_cfg2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg4 --steps 20 --warmup 3 > gpurun_out/r6_15_bench_cfg4.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --steps 20 --warmup 3 > gpurun_out/r6_15_bench_cfg5.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config cfg5 --resident --steps 20 --warmup 3 > gpurun_out/r6_15_bench_cfg5r.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r6_15_headline -- python3 bench.py --steps 10 --warmup 3 --no-also-incremental --no-also-bounded > gpurun_out/r6_15_prof_headline.log 2>&1 || exit $?
python3 scripts/summarize_prof.py gpurun_out/prof_r6_15_headline --title "headline (bench.py N=1e8 D=128 K=1024 bf16), rocprofv3, round 6" > gpurun_out/r6_15_rocprof_headline.md || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r6_15_cfg5r -- python3 bench.py --config cfg5 --resident --steps 10 --warmup 3 > gpurun_out/r6_15_prof_cfg5r.log 2>&1 || exit $?
python3 scripts/summarize_prof.py gpurun_out/prof_r6_15_cfg5r --title "cfg5 resident (bench.py --config cfg5 --resident), rocprofv3, round 6" > gpurun_out/r6_15_rocprof_cfg5r.md || exit $?
echo done

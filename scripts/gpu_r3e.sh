#!/bin/bash
# Round-3 session E: smoke, the three benches, then rocprofv3 kernel stats of each config.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log"; return $rc; }
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
run bench 300 python -u bench.py || exit 1
run bench4 300 python -u bench.py --config cfg4 || exit 1
run bench5r 300 python -u bench.py --config cfg5 --resident || exit 1
bash scripts/prof_cfg.sh headline --steps 10 --warmup 3 --no-also-incremental || exit 1
bash scripts/prof_cfg.sh cfg4 --config cfg4 --steps 10 --warmup 3 || exit 1
bash scripts/prof_cfg.sh cfg5r --config cfg5 --resident --steps 10 --warmup 3 || exit 1
exit 0

#!/bin/bash
# rocprofv3 kernel stats of one bench config: prof_cfg.sh <name> <bench args...>
# -> gpurun_out/prof_<name>/ (raw) and gpurun_out/prof_<name>.md (summary)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
name=$1; shift
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -- \
  python3 bench.py "$@" > gpurun_out/prof_$name.log 2>&1 || exit $?
python3 scripts/summarize_prof.py gpurun_out/prof_$name --title "$name: bench.py $*" > gpurun_out/prof_$name.md
tail -3 gpurun_out/prof_$name.log

#!/bin/bash
# the round-end GPU tiers: full pytest -m gpu, then smoke()
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
tag=${1:-full}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
echo done

#!/bin/bash
# Round-3 session L: MFMA issue-order study in the shape microbench (16x16x32 and 32x32x16,
# q-major vs point-block-major, in-kernel clock), then rocprofv3 kernel stats of the three
# bench configs with the PMAJ build.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -14 "gpurun_out/$name.log"; return $rc; }
hipcc -O3 --offload-arch=gfx950 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 scripts/microbench/mfma_shape.hip \
  -o gpurun_out/mfma_shape 2> gpurun_out/mfma_shape_build.log || exit 1
run mfma_order 240 ./gpurun_out/mfma_shape 2048 400 1 || exit 1
bash scripts/prof_cfg.sh headline --steps 10 --warmup 3 --no-also-incremental || exit 1
bash scripts/prof_cfg.sh cfg4 --config cfg4 --steps 10 --warmup 3 || exit 1
bash scripts/prof_cfg.sh cfg5r --config cfg5 --resident --steps 10 --warmup 3 || exit 1
exit 0

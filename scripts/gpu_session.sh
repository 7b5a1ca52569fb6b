#!/bin/bash
# One gpurun session: smoke -> GPU tests -> bench -> rocprof.  Stops at the first
# step that faults, aborts or times out (exit >= 124 or signal); a plain test
# failure (pytest exit 1) does not stop the bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-smoke tests bench prof}; do
  case $s in
    smoke) step smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step pytest_gpu 1200 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ;;
    kern) step pytest_kern 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread ;;
    kbench) step kbench 300 python scripts/kbench.py ${KB_ARGS:-} ;;
    kbench4) step kbench4 300 python scripts/kbench.py --n 10000000 --d 64 --k 4096 ;;
    kbench2) step kbench2 300 python scripts/kbench.py --n 1000000 --d 128 --k 256 --dtype f32 --reps 20 ;;
    mstep) step pytest_mstep 300 python -u -m pytest tests/test_gpu_mstep.py -x -v --timeout 120 --timeout-method thread ;;
    rccl) step pytest_rccl 300 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 120 --timeout-method thread ;;
    multirank) step pytest_multirank 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 400 --timeout-method thread ;;
    memplan) step pytest_memplan 600 python -u -m pytest tests/test_gpu_memplan.py tests/test_gpu_minibatch.py -v --timeout 200 --timeout-method thread ;;
    newkern) step pytest_newkern 600 python -u -m pytest tests/test_gpu_kernels.py -v --timeout 200 --timeout-method thread \
               -k "${NK_SEL:-persistent or wide or transform or d768 or col_absmax or matches_reference or past_1024}" ;;
    init) step pytest_init 300 python -u -m pytest tests/test_gpu_init.py -v --timeout 200 --timeout-method thread ;;
    abr3) for sh in "--d 128 --k 1024 --n 20000000" "--d 64 --k 4096 --n 10000000" "--d 256 --k 512 --n 16777216"; do
            step "ab_r3_$(echo $sh | cut -d' ' -f2)" 300 python -u scripts/ab_ext.py run ${AB_MOD:-scripts/abbin/_C_ab_2c7aa1c1dd03.so} $sh
          done ;;
    bounded) step pytest_bounded 400 python -u -m pytest tests/test_gpu_bounded.py -v --timeout 200 --timeout-method thread ;;
    hamerly) step hamerly 400 python -u scripts/hamerly_ab.py ${HAM_ARGS:-} ;;
    top2ab) step pytest_bounded_p4 400 env MIKMEANS_ASSIGN_TOP2_GEOM=1 python -u -m pytest tests/test_gpu_bounded.py -q --timeout 200 --timeout-method thread
            step hamerly_kpar_p2 400 python -u scripts/hamerly_ab.py --init "k-means||" --iters 40
            step hamerly_kpar_p4 400 env MIKMEANS_ASSIGN_TOP2_GEOM=1 python -u scripts/hamerly_ab.py --init "k-means||" --iters 40 ;;
    hamerly_big) step hamerly_kpar_n1e8 600 python -u scripts/hamerly_ab.py --n 100000000 --init "k-means||" --iters 30 ;;
    hamerly2) step hamerly_kpar 400 python -u scripts/hamerly_ab.py --init "k-means||" --iters 40 ;;
    dp2host) step bench_dp2host 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
               --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --comm host --steps 10 --warmup 2 ;;
    ab_head) step ab_head 300 python -u scripts/assign_ab.py --arms "default;assign_persist=1;assign_geom=4;assign_geom=4,assign_persist=1" ;;
    ab_d256) step ab_d256 300 python -u scripts/assign_ab.py --d 256 --k 512 --n 16777216 \
               --arms "default;assign_geom=3;assign_persist=1;assign_geom=3,assign_persist=1" ;;
    ab_d64) step ab_d64 300 python -u scripts/assign_ab.py --d 64 --k 4096 --n 10000000 --arms "default;assign_persist=1" ;;
    ab_f32) step ab_f32 300 python -u scripts/assign_ab.py --d 128 --k 256 --n 1000000 --dtype f32 --reps 20 \
               --arms "default;assign_persist=1" ;;
    blobs) step blobs 200 python -u scripts/blobs_bench.py ;;
    ab_g256) step ab_g256 400 python -u scripts/assign_ab.py --d 256 --k 512 --n 125000000 --gather 16777216 \
               --arms "default;assign_geom=1;assign_geom=2;assign_geom=3" ;;
    ab_wide) step ab_wide 300 python -u scripts/assign_ab.py --d 768 --k 1024 --n 4000000 --arms "default" ;;
    bench) step bench 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 ;;
    benchauto) step bench_nopg 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --pg auto --no-also-incremental ;;
    bench2) step bench_cfg2 300 python bench.py --config cfg2 --steps 50 --warmup 5 ;;
    bench4) step bench_cfg4 300 python bench.py --config cfg4 --steps 20 --warmup 3 ;;
    bench5) step bench_cfg5 300 python bench.py --config cfg5 --steps 20 --warmup 3 ;;
    bench5r) step bench_cfg5r 300 python bench.py --config cfg5 --resident --steps 20 --warmup 3 ;;
    bench4ts) step bench_cfg4_2s 300 python bench.py --config cfg4 --steps 20 --warmup 3 --kpp-sampling two-stage ;;
    prof5r) cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
          step rocprof5r 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5r -- python3 bench.py --config cfg5 --resident --steps 5 --warmup 1 ;;
    profb) cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
          step rocprof_bounded 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profb -- python3 scripts/hamerly_ab.py --n 20000000 --init "k-means||" --iters 20 ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
          step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -- python3 bench.py --steps 5 --warmup 1 ;;
  esac
done
exit 0

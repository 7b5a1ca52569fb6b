#!/bin/bash
# HBM ceilings (fill / copy / read) beside the blob generator and the column-statistics pass
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/hbm_ceiling.py > gpurun_out/r6_10_hbm_ceiling.log 2>&1

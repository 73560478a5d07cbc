#!/bin/bash
# Sweep the split-K fill target / min K-tiles per split on the ResNet-50 bench (one GPU).
# Each run is bounded by its own timeout; the sweep stops at the first failing run.
set -e
mkdir -p gpurun_out
for tb in ${TBS:-512 1024 2048}; do
  for mk in ${MKS:-4}; do
    TFK_TARGET_BLOCKS=$tb TFK_SPLIT_MIN_KTILES=$mk timeout -k 10 150 python bench.py --steps 20 --warmup 5 \
      > gpurun_out/sweep_tb${tb}_mk${mk}.log 2>&1
    echo "tb=$tb mk=$mk $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_tb${tb}_mk${mk}.log)"
  done
done

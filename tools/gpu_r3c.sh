#!/bin/bash
# halo weight gradient: numerics, micro-bench, ResNet-50 A/B
bash tools/gpu_session.sh \
  "t_hwg:300:python -u -m pytest tests/test_hwgrad_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "hwg_bench:240:python tools/hwgrad_bench.py" \
  "b_resnet:180:python bench.py --steps 30 --warmup 8" \
  "b_resnet_nohwg:180:TFK_HWGRAD=0 python bench.py --steps 30 --warmup 8"

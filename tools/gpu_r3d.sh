#!/bin/bash
bash tools/gpu_session.sh \
  "t_hwg:300:python -u -m pytest tests/test_hwgrad_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "hwg_bench:240:python tools/hwgrad_bench.py" \
  "b_resnet:180:python bench.py --steps 30 --warmup 8" \
  "b_tbig_fp8:180:python bench.py --model transformer-big --fp8 1 --steps 20 --warmup 6" \
  "b_tbig:180:python bench.py --model transformer-big --steps 20 --warmup 6"

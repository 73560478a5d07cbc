#!/bin/bash
bash tools/gpu_session.sh \
  "t_fp8:300:python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "b_ns:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_split:180:TFK_FP8_WGRAD_NOSPLIT=0 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_ns2:180:TFK_FP8_WGRAD_NOSPLIT=128 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_ns3:180:TFK_FP8_WGRAD_NOSPLIT=256 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10"

#!/bin/bash
bash tools/gpu_session.sh \
  "d1:180:python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "t512:180:TFK_FP8_WGRAD_TARGET=512 python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "t128:180:TFK_FP8_WGRAD_TARGET=128 python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "k4:180:TFK_FP8_WGRAD_MIN_KT=4 python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "k16:180:TFK_FP8_WGRAD_MIN_KT=16 python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "d2:180:python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10"

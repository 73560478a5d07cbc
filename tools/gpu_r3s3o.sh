#!/bin/bash
bash tools/gpu_session.sh \
  "a1:180:python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "b1:180:TFK_MXQ_GRID=2048 python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "c1:180:TFK_MXQ_GRID=4096 python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "a2:180:python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "b2:180:TFK_MXQ_GRID=2048 python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10" \
  "c2:180:TFK_MXQ_GRID=4096 python bench.py --model transformer-big --fp8 1 --steps 40 --warmup 10"

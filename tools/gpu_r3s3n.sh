#!/bin/bash
# knob A/B (no code change): attention waves per block, dual-quantizer resident grid
bash tools/gpu_session.sh \
  "tb8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "tb8_w4:180:TFK_ATTN_WAVES=4 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "tb8_g512:180:TFK_MXQ_GRID=512 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "tb8_g2048:180:TFK_MXQ_GRID=2048 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "bert:180:python bench.py --model bert-base --steps 30 --warmup 10" \
  "bert_w4:180:TFK_ATTN_WAVES=4 python bench.py --model bert-base --steps 30 --warmup 10" \
  "tb:180:python bench.py --model transformer-big --steps 30 --warmup 10" \
  "tb_w4:180:TFK_ATTN_WAVES=4 python bench.py --model transformer-big --steps 30 --warmup 10"

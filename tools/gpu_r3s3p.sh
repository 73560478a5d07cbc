#!/bin/bash
# ResNet-50 knob re-check after round 3's kernel changes (alternating, same box)
bash tools/gpu_session.sh \
  "r_a:180:python bench.py --steps 40 --warmup 15" \
  "r_sh8:180:TFK_BN_SHARDS=8 python bench.py --steps 40 --warmup 15" \
  "r_ss075:180:TFK_WGRAD_SPLIT_SCALE=0.75 python bench.py --steps 40 --warmup 15" \
  "r_ss15:180:TFK_WGRAD_SPLIT_SCALE=1.5 python bench.py --steps 40 --warmup 15" \
  "r_ws3:180:TFK_WGRAD_STREAMS=3 python bench.py --steps 40 --warmup 15" \
  "r_b:180:python bench.py --steps 40 --warmup 15" \
  "r_persist:180:TFK_G4_PERSIST=1 python bench.py --steps 40 --warmup 15"

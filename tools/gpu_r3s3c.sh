#!/bin/bash
bash tools/gpu_session.sh \
  "b_tbig8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "opprof8:300:python tools/op_profile.py --model transformer-big --batch 32 --fp8 1 --steps 2" \
  "opprof16:300:python tools/op_profile.py --model transformer-big --batch 32 --steps 2"

#!/bin/bash
# Round-3 re-entry check: GPU tests, then benches of every model at HEAD.
bash tools/gpu_session.sh \
  "tests:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "b_resnet:180:python bench.py --steps 30 --warmup 8" \
  "b_resnet_fc:180:python bench.py --steps 30 --warmup 8 --force-comm" \
  "b_tbig:180:python bench.py --model transformer-big --steps 30 --warmup 8" \
  "b_tbig_fp8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 8" \
  "b_bert:180:python bench.py --model bert-base --steps 30 --warmup 8"

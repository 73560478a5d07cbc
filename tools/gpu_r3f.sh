#!/bin/bash
bash tools/gpu_session.sh \
  "t_sk:300:python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k splitk" \
  "b_resnet:180:python bench.py --steps 30 --warmup 8" \
  "b_tbig:180:python bench.py --model transformer-big --steps 20 --warmup 6" \
  "b_tbig8:180:python bench.py --model transformer-big --fp8 1 --steps 20 --warmup 6" \
  "b_bert:180:python bench.py --model bert-base --steps 20 --warmup 6"

#!/bin/bash
bash tools/gpu_session.sh \
  "t_models:600:python -u -m pytest tests/test_transformer_models_gpu.py tests/test_parity_gpu.py tests/test_device_schedule.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "b_tbig:180:python bench.py --model transformer-big --steps 30 --warmup 10" \
  "b_tbig8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_bert:180:python bench.py --model bert-base --steps 30 --warmup 10"

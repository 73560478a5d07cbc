#!/bin/bash
bash tools/gpu_session.sh \
  "t_fp8:400:python -u -m pytest tests/test_fp8_gpu.py tests/test_transformer_ops_gpu.py -x -q -s --timeout 200 --timeout-method thread" \
  "t_models:600:python -u -m pytest tests/test_transformer_models_gpu.py tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread" \
  "b_tbig8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_tbig8_np:180:TFK_FP8_MX_PRODUCERS=0 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_tbig:180:python bench.py --model transformer-big --steps 30 --warmup 10"

#!/bin/bash
bash tools/gpu_session.sh \
  "t_fp8:300:python -u -m pytest tests/test_fp8_gpu.py tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "t_models:600:python -u -m pytest tests/test_transformer_models_gpu.py tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread" \
  "b_tbig8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_tbig8_noprod:180:TFK_FP8_MX_PRODUCERS=0 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_tbig:180:python bench.py --model transformer-big --steps 30 --warmup 10" \
  "b_bert:180:python bench.py --model bert-base --steps 30 --warmup 10" \
  "prof_tbig8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/t8c -o t8 -- python3 bench.py --model transformer-big --fp8 1 --steps 8 --warmup 5"

#!/bin/bash
bash tools/gpu_session.sh \
  "t_ops:500:python -u -m pytest tests/test_fp8_gpu.py tests/test_transformer_ops_gpu.py tests/test_kernels_gpu.py -x -q -s --timeout 200 --timeout-method thread -k 'not conv_fwd_dgrad_wgrad'" \
  "t_models:600:python -u -m pytest tests/test_transformer_models_gpu.py tests/test_parity_gpu.py tests/test_resnet_gpu.py -x -q --timeout 300 --timeout-method thread" \
  "b_r50:180:python bench.py --steps 40 --warmup 15" \
  "b_r50_noflip:180:TFK_FLIP_GROUP=0 python bench.py --steps 40 --warmup 15" \
  "b_tbig8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_tbig8_np:180:TFK_FP8_MX_PRODUCERS=0 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_tbig:180:python bench.py --model transformer-big --steps 30 --warmup 10"

#!/bin/bash
bash tools/gpu_session.sh \
  "t_ops:400:python -u -m pytest tests/test_transformer_ops_gpu.py tests/test_transformer_models_gpu.py tests/test_device_schedule.py tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread" \
  "tb:180:python bench.py --model transformer-big --steps 30 --warmup 10" \
  "tb_at:180:TFK_EMB_ATOMIC=1 python bench.py --model transformer-big --steps 30 --warmup 10" \
  "tb8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "bert:180:python bench.py --model bert-base --steps 30 --warmup 10" \
  "bert_at:180:TFK_EMB_ATOMIC=1 python bench.py --model bert-base --steps 30 --warmup 10"

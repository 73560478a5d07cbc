#!/bin/bash
# attention dropout v2 (one hash per 4 elements, unmasked interior tiles) + MX quantizer v3 (coalesced q_c lines)
bash tools/gpu_session.sh \
  "t_ops:600:python -u -m pytest tests/test_transformer_ops_gpu.py tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "mxq:120:python tools/mxq_bench.py" \
  "attn:180:python tools/attn_bench.py" \
  "t_models:600:python -u -m pytest tests/test_transformer_models_gpu.py tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread" \
  "b_tbig:180:python bench.py --model transformer-big --steps 30 --warmup 10" \
  "b_tbig8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_bert:180:python bench.py --model bert-base --steps 30 --warmup 10" \
  "prof_tbig8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/t8 -o t8 -- python3 bench.py --model transformer-big --fp8 1 --steps 8 --warmup 5"

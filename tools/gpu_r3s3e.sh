#!/bin/bash
# LN+MX loads-up-front, LN backward row pipelining, AdamW v2 (A/B), ResNet-50 re-check, GEMM-vs-hipBLASLt table
bash tools/gpu_session.sh \
  "t_k:300:python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k 'adamw or lamb or sgd or layernorm or mx_epilogue'" \
  "b_tbig8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_tbig8_adam1:180:TFK_ADAMW_V2=0 python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_tbig:180:python bench.py --model transformer-big --steps 30 --warmup 10" \
  "b_bert:180:python bench.py --model bert-base --steps 30 --warmup 10" \
  "b_r50:180:python bench.py --steps 40 --warmup 15" \
  "prof_tbig:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/tb3 -o tb -- python3 bench.py --model transformer-big --steps 8 --warmup 5" \
  "gemm:400:python tools/gemm_bench.py --iters 30"

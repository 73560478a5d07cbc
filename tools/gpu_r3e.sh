#!/bin/bash
# profiles: ResNet-50 per-op + kernel trace; Transformer-big fp8 kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
bash tools/gpu_session.sh \
  "t_hwg:300:python -u -m pytest tests/test_hwgrad_gpu.py -x -q --timeout 120 --timeout-method thread -k stem" \
  "hwg_bench:240:python tools/hwgrad_bench.py" \
  "b_resnet:180:python bench.py --steps 30 --warmup 8" \
  "opprof:300:python tools/op_profile.py --model resnet50 --batch 256 --steps 2 --out gpurun_out/opprof_r3.jsonl" \
  "prof_resnet:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/rn -o rn -- python3 bench.py --steps 8 --warmup 5" \
  "prof_tbig8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/t8 -o t8 -- python3 bench.py --model transformer-big --fp8 1 --steps 8 --warmup 5" \
  "prof_tbig:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/tb -o tb -- python3 bench.py --model transformer-big --steps 8 --warmup 5"

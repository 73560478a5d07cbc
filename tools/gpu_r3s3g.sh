#!/bin/bash
# elementwise dropout 4-per-hash masks + LayerNorm-backward consumer bias gradient: full suite + benches
bash tools/gpu_session.sh \
  "suite:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "b_tbig8:180:python bench.py --model transformer-big --fp8 1 --steps 30 --warmup 10" \
  "b_tbig:180:python bench.py --model transformer-big --steps 30 --warmup 10" \
  "b_bert:180:python bench.py --model bert-base --steps 30 --warmup 10" \
  "b_r50:180:python bench.py --steps 40 --warmup 15" \
  "prof_tbig8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/t8d -o t8 -- python3 bench.py --model transformer-big --fp8 1 --steps 8 --warmup 5"

#!/bin/bash
# final kernel traces at HEAD for profiles/
bash tools/gpu_session.sh \
  "prof_bert:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bert4 -o bert -- python3 bench.py --model bert-base --steps 8 --warmup 5" \
  "prof_tb:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/tb4 -o tb -- python3 bench.py --model transformer-big --steps 8 --warmup 5" \
  "prof_tb8:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/t84 -o t8 -- python3 bench.py --model transformer-big --fp8 1 --steps 8 --warmup 5"

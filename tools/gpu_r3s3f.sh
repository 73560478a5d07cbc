#!/bin/bash
# round-end rehearsal: whole GPU suite + smoke, then ResNet-50 kernel trace and the fp8 per-op profile
bash tools/gpu_session.sh \
  "suite:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "prof_r50:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof/rn3 -o rn -- python3 bench.py --steps 8 --warmup 5" \
  "opprof8:300:python tools/op_profile.py --model transformer-big --batch 32 --fp8 1 --steps 2"

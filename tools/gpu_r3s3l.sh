#!/bin/bash
# round-end rehearsal at HEAD: whole GPU suite, smoke, the driver's bench command
bash tools/gpu_session.sh \
  "suite:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py --gpus 1 --steps 20 --warmup 5" \
  "b_bert:180:python bench.py --model bert-base --steps 30 --warmup 10"

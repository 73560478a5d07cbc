#!/bin/bash
# Split-K fill target sweep for one model: MODEL=bert-base TBS="256 512 1024" tools/sweep_splitk_model.sh
set -e
mkdir -p gpurun_out
for tb in ${TBS:-512 1024}; do
  TFK_TARGET_BLOCKS=$tb timeout -k 10 150 python bench.py --model ${MODEL:-bert-base} --steps 20 --warmup 5 \
    > gpurun_out/sweep_${MODEL:-bert-base}_tb${tb}.log 2>&1
  echo "model=${MODEL:-bert-base} tb=$tb $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_${MODEL:-bert-base}_tb${tb}.log)"
done

set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fp8_gpu.py > gpurun_out/r3/t9.log 2>&1 &&
timeout -k 10 400 python tools/fp8_bench.py > gpurun_out/r3/fp8c.log 2>&1 &&
timeout -k 10 300 python bench.py --model transformer-big --steps 30 --warmup 10 > gpurun_out/r3/b_tfm_bf16.log 2>&1 &&
timeout -k 10 300 python bench.py --model transformer-big --steps 30 --warmup 10 --fp8 1 > gpurun_out/r3/b_tfm_fp8.log 2>&1

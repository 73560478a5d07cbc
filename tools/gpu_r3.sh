set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py -k "g4_fp8 or exact or epilogues" > gpurun_out/r3/t8.log 2>&1 &&
timeout -k 10 400 python tools/fp8_bench.py > gpurun_out/r3/fp8b.log 2>&1

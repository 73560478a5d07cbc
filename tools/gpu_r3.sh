set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_parity_gpu.py tests/test_kernels_gpu.py tests/test_bench_gpu.py > gpurun_out/r3/t4.log 2>&1 &&
timeout -k 10 200 env TFK_BN_PREMASK=0 python bench.py --steps 50 --warmup 20 > gpurun_out/r3/b_pm0.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 20 > gpurun_out/r3/b_pm1.log 2>&1 &&
timeout -k 10 200 env TFK_BN_PREMASK=0 python bench.py --steps 50 --warmup 20 > gpurun_out/r3/b_pm0b.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 20 > gpurun_out/r3/b_pm1b.log 2>&1

set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_halo_gpu.py > gpurun_out/r3/t6.log 2>&1 &&
timeout -k 10 120 python tools/halo_bench.py > gpurun_out/r3/hbench2.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_parity_gpu.py tests/test_kernels_gpu.py tests/test_transformer_models_gpu.py tests/test_transformer_ops_gpu.py > gpurun_out/r3/t6b.log 2>&1 &&
timeout -k 10 200 env TFK_HALO=0 python bench.py --steps 50 --warmup 20 > gpurun_out/r3/b_h0.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 20 > gpurun_out/r3/b_h1.log 2>&1 &&
timeout -k 10 200 env TFK_HALO=0 python bench.py --steps 50 --warmup 20 > gpurun_out/r3/b_h0b.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 50 --warmup 20 > gpurun_out/r3/b_h1b.log 2>&1 &&
timeout -k 10 200 python bench.py --model bert-base --steps 30 --warmup 10 > gpurun_out/r3/b_bert2.log 2>&1 &&
timeout -k 10 200 python bench.py --model transformer-big --steps 30 --warmup 10 > gpurun_out/r3/b_tfm2.log 2>&1

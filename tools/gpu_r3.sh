set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_tfk_comm_gpu.py tests/test_mwms_gpu.py > gpurun_out/r3/t1.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/r3/b_nocomm.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 30 --warmup 10 --force-comm > gpurun_out/r3/b_comm.log 2>&1

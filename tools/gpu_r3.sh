set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_bench_gpu.py tests/test_tfjob_gpu.py "tests/test_parity_gpu.py::test_fullwidth_dropout_on_gradient_cosine" > gpurun_out/r3/t3.log 2>&1

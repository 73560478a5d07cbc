export TMPDIR=/tmp; O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_kernels_gpu.py -k "fp8 or mx or splitk or dgrad" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 200 python bench.py --model transformer-big --steps 10 --warmup 4 > $O/tb.log 2>&1 &&
timeout -k 10 200 python bench.py --model transformer-big --fp8 1 --steps 10 --warmup 4 > $O/tb_fp8.log 2>&1 &&
timeout -k 10 300 python tools/linear_ab.py --iters 20 --rounds 2 > $O/linear_ab.jsonl 2> $O/linear_ab.err &&
timeout -k 10 300 python tools/wgrad_blas_ab.py --iters 10 --rounds 2 > $O/wgrad_ab.jsonl 2> $O/wgrad_ab.err

set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_device_schedule.py tests/test_transformer_ops_gpu.py tests/test_transformer_models_gpu.py > gpurun_out/r3/t2.log 2>&1 &&
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/r3/b_bert.log 2>&1 &&
timeout -k 10 300 python bench.py --model transformer-big --steps 20 --warmup 5 > gpurun_out/r3/b_tfm.log 2>&1 &&
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 --graph 0 > gpurun_out/r3/b_bert_eager.log 2>&1 &&
timeout -k 10 300 python bench.py --model transformer-big --steps 20 --warmup 5 --graph 0 > gpurun_out/r3/b_tfm_eager.log 2>&1

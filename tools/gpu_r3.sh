set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python tools/ext_bench.py > gpurun_out/r3/ext.log 2>&1

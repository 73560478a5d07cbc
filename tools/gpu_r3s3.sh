# round-3 session-3 GPU pass: fp8 quantizer tests, quantizer micro-bench, the GPU suite, benches.
# A GPU step that times out / aborts / faults ends the script (no further GPU work).
set -o pipefail
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/fp8_tests.log; fatal $rc fp8
timeout -k 10 120 python tools/mxq_bench.py > gpurun_out/mxq.jsonl 2>&1; rc=$?; cat gpurun_out/mxq.jsonl; fatal $rc mxq
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r3s3.log 2>&1; rc=$?; tail -n 3 gpurun_out/gputest_r3s3.log; fatal $rc suite
for spec in "r50::" "r50fc::--force-comm" "tb:--model transformer-big:" "tb8:--model transformer-big --fp8 1:"; do
  name=${spec%%:*}; rest=${spec#*:}; a=${rest%%:*}; b=${rest#*:}
  timeout -k 10 240 python bench.py $a $b --steps 40 --warmup 15 > gpurun_out/b_$name.json 2>gpurun_out/b_$name.err; rc=$?
  echo "$name rc=$rc $(tail -c 600 gpurun_out/b_$name.json)"; fatal $rc $name
done

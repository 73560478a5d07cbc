#!/bin/bash
# Full GPU tier on one MI355X box (round-end shape): pytest -m gpu with per-test timeouts, then smoke().
export TMPDIR=/tmp
O=${1:-gpurun_out/suite}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
exit $rc

#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, each under its own kill timer) over the
# pointwise-GEMM probe and the dense GEMM probe. Writes under gpurun_out/.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
for prog in pw_probe gemm_probe; do
  ARGS=""; [ $prog = pw_probe ] && ARGS="--reps 5"
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/${prog}_kt -o kt -- python3 $R/tools/$prog.py $ARGS > $O/${prog}_kt.log 2>&1 || exit 3
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/${prog}_p1 -o p1 -- python3 $R/tools/$prog.py $ARGS > $O/${prog}_p1.log 2>&1 || exit 4
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/${prog}_p2 -o p2 -- python3 $R/tools/$prog.py $ARGS > $O/${prog}_p2.log 2>&1 || exit 5
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $O/${prog}_p3 -o p3 -- python3 $R/tools/$prog.py $ARGS > $O/${prog}_p3.log 2>&1 || exit 6
done
echo pmc done

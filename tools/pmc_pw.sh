cd /tmp && export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pw_kt -o kt -- python3 $R/tools/pw_probe.py > $R/gpurun_out/pw_kt.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/pw_p1 -o p1 -- python3 $R/tools/pw_probe.py > $R/gpurun_out/pw_p1.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $R/gpurun_out/pw_p2 -o p2 -- python3 $R/tools/pw_probe.py > $R/gpurun_out/pw_p2.log 2>&1 || exit 5
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pw_p3 -o p3 -- python3 $R/tools/pw_probe.py > $R/gpurun_out/pw_p3.log 2>&1 || exit 6
echo pmc done

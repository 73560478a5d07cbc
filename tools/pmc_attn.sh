#!/bin/bash
# rocprofv3 passes over the attention kernels (tools/attn_bench.py): counter list, kernel trace,
# then one PMC group per run, each under its own kill timer. Writes under gpurun_out/.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/attn_kt -o kt -- python3 $R/tools/attn_bench.py > $O/attn_kt.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/attn_p1 -o p1 -- python3 $R/tools/attn_bench.py > $O/attn_p1.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM -d $O/attn_p2 -o p2 -- python3 $R/tools/attn_bench.py > $O/attn_p2.log 2>&1 || exit 5
echo pmc done

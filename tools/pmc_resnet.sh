#!/bin/bash
# rocprofv3 PMC passes over one eager ResNet-50 bs256 training step (tools/op_profile.py): one counter
# group per run, each under its own kill timer; tools/pmc_derived.py joins them per kernel.
# Writes under $PMC_OUT (default gpurun_out/pmc_r50/; the databases run to ~100 MB: summarise them on the box).
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=${PMC_OUT:-$R/gpurun_out/pmc_r50}
mkdir -p $O
P="python3 $R/tools/op_profile.py --model resnet50 --steps 1 --warmup 1 --top 0"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/p1 -o p1 -- $P > $O/p1.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SALU -d $O/p2 -o p2 -- $P > $O/p2.log 2>&1 || exit 5
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/p3 -o p3 -- $P > $O/p3.log 2>&1 || exit 6
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/p4 -o p4 -- $P > $O/p4.log 2>&1 || exit 7
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/p5 -o p5 -- $P > $O/p5.log 2>&1 || exit 8
echo pmc done

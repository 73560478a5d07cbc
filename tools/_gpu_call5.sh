export TMPDIR=/tmp; O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 300 python tools/linear_ab.py --iters 20 --rounds 2 > $O/linear_ab.jsonl 2> $O/linear_ab.err &&
TFK_LIB_GEMM=1 timeout -k 10 200 python bench.py --model transformer-big --steps 10 --warmup 4 > $O/tb_lib1.log 2>&1 &&
TFK_LIB_GEMM=0 timeout -k 10 200 python bench.py --model transformer-big --steps 10 --warmup 4 > $O/tb_lib0.log 2>&1 &&
TFK_LIB_GEMM=0 TFK_G5=9 timeout -k 10 200 python bench.py --model transformer-big --steps 10 --warmup 4 > $O/tb_lib0_g5.log 2>&1 &&
TFK_LIB_GEMM=1 timeout -k 10 200 python bench.py --model bert-base --steps 10 --warmup 4 > $O/bb_lib1.log 2>&1 &&
TFK_LIB_GEMM=0 timeout -k 10 200 python bench.py --model bert-base --steps 10 --warmup 4 > $O/bb_lib0.log 2>&1 &&
TFK_G5=9 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/r50_g5.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/r50.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e/prof -o r50 -- python3 bench.py --steps 8 --warmup 5 > gpurun_out/r5e/prof_r50.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e/prof -o tbig -- python3 bench.py --model transformer-big --steps 8 --warmup 5 > gpurun_out/r5e/prof_tbig.log 2>&1

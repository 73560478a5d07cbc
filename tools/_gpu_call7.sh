export TMPDIR=/tmp; O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "tail_split or splitk" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 200 python bench.py --model transformer-big --steps 10 --warmup 4 > $O/tb.log 2>&1 &&
cd /tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o tbig -- python3 bench.py --model transformer-big --steps 8 --warmup 5 > $O/prof_tbig.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o tbig8 -- python3 bench.py --model transformer-big --fp8 1 --steps 8 --warmup 5 > $O/prof_tbig8.log 2>&1

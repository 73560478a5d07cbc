export TMPDIR=/tmp; O=gpurun_out/r5c; mkdir -p $O
set -o pipefail
timeout -k 10 240 python bench.py --model transformer-big --force-comm --steps 6 --warmup 3 --report-update --graph 0 > $O/tbig_fc_eager.log 2>&1 &&
timeout -k 10 240 python bench.py --model transformer-big --force-comm --steps 6 --warmup 3 --report-update > $O/tbig_fc_graph.log 2>&1 &&
timeout -k 10 240 python tools/ps_capture_diag.py --variant none -- --model bert-base --strategy ps --ps-transport rccl --force-comm --steps 6 --warmup 3 --report-update > $O/bert_ps_graph.log 2>&1 &&
timeout -k 10 240 python bench.py --model bert-base --strategy ps --ps-transport rccl --force-comm --steps 6 --warmup 3 --report-update --graph 0 > $O/bert_ps_eager.log 2>&1 &&
timeout -k 10 300 python tools/tile_ab.py --iters 20 --rounds 2 --dirs fwd,conv --tiles 256x256,g5,g5s,g5t > $O/tile_g5t.jsonl 2> $O/tile_g5t.err

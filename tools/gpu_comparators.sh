set -o pipefail
O=gpurun_out/cmp
mkdir -p $O
timeout -k 10 200 python bench.py --via-operator > $O/via_op.log 2>&1; echo "via_op rc=$?"
for m in bert-base transformer-big; do
  for pr in bf16 autocast; do
    timeout -k 10 150 python tools/stock_transformer.py --model $m --precision $pr > $O/stock_${m}_${pr}.log 2>&1; echo "$m $pr rc=$?"
  done
done
timeout -k 10 150 python tools/stock_resnet.py --precision bf16 > $O/stock_r50_bf16.log 2>&1; echo "r50 bf16 rc=$?"
timeout -k 10 150 python tools/stock_resnet.py --precision autocast > $O/stock_r50_ac.log 2>&1; echo "r50 ac rc=$?"
grep -h "{" $O/*.log | grep -v Traceback | cut -c1-400

export TMPDIR=/tmp; O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 240 python tools/graph_memset_probe.py --replays 40 > $O/probe.jsonl 2> $O/probe.err || exit 1
python - <<'PY' || exit 0
import json, sys
rows = [json.loads(l) for l in open("gpurun_out/r5b/probe.jsonl") if '"variant"' in l]
print(rows)
bad = {r["variant"]: r["bad_replays"] for r in rows}
# go on to the real captured step only if the probe reproduced the memset-ordering problem
sys.exit(0 if (bad.get("plain", 1) == 0 and (bad.get("fork", 0) > 0 or bad.get("rccl", 0) > 0)) else 3)
PY
echo "probe reproduced the memset ordering fault; running the fixed captured step" > $O/decision.txt
timeout -k 10 240 python bench.py --model transformer-big --force-comm --steps 6 --warmup 3 --report-update > $O/mwms_fc_fixed.log 2>&1

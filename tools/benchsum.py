"""Summarise bench.py JSON lines from log files: value, ms/step, hipgraph, loss (one row per file)."""
import json
import sys

for path in sys.argv[1:]:
    try:
        rows = [json.loads(l) for l in open(path) if l.startswith("{") and '"metric"' in l]
    except OSError as e:
        print(f"{path}: {e}")
        continue
    if not rows:
        print(f"{path}: no bench line")
        continue
    d = rows[-1]
    print(f"{path}: {d['value']} {d['unit']} {d['ms_per_step']} ms/step median {d.get('step_ms', {}).get('median')} "
          f"graph={d['config'].get('hipgraph')} loss={d.get('loss')}")

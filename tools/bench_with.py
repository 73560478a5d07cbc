#!/usr/bin/env python3
"""bench.py with native A/B switches applied first: --set NAME=INT calls lib().NAME(INT) (e.g.
g5_set=9, g8_set=1, gemm_set_shortk=4) before the model is built; everything else goes to bench.py.
A/B against plain `bench.py` in the same gpurun session.

    python tools/bench_with.py --set g5_set=9 --model transformer-big --steps 20 --warmup 5
"""
import argparse
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--set", action="append", default=[], help="NAME=INT: lib().NAME(INT)")
a, rest = ap.parse_known_args()
for kv in a.set:
    name, val = kv.split("=", 1)
    getattr(lib(), name)(int(val))
sys.argv = [os.path.join(ROOT, "bench.py")] + rest
runpy.run_path(sys.argv[0], run_name="__main__")

#!/usr/bin/env python3
"""ResNet-50 bench with the weight-gradient fork grouping of runtime.streams set from the command
line: --defer 0|1, --flush-every N (forks per N residual blocks); the rest goes to bench.py.
A/B against plain `bench.py` in the same gpurun session."""
import argparse
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tensorflow_k8s_amd.runtime import streams  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--defer", type=int, default=1)
ap.add_argument("--flush-every", type=int, default=1)
a, rest = ap.parse_known_args()
streams.DEFER = bool(a.defer)
streams.FLUSH_EVERY = a.flush_every
sys.argv = [os.path.join(ROOT, "bench.py")] + rest
runpy.run_path(sys.argv[0], run_name="__main__")

#!/usr/bin/env python3
"""bench.py against a given library build (timing-only variants under tools/variants/):
  python tools/bench_with_lib.py <lib.so> [bench.py args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning-2048_amd")]
from g2048 import _native as N  # noqa: E402

N.LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
import bench  # noqa: E402

bench.main()

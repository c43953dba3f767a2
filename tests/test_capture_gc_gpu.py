"""Garbage collection inside a hipGraph capture (round 6): bench.py's driver command once failed
its conv leg's loop capture with "operation failed due to a previous error during capture" --
a collection during the capture freed an earlier leg's graph, whose destructor
(hipGraphExecDestroy) is an unsafe call on the capturing thread.  g2048.dist.graph_capture, which
every capture of the package and of bench.py goes through, collects before the capture and keeps
the collector off during it.  Here: an old graph in a reference cycle, freed by a collection in
the middle of a plain torch.cuda.graph capture, invalidates it (run in a child process: a failed
capture leaves the stream unusable); the same under graph_capture records and replays fine."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import gc, sys
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/reinforcement-learning-2048_amd"]
import torch
from g2048.dist import graph_capture
x = torch.ones(1 << 16, device="cuda")

def old_graph_in_a_cycle():
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        x.mul_(1.0)
    g.replay()
    box = {"g": g}
    box["self"] = box  # only the cyclic collector frees it
    torch.cuda.synchronize()

gc.disable()
old_graph_in_a_cycle()
g2 = torch.cuda.CUDAGraph()
if sys.argv[2] == "plain":
    with torch.cuda.graph(g2):
        x.add_(1.0)
        gc.collect()  # frees the old graph in the middle of the capture
        x.add_(1.0)
else:
    with graph_capture(g2):
        x.add_(1.0)
        gc.collect()  # a no-op for the old graph: graph_capture collected it first
        x.add_(1.0)
g2.replay()
torch.cuda.synchronize()
print("replayed", float(x[0]))
"""


@pytest.mark.parametrize("form", ["plain", "graph_capture"])
def test_collection_during_capture(form):
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT, form], capture_output=True, text=True,
                         timeout=120)
    if form == "plain":
        # the hazard itself (if this runtime ever makes hipGraphExecDestroy capture-safe, the
        # plain form passes too and this half of the test only documents the history)
        if out.returncode == 0:
            pytest.xfail("this HIP runtime tolerates a graph destroyed during a capture")
        assert "capture" in out.stderr, out.stderr[-2000:]
    else:
        assert out.returncode == 0, out.stderr[-2000:]
        assert "replayed 3.0" in out.stdout

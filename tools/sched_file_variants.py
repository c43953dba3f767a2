#!/usr/bin/env python3
"""Timing-only library variants (tools/variants/) that differ from the in-tree build in ONE
source's machine-scheduler strategy: for each (source, strategy) pair, that source's object is
rebuilt with the strategy and linked with the other sources' in-tree objects.
  python tools/sched_file_variants.py src1.hip,src2.hip strategy1,strategy2"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402

G.build()  # the in-tree objects
objdir = os.path.join(os.path.dirname(G.LIB), ".objs")
out = os.path.join(ROOT, "tools", "variants")
os.makedirs(out, exist_ok=True)
srcs, strategies = sys.argv[1].split(","), sys.argv[2].split(",")


def one(pair):
    src, st = pair
    path = os.path.join(G.CSRC, src)
    # a strategy name, or "opt:<llvm option>" for any other -mllvm scheduling option
    knob = st[4:] if st.startswith("opt:") else f"--amdgpu-sched-strategy={st}"
    flags = [f for f in G.HIPFLAGS if f != "-shared"] + ["-mllvm", knob]
    obj = os.path.join(out, f"{src}.{st.replace('opt:', '').replace('=', '').replace('-', '')}.o")
    subprocess.run([G.HIPCC, *flags, "-c", path, "-o", obj], check=True)
    objs = [obj if f == src else os.path.join(objdir, f + ".o") for f in G.SRCS]
    tag = st.replace("opt:", "").replace("=", "").replace("-", "")
    lib = os.path.join(out, f"libg2048_{src.replace('.hip', '')}_{tag}.so")
    link = [f for f in G.HIPFLAGS if f in ("--offload-arch=gfx950", "-shared", "-fPIC")]
    subprocess.run([G.HIPCC, *link, "-o", lib, *objs], check=True)
    return lib


with ThreadPoolExecutor(max_workers=8) as ex:
    for lib in ex.map(one, [(s, t) for s in srcs for t in strategies]):
        print(lib)

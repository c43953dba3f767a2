"""Instruction counts per region of the rollout kernel's lean loop, from a marker build:
    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -DG2048_ISA_MARKS \\
          tools/rollexp.hip -o /tmp/roll_marks.s
    python tools/isa_regions.py /tmp/roll_marks.s
Counts every instruction between consecutive ';; region X' markers inside the main loop (two
4-step quads per iteration: the figures are summed over 8 steps, and over both quads' Philox
blocks), split into VALU / SALU / VMEM / LDS / other.  The auto-reset block is counted as if taken
every step; the wave takes it on the steps where one of its 64 boards ends an episode.  The markers fix the instruction order, so the counts describe the marker build; the
timed library is built without them."""
import re
import sys
from collections import Counter, defaultdict

KERNEL = "_ZN12_GLOBAL__N_114k_rollout_leanILb0ELb0ELb1ELi31ELi4EEEvNS_8StepArgsE"  # <kSum=0, kP410=0, kQR=1, all stores>


def kind(op):
    if op.startswith(("buffer_", "global_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait/nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "SALU"
    return "VALU"


def main(path, dump=None):
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if l.startswith(KERNEL + ":"))
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    f = lines[st:en]
    # the main loop: the largest body from a loop header to the last branch back to it
    best = None
    for head, l in enumerate(f):
        if "Loop Header" not in l:
            continue
        label = l.split(":")[0]
        backs = [i for i, x in enumerate(f) if label in x and ("s_branch" in x or "s_cbranch" in x)]
        if backs and (best is None or max(backs) - head > best[1] - best[0]):
            best = (head, max(backs))
    head, tail = best
    region = "loop_head"
    per = defaultdict(Counter)
    for l in f[head:tail + 1]:
        t = l.strip()
        m = re.match(r";; region (\w+)", t)
        if m:
            region = m.group(1)
            continue
        if dump == region and t and not t.startswith(";;#ASM"):
            print("   ", t)
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        per[region][kind(t.split()[0])] += 1
    tot = Counter()
    print(f"{'region':14s} {'all':>5s}  " + "  ".join(f"{k:>8s}" for k in ("VALU", "SALU", "VMEM", "LDS", "wait/nop", "branch")))
    for r, c in per.items():
        tot.update(c)
        print(f"{r:14s} {sum(c.values()):5d}  " + "  ".join(f"{c[k]:8d}" for k in ("VALU", "SALU", "VMEM", "LDS", "wait/nop", "branch")))
    print(f"{'loop total':14s} {sum(tot.values()):5d}  " + "  ".join(f"{tot[k]:8d}" for k in ("VALU", "SALU", "VMEM", "LDS", "wait/nop", "branch")))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)

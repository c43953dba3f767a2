"""Static audit of hipcc's output for the VMEM-store data hazard on gfx950: a store of more than
8 bytes (dwordx3 / dwordx4) reads its data VGPRs late, and a write of those VGPRs within the next
two wait states can land before the read -- the store then writes the new value (seen on
k_rollout_lean's board store at 1M+ boards, under store-queue back-pressure).

What is checked: every instruction whose first operand is a VGPR destination -- VALU (v_*),
LDS reads (ds_read* / ds_load*, ds_*_rtn*) and VMEM loads (buffer_ / global_ / flat_ / scratch_
load*, returning into vdst).  A VALU writer inside the window is a HAZARD (audit() counts it; the
ISA's hazard table and LLVM's GCNHazardRecognizer list VALU writers only).  A load writer is
reported as a NOTE and not counted: its data returns through the memory pipeline tens of cycles
after issue, long after the store's data read; hipcc itself counts such a load as a wait state.
The scan follows control flow for the two wait states: it falls through labels, takes both paths
of an s_cbranch_* and the target of an s_branch, and stops at s_endpgm / s_setpc.  Each
instruction is one wait state; s_nop N is N + 1.

Limits (the 1M-board rollout-vs-oracle GPU tests stay the real check): an indirect branch
(s_setpc) ends the scan, and the window is the documented two wait states -- a hazard that needs
more would not be seen.  Usage: python tools/store_hazard_audit.py file.s [...]"""
import re
import sys

STORE = re.compile(r"^\s*(buffer|global|flat|scratch)_store_dword(x3|x4)\s+(\S+?),\s*(\S+?),")
REG = re.compile(r"v\[(\d+):(\d+)\]")
# instructions whose first operand is a VGPR destination
WRITER = re.compile(r"^\s*(v_\w+|ds_(?:read|load)\w*|ds_\w+_rtn\w*|(?:buffer|global|flat|scratch)_load\w*)"
                    r"\s+(?:v(\d+)|v\[(\d+):(\d+)\])(?:\s|,|$)")
LABEL = re.compile(r"^([.\w$]+):")
BRANCH = re.compile(r"^s_(c?)branch\w*\s+([.\w$]+)")


def _labels(lines):
    return {m.group(1): i for i, l in enumerate(lines) for m in [LABEL.match(l.strip())] if m}


def _scan(lines, labels, j, states, lo, hi, seen):
    """Instructions reachable from line j within 2 - states wait states that write v[lo:hi]."""
    hits = []
    while states < 2 and j < len(lines):
        if (j, states) in seen:
            return hits
        seen.add((j, states))
        t = lines[j].strip()
        j += 1
        if not t or t.startswith((";", ".")) or LABEL.match(t):
            continue
        if t.startswith(("s_endpgm", "s_setpc")):
            return hits
        n = re.match(r"s_nop\s+(\d+)", t)
        if n:
            states += int(n.group(1)) + 1
            continue
        w = WRITER.match(t)
        if w:
            a = int(w.group(2) or w.group(3))
            b = int(w.group(2) or w.group(4))
            if a <= hi and b >= lo:
                hits.append((t, states))
        b = BRANCH.match(t)
        if b and b.group(2) in labels:
            hits += _scan(lines, labels, labels[b.group(2)], states + 1, lo, hi, seen)
            if not b.group(1):  # s_branch: no fall-through
                return hits
        states += 1
    return hits


def audit(path, notes=None):
    """The number of VALU writes of a wide store's data VGPRs within two wait states; load
    writers in the same window are appended to `notes` (when given) and printed as notes."""
    lines = open(path).read().split("\n")
    labels = _labels(lines)
    kernel, bad = None, 0
    for i, l in enumerate(lines):
        k = re.match(r"^(_Z\w+):", l)
        if k:
            kernel = k.group(1)
        m = STORE.match(l)
        if not m:
            continue
        # buffer_store data, vaddr, ...; global/flat_store vaddr, data, ...
        r = REG.match(m.group(3) if m.group(1) == "buffer" else m.group(4))
        if not r:
            continue
        lo, hi = int(r.group(1)), int(r.group(2))
        for t, states in _scan(lines, labels, i + 1, 0, lo, hi, set()):
            what = "HAZARD" if t.startswith("v_") else "note (load)"
            print(f"{path}:{i + 1}: {what} in {kernel}\n    {l.strip()}\n    {t}  ({states} wait states)")
            if t.startswith("v_"):
                bad += 1
            elif notes is not None:
                notes.append((kernel, l.strip(), t))
    return bad


if __name__ == "__main__":
    total = sum(audit(p) for p in sys.argv[1:])
    print(f"{total} store(s) whose data VGPRs a VALU op rewrites within 2 wait states")
    sys.exit(1 if total else 0)

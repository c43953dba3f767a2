"""Static audit of hipcc's output for the VMEM-store data hazard on gfx950: a store of more than
8 bytes (dwordx3 / dwordx4) reads its data VGPRs late, and a VALU write of those VGPRs within the
next two instructions (fewer than two wait states) can land before the read -- the store then
writes the new value (seen on k_rollout_lean's board store at 1M+ boards, under store-queue
back-pressure).  Usage: python tools/store_hazard_audit.py file.s [...]"""
import re
import sys

STORE = re.compile(r"^\s*(buffer|global|flat)_store_dword(x3|x4)\s+(\S+?),\s*(\S+?),")
REG = re.compile(r"v\[(\d+):(\d+)\]")
DST = re.compile(r"^\s*(v_\w+)\s+v(\d+)\b|^\s*(v_\w+)\s+v\[(\d+):(\d+)\]")


def audit(path):
    lines = open(path).read().split("\n")
    kernel, bad = None, 0
    for i, l in enumerate(lines):
        if re.match(r"^_Z\w+:$", l) or re.match(r"^\w+:$", l) and not l.startswith("."):
            kernel = l[:-1]
        m = STORE.match(l)
        if not m:
            continue
        # buffer_store data, vaddr, ...; global/flat_store vaddr, data, ...
        r = REG.match(m.group(3) if m.group(1) == "buffer" else m.group(4))
        if not r:
            continue
        lo, hi = int(r.group(1)), int(r.group(2))
        states, j = 0, i + 1
        while states < 2 and j < len(lines):
            t = lines[j].strip()
            j += 1
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            n = re.match(r"s_nop\s+(\d+)", t)
            if n:
                states += int(n.group(1)) + 1
                continue
            d = DST.match(t)
            if d:
                a = int(d.group(2) or d.group(4))
                b = int(d.group(2) or d.group(5))
                if a <= hi and b >= lo:
                    bad += 1
                    print(f"{path}:{i + 1}: {kernel}\n    {l.strip()}\n    {t}  ({states} wait states)")
            states += 1
    return bad


if __name__ == "__main__":
    total = sum(audit(p) for p in sys.argv[1:])
    print(f"{total} store(s) whose data VGPRs a VALU rewrites within 2 wait states")
    sys.exit(1 if total else 0)

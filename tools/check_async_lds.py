"""Static check of the inline-asm asynchronous LDS reads in a kernel's ISA.

The fused MLP kernels issue ds_read_b128 through inline asm and wait for them
explicitly (s_waitcnt lgkmcnt(0)); the compiler believes the destination
registers are written when the asm issues. This script flags any instruction
between such a read and its drain that reads or writes one of the pending
destination VGPRs (a stale read, or a register the late data would clobber).

    python tools/check_async_lds.py build/asm/mlp_x3.s
"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    if m:
        return {int(m.group(1))}
    return set()


def _parse(t):
    op = t.split()[0]
    ops = [x.strip() for x in t[len(op):].split(",")]
    used = set()
    for o in ops:
        used |= regs(o.split()[0] if o else "")
    return op, ops, used


def _scan_edge(lines, start, pending, path, src):
    """Reads still pending at a backward branch (src) flow to its target: check the
    target's instructions up to the first lgkmcnt(0) drain."""
    bad = 0
    for j in range(start, len(lines)):
        t = lines[j].strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        op, ops, used = _parse(t)
        if op == "s_waitcnt" and "lgkmcnt(0)" in t:
            break
        if op == "ds_read_b128":
            hit = regs(ops[0]) & set(pending)
        elif op.startswith("s_") and not op.startswith("s_waitcnt"):
            continue
        else:
            hit = used & set(pending)
        if hit:
            print(f"{path}:{j + 1}: '{t}' touches regs {sorted(hit)} still pending at the "
                  f"loop branch on line {src + 1}")
            bad += 1
    return bad


def main(path):
    lines = open(path).read().split("\n")
    labels = {}
    for i, raw in enumerate(lines):
        m = re.match(r"^(\.?[A-Za-z_$][\w.$]*):", raw.strip())
        if m:
            labels[m.group(1)] = i
    pending = {}   # reg -> line of the asm read
    in_asm = False
    bad = 0
    for i, raw in enumerate(lines):
        t = raw.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        if op == "s_waitcnt" and "lgkmcnt(0)" in t:
            pending.clear()
            continue
        ops = [x.strip() for x in t[len(op):].split(",")]
        used = set()
        for o in ops:
            used |= regs(o.split()[0] if o else "")
        if in_asm and op == "ds_read_b128":
            dst = regs(ops[0])
            clash = dst & set(pending)
            if clash:
                print(f"{path}:{i + 1}: asm read overwrites pending regs {sorted(clash)}")
                bad += 1
            for r in dst:
                pending[r] = i + 1
            continue
        if (op.startswith("s_cbranch") or op == "s_branch") and pending:
            tgt = labels.get(ops[0])
            if tgt is not None and tgt < i:   # loop back edge
                bad += _scan_edge(lines, tgt, pending, path, i)
            continue
        if op.startswith("s_") and not op.startswith("s_waitcnt"):
            continue
        hit = used & set(pending)
        if hit:
            print(f"{path}:{i + 1}: '{t}' touches pending LDS-read regs {sorted(hit)} "
                  f"(read issued at line {pending[min(hit)]})")
            bad += 1
    print("violations:", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))

"""Static check of the inline-asm asynchronous LDS reads in a kernel's ISA.

The fused MLP kernels issue ds_read_* (b128 fragments, u16 mask words) through
inline asm and wait for them explicitly (s_waitcnt lgkmcnt(0)); every kernel
of the file is checked. The compiler believes the destination
registers are written when the asm issues. This script flags any instruction
between such a read and its drain that reads or writes one of the pending
destination VGPRs or AGPRs (a stale read, or a register the late data would
clobber).

A counted wait lgkmcnt(N) retires the reads with at least N LGKM operations
issued after them (LDS returns in order), unless an SMEM / FLAT operation
(out of order) is outstanding: then only lgkmcnt(0) drains.
The pending set is propagated over the control-flow graph of the .s (basic
blocks split at labels and branches; successors from s_branch / s_cbranch_* /
fall-through), so reads left in flight across a loop back edge or a branch
are followed to every instruction they can reach.

    python tools/check_async_lds.py build/asm/mlp_x3.s
"""
import re
import sys


def regs(tok):
    """VGPRs and AGPRs named by an operand token, as 'v8' / 'a130' strings."""
    m = re.match(r"([va])\[(\d+):(\d+)\]$", tok)
    if m:
        return {f"{m.group(1)}{r}" for r in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    if m:
        return {f"{m.group(1)}{m.group(2)}"}
    return set()


LABEL = re.compile(r"^(\.?[A-Za-z_$][\w.$]*):")


def _instructions(lines):
    """[(line index, text, in_asm)] of the instructions, and labels -> position."""
    out, labels = [], {}
    in_asm = False
    for i, raw in enumerate(lines):
        t = raw.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = LABEL.match(t)
        if m:
            labels[m.group(1)] = len(out)
            out.append((i, None, False))        # label marker
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        out.append((i, t.split(";")[0].strip(), in_asm))
    return out, labels


def _blocks(ins, labels):
    """Basic blocks as (start, end) positions into ins, and successor lists."""
    starts = {0}
    for p, (_, t, _) in enumerate(ins):
        if t is None:
            starts.add(p)
        elif t.startswith("s_branch") or t.startswith("s_cbranch") or t.startswith("s_endpgm") \
                or t.startswith("s_setpc"):
            starts.add(p + 1)
    starts = sorted(s for s in starts if s < len(ins))
    bounds = list(zip(starts, starts[1:] + [len(ins)]))
    at = {s: k for k, (s, _) in enumerate(bounds)}
    succ = []
    for k, (s, e) in enumerate(bounds):
        last = next((ins[p][1] for p in range(e - 1, s - 1, -1) if ins[p][1] is not None), "")
        op = last.split()[0] if last else ""
        nxt = [k + 1] if k + 1 < len(bounds) else []
        if op == "s_branch":
            tgt = labels.get(last.split()[1])
            succ.append([at[tgt]] if tgt in at else [])
        elif op.startswith("s_cbranch"):
            tgt = labels.get(last.split()[1])
            succ.append(nxt + ([at[tgt]] if tgt in at else []))
        elif op in ("s_endpgm", "s_setpc_b64"):
            succ.append([])
        else:
            succ.append(nxt)
    return bounds, succ


LGKM_CNT = re.compile(r"lgkmcnt\((\d+)\)")
SMEM = "__smem__"   # an SMEM / FLAT op since the last full drain: counted waits prove nothing


def _lgkm_op(op):
    """Does the instruction count in lgkmcnt? ('lds' in order, 'smem' not)."""
    if op.startswith("ds_") and op not in ("ds_nop",):
        return "lds"
    if op.startswith("s_load") or op.startswith("s_buffer_load") or op.startswith("flat_") \
            or op.startswith("s_memtime") or op.startswith("s_memrealtime"):
        return "smem"
    return None


def _run_block(ins, s, e, pending, report):
    # pending: register -> (line of the asm read that targets it, number of
    # LGKM ops issued after that read). LDS ops return in order, so a counted
    # wait lgkmcnt(N) retires every read with at least N LGKM ops behind it --
    # unless an SMEM / FLAT op (which may return out of order) is outstanding.
    pending = dict(pending)
    for p in range(s, e):
        line, t, in_asm = ins[p]
        if t is None:
            continue
        op = t.split()[0]
        if op == "s_waitcnt" and "lgkmcnt" in t:
            n = int(LGKM_CNT.search(t).group(1))
            if n == 0:
                pending.clear()
            elif SMEM not in pending:
                pending = {r: v for r, v in pending.items() if v[1] < n}
            continue
        kind = _lgkm_op(op)
        ops = [x.strip() for x in t[len(op):].split(",")]
        used = set()
        for o in ops:
            used |= regs(o.split()[0] if o else "")
        if kind:
            pending = {r: (v if r == SMEM else (v[0], v[1] + 1)) for r, v in pending.items()}
            if kind == "smem" and pending:
                pending[SMEM] = (line + 1, 0)
        if in_asm and op.startswith("ds_read"):
            # another asm read into a pending register is harmless (LDS returns in
            # order: the later read's data land last), e.g. a fragment group the
            # compiler found dead re-using one destination; any other access is not
            dst = regs(ops[0])
            for r in dst:
                pending[r] = (line + 1, 0)
            continue
        if op.startswith("s_") and not op.startswith("s_waitcnt"):
            continue
        hit = used & set(pending)
        if hit:
            report(line, f"'{t}' touches pending LDS-read regs {sorted(hit)} "
                         f"(read issued at line {pending[min(hit)][0]})")
    return pending


def main(path):
    lines = open(path).read().split("\n")
    ins, labels = _instructions(lines)
    bounds, succ = _blocks(ins, labels)
    entry = [dict() for _ in bounds]
    seen = [False] * len(bounds)
    # every kernel of the file: each function symbol's block is an entry (a
    # walk from block 0 alone only reaches the first kernel)
    at = {s: k for k, (s, _) in enumerate(bounds)}
    work = sorted({0} | {at[p] for name, p in labels.items()
                         if not name.startswith(".") and p in at})
    for k in work:
        seen[k] = True
    while work:                                 # forward dataflow to a fixpoint
        k = work.pop()
        out = _run_block(ins, *bounds[k], entry[k], lambda *a: None)
        for n in succ[k]:
            merged = dict(entry[n])
            changed = not seen[n]
            for r, v in out.items():
                if r not in merged:
                    merged[r] = v
                    changed = True
                elif r != SMEM and v[1] < merged[r][1]:   # the most recent on any path
                    merged[r] = v
                    changed = True
            if changed:
                entry[n], seen[n] = merged, True
                work.append(n)
    found = {}

    def report(line, msg):
        found.setdefault(line, msg)
    for k in range(len(bounds)):
        if seen[k]:
            _run_block(ins, *bounds[k], entry[k], report)
    for line in sorted(found):
        print(f"{path}:{line + 1}: {found[line]}")
    print("violations:", len(found))
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))

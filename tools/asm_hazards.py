"""Static check of a kernel's ISA for inline-asm load hazards.

The persistent conv forward (csrc/conv5.hip) issues its weight-fragment loads in inline asm, so the compiler does not know the destination registers are written ASYNCHRONOUSLY: if its
register allocator copies or reuses such a register before the kernel's own `s_waitcnt vmcnt(N)` retires
the load, the late write corrupts whatever lives there (a wrong value -- or an address, and the kernel
faults).  This runs a forward dataflow over the kernel's basic blocks: the state is the in-order queue of
vector-memory operations (loads, stores, atomics; `vmcnt(N)` retires all but the youngest N), merged at
joins by keeping every entry either path may still have in flight.  Every instruction other than a wait
that reads or writes a register of a load that may still be in flight is reported.

    hipcc ... --cuda-device-only -S -o k.s csrc/conv5.hip
    python tools/asm_hazards.py k.s conv_fwd5_kernelILb1
"""
import re
import sys

REG = re.compile(r"\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]")
VMEM = re.compile(r"^(global_|buffer_|scratch_|flat_)")
BR = re.compile(r"^(s_cbranch_\w+|s_branch)\s+(\.LBB\S+)")


def regs_of(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            k, a, b = m.group(3), int(m.group(4)), int(m.group(5))
            out.update((k, i) for i in range(a, b + 1))
    return out


def kernel_insts(path, name):
    """[(line number, label or None, instruction text)] of the kernel's function body; instructions from
    inline asm (between the compiler's ;;#ASMSTART / ;;#ASMEND markers) carry a leading '@'."""
    out, on, in_asm = [], False, False
    for no, ln in enumerate(open(path), 1):
        if re.match(r"^_Z\S*%s\S*:" % re.escape(name), ln):
            on = True
            continue
        if not on:
            continue
        if ";;#ASMSTART" in ln:
            in_asm = True
        if ";;#ASMEND" in ln:
            in_asm = False
        t = ln.split(";")[0].strip()
        if t.startswith(".Lfunc_end"):
            break
        if re.match(r"^\.LBB\S+:$", t):
            out.append((no, t[:-1], None))
        elif t and not t.startswith("."):
            out.append((no, None, ("@" if in_asm else "") + t))
    return out


def blocks_of(insts):
    blocks, cur, label = [], [], None
    for no, lab, t in insts:
        if lab is not None:
            if cur or label is not None:
                blocks.append((label, cur))
            cur, label = [], lab
            continue
        cur.append((no, t))
        if t.startswith("s_branch") or t.startswith("s_cbranch") or t.startswith("s_endpgm") \
                or t.startswith("s_setpc"):
            blocks.append((label, cur))
            cur, label = [], None
    if cur or label is not None:
        blocks.append((label, cur))
    index = {lab: i for i, (lab, _) in enumerate(blocks) if lab is not None}
    succ = []
    for i, (_, body) in enumerate(blocks):
        s = []
        last = body[-1][1] if body else ""
        m = BR.match(last)
        if m:
            s.append(index[m.group(2)])
            if last.startswith("s_cbranch") and i + 1 < len(blocks):
                s.append(i + 1)
        elif not last.startswith("s_endpgm") and i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    return blocks, succ


def merge(a, b):
    """Queues aligned at their youngest end, element-wise union (may-be-in-flight)."""
    if a is None:
        return b
    n = max(len(a), len(b))
    pa = (frozenset(),) * (n - len(a)) + a
    pb = (frozenset(),) * (n - len(b)) + b
    return tuple(x | y for x, y in zip(pa, pb))


def step(queue, t, report=None, no=0):
    from_asm = t.startswith("@")
    t = t.lstrip("@")
    m = re.match(r"s_waitcnt\s+(.*)", t)
    if m:  # (an asm wait that names in-flight registers as operands is the consuming wait: not a use)
        v = re.search(r"vmcnt\((\d+)\)", m.group(1))
        if v:
            n = int(v.group(1))
            if len(queue) > n:
                queue = queue[len(queue) - n:] if n else ()
        return queue
    op = t.split()[0]
    rs = regs_of(t[len(op):])
    pending = set().union(*queue) if queue else set()
    dst = set()
    if VMEM.match(op):
        # only loads written in inline asm are tracked: the compiler orders its own loads' registers itself
        if from_asm and "load" in op and "lds" not in op:
            dst = regs_of(t[len(op):].split(",")[0])
        first = regs_of(t[len(op):].split(",")[0]) if ("load" in op and "lds" not in op) else set()
        bad = (rs - first) & pending
        bad |= first & pending          # any load (asm or compiler) landing on an asm load still in flight
        if bad and report is not None:
            report.append((no, t, sorted(bad)[:4]))
        return queue + (frozenset(dst),)
    bad = rs & pending
    if bad and report is not None:
        report.append((no, t, sorted(bad)[:4]))
    return queue


def main(path, name):
    insts = kernel_insts(path, name)
    blocks, succ = blocks_of(insts)
    ins = [None] * len(blocks)
    ins[0] = ()
    work = [0]
    it = 0
    while work and it < 200000:
        it += 1
        i = work.pop()
        q = ins[i]
        for no, t in blocks[i][1]:
            q = step(q, t)
        for j in succ[i]:
            new = merge(ins[j], q)
            if new != ins[j]:
                ins[j] = new
                work.append(j)
    report = []
    for i, (_, body) in enumerate(blocks):
        q = ins[i]
        if q is None:
            continue
        for no, t in body:
            q = step(q, t, report, no)
    for no, t, regs in report:
        print(f"HAZARD line {no}: {t}   (in-flight load registers {regs})")
    print(f"{name}: {len(report)} hazard(s) over {len(blocks)} blocks ({it} block visits)")
    return len(report)


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1], sys.argv[2]) else 0)

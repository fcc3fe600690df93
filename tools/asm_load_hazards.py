"""Static check of the inline-asm loads (asm_ld16 / asm_ld4 / global_load_dwordx2 in ;;#ASMSTART blocks): hipcc
does not know these loads complete asynchronously, so it may read, copy or overwrite a destination register before
the counted `s_waitcnt vmcnt` that retires the load (e.g. a live-range-split v_mov placed above the wait).  This
scans the gfx950 assembly of the listed kernels in layout order and reports every instruction that touches a
register of a load still in flight.  Usage: python tools/asm_load_hazards.py file.s [kernel-substring ...]"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def functions(asm):
    for m in re.finditer(r"^(_Z[^:\s]+):", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        yield m.group(1), asm[m.end():end]


def check(body):
    """returns [(line_no, instruction, registers)] of hazards"""
    inflight = []  # [dst regs or None (not an asm load)] in issue order (vmcnt retires the oldest first)
    bad = []
    in_asm = False
    for no, raw in enumerate(body.split("\n")):
        line = raw.strip()
        if line.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if line.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not line or line.startswith((";", ".")) or line.endswith(":"):
            continue
        op = line.split()[0]
        m = re.search(r"vmcnt\((\d+)\)", line) if op == "s_waitcnt" else None
        if m:
            n = int(m.group(1))
            while len(inflight) > n:
                inflight.pop(0)
            continue
        if op == "s_waitcnt" and "vmcnt" not in line and "lgkmcnt" not in line and "expcnt" not in line:
            inflight.clear()  # s_waitcnt 0
            continue
        is_vmem = op.startswith(("global_", "buffer_", "flat_", "scratch_"))
        args = line[len(op):].split(";")[0]
        if is_vmem:
            touched = regs(args)
            if "_lds_" in op:  # LDS-DMA (global_load_lds_*): the VGPR operand is the address, the data goes to LDS
                dst, src = set(), touched
            elif "load" in op or "atomic" in op and "glc" in args:
                dst = regs(args.split(",")[0])
                src = touched - dst
            else:
                dst, src = set(), touched
            hit = {r for d in inflight if d for r in d} & (src | dst)
            if hit and not in_asm:
                bad.append((no, line, sorted(hit)))
            inflight.append(dst if (in_asm and "load" in op) else None)
            continue
        touched = regs(args)
        hit = {r for d in inflight if d for r in d} & touched
        if hit:
            bad.append((no, line, sorted(hit)))
    return bad


def check_ring(body, n=16):
    """The weight-ring loaders (talker_tail.hip) publish a slot behind an inline-asm `s_waitcnt vmcnt(n)` that is right
    only if exactly the slot's n LDS-DMA transfers (global_load_lds_*, invisible to hipcc's counters) are the VMEM ops
    issued since the previous slot: in layout order the run of VMEM instructions before each such wait must be n
    global_load_lds and nothing else.  Returns [(line_no, problem)]; the number of waits checked is len of the second
    list."""
    bad, seen = [], []
    in_asm = False
    vmem = []  # VMEM instruction names in layout order since the last wait of any kind
    for no, raw in enumerate(body.split("\n")):
        line = raw.strip()
        if line.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if line.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not line or line.startswith((";", ".")) or line.endswith(":"):
            continue
        op = line.split()[0]
        if op == "s_waitcnt" and in_asm and re.search(rf"vmcnt\({n}\)", line):
            seen.append(no)
            run = 0
            for v in reversed(vmem):
                if "_lds_" not in v:
                    break
                run += 1
            if run != n or any("_lds_" not in v for v in vmem[-n:]):
                bad.append((no, f"vmcnt({n}) after a run of {run} global_load_lds (last VMEM ops {vmem[-(n + 2):]})"))
            continue
        if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            vmem.append(op)
    return bad, seen


def check_r1(body):
    """R1 publication order (MI355X_MICROARCH.md, visibility): every 32-bit sc1 flag store (global_store_dword ... sc1)
    comes after an `s_waitcnt vmcnt(0)` that follows the last sc1 payload store (buffer_store_* ... sc1) before it in
    layout order.  Returns ([(line_no, flag store)], flags checked)."""
    bad, n = [], 0
    undrained = False
    for no, raw in enumerate(body.split("\n")):
        line = raw.strip()
        if not line or line.startswith((";", ".")) or line.endswith(":"):
            continue
        op = line.split()[0]
        if op.startswith("buffer_store") and " sc1" in line:
            undrained = True
        elif op == "s_waitcnt" and "vmcnt(0)" in line:
            undrained = False
        elif op == "global_store_dword" and line.endswith("sc1"):
            n += 1
            if undrained:
                bad.append((no, line))
    return bad, n


def main():
    asm = open(sys.argv[1]).read()
    keys = sys.argv[2:]
    total = 0
    for name, body in functions(asm):
        if keys and not any(k in name for k in keys):
            continue
        if ";;#ASMSTART" not in body:
            continue
        bad = check(body)
        total += len(bad)
        print(f"{name}: {len(bad)} hazard(s)")
        for no, line, r in bad[:20]:
            print(f"   line {no}: {line}   <- v{r}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())

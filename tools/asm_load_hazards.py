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

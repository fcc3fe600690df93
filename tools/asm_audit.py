import re, sys
lines = open(sys.argv[1]).read().split('\n')
ev = []  # (line, kind, regs or count)
inasm = False
for i, l in enumerate(lines):
    if ';;#ASMSTART' in l: inasm = True; continue
    if ';;#ASMEND' in l: inasm = False; continue
    if 'global_load' in l or 'global_store' in l or 'buffer_' in l:
        if inasm and 'global_load' in l:
            m = re.search(r'global_load_\w+\s+v\[?(\d+)(?::(\d+))?\]?', l)
            a = int(m.group(1)); b = int(m.group(2) or m.group(1))
            ev.append((i, 'L', set(range(a, b + 1))))
        else:
            ev.append((i, 'O', None))  # any other vmem op counts in vmcnt too
    m = re.search(r's_waitcnt vmcnt\((\d+)\)', l)
    if m: ev.append((i, 'W', int(m.group(1))))
def regs_of(l):
    out = set()
    for m in re.finditer(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b', l):
        if m.group(3): out.add(int(m.group(3)))
        else: out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    return out
bad = 0
for k, (i, kind, regs) in enumerate(ev):
    if kind != 'L': continue
    # find first wait after i with n <= number of vmem ops issued between the load and the wait (straight-line view)
    younger = 0; done_at = None
    for (j, kj, x) in ev[k + 1:]:
        if kj in ('L', 'O'): younger += 1
        elif kj == 'W' and x <= younger: done_at = j; break
    end = done_at if done_at is not None else len(lines)
    ia = False
    for j in range(i + 1, end):
        l = lines[j]
        if ';;#ASMSTART' in l: ia = True; continue
        if ';;#ASMEND' in l: ia = False; continue
        if ia or l.strip().startswith(';') or not l.strip() or l.strip().startswith('.'): continue
        r = regs_of(l)
        if regs & r:
            print(f"load@{i} v{min(regs)}-{max(regs)} (complete @{done_at}) touched @{j}: {l.strip()}")
            bad += 1
            break
print("asm loads", sum(1 for e in ev if e[1] == 'L'), "touched before completion:", bad)

"""In-flight register check for the asm load rings (tests/test_isa.py helper,
test infrastructure): every control-flow path from an asm load to the wait
that retires it (s_waitcnt vmcnt(N) with N <= the vector memory operations
issued after the load on that path) must leave the load's destination VGPRs
alone; a register copy there reads data that has not landed yet.  The search
follows every branch, including branch combinations the kernel never takes,
so it is exact only for kernels without such correlated branches (the
pipelined k_flat2 sweep); for the other rings it over-reports."""
import re

REG = re.compile(r'v\[(\d+):(\d+)\]|\bv(\d+)\b')


def regs_of(s):
    out = set()
    for a, b, c in REG.findall(s):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def blocks(lines):
    """[(label or None, [instructions])] in layout order."""
    bl, cur = [], [None, []]
    for l in lines:
        if l.endswith(':'):
            if cur[1] or cur[0] is not None:
                bl.append(cur)
            cur = [l[:-1], []]
            continue
        cur[1].append(l)
        if l.startswith(('s_branch', 's_cbranch', 's_endpgm', 's_setpc')):
            bl.append(cur)
            cur = [None, []]
    if cur[1] or cur[0] is not None:
        bl.append(cur)
    return bl


def inflight_hazards(lines, load_re):
    """Instructions that touch the destination VGPRs of an asm ring load (load_re)
    on some control-flow path before a wait retires it (s_waitcnt vmcnt(N) with N
    <= the vector memory operations issued after the load on that path)."""
    bl = blocks(lines)
    label_idx = {b[0]: i for i, b in enumerate(bl) if b[0]}

    def succ(i):
        ins = bl[i][1]
        last = ins[-1] if ins else ''
        nxt = [i + 1] if i + 1 < len(bl) else []
        if last.startswith('s_branch'):
            return [label_idx[last.split()[1]]]
        if last.startswith('s_cbranch'):
            return [label_idx[last.split()[1]]] + nxt
        if last.startswith(('s_endpgm', 's_setpc')):
            return []
        return nxt

    bad = []
    for bi, (_, ins) in enumerate(bl):
        for ii, l in enumerate(ins):
            if not re.match(load_re, l):
                continue
            dest = regs_of(l.split(',')[0])
            stack, seen = [(bi, ii + 1, 0)], set()
            while stack:
                b, k, after = stack.pop()
                if (b, k, after) in seen:
                    continue
                seen.add((b, k, after))
                done = False
                ins_b = bl[b][1]
                while k < len(ins_b):
                    s = ins_b[k]
                    w = re.match(r's_waitcnt\b.*vmcnt\((\d+)\)', s)
                    if w and int(w.group(1)) <= after:
                        done = True
                        break
                    if s.startswith(('global_', 'buffer_', 'flat_')) and 'lds' not in s.split()[0] or \
                            s.startswith('global_load_lds'):
                        if regs_of(s) & dest and not re.match(load_re, s):
                            bad.append((l, s))
                            done = True
                            break
                        after = min(after + 1, 64)
                    elif not s.startswith('s_waitcnt') and regs_of(s) & dest:
                        bad.append((l, s))
                        done = True
                        break
                    k += 1
                if done:
                    continue
                for n in succ(b):
                    stack.append((n, 0, after))
    return bad

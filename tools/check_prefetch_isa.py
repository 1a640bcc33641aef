"""ISA check for the untracked prefetch of the SIFT_FLAG_FAST pyramids:
pyramid_fast.hip's ld2_async / ld1_async (pyr_fast_kernel) and
pyramid_pair.hip's pp_ld1 / pp_ld2 (pyr_pair_kernel).

The loads are inline asm, so the compiler neither waits for them nor knows
their destinations are in flight; an explicit `s_waitcnt vmcnt(N)` names the
destinations as operands.  This compiles each file to gfx950 assembly and,
per kernel instance, walks the control-flow graph from every asm load until
an `s_waitcnt vmcnt` on every path, and flags any instruction on the way that
reads or writes a destination register of the load (a copy before the wait
would read a register the load has not yet written).  It also reports the
VMEM stores on the way.  Exit status 1 on a violation.

    python tools/check_prefetch_isa.py
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (file, kernel, method): "cfg" walks every control-flow path from a load to
# a wait; "linear" follows program order to the next wait (and a rotated
# loop's back edge) -- pyr_fast_kernel issues its prefetch and its wait
# under the same `more` condition in two places, which only program order
# sees as correlated (the CFG walk reports paths that never execute).
SRCS = [('pyramid_fast.hip', 'pyr_fast_kernel', 'linear'), ('pyramid_pair.hip', 'pyr_pair_kernel', 'cfg')]


def flight_linear(L, labels, i):
    waits = [j for j, l in enumerate(L) if re.search(r's_waitcnt vmcnt\(\d+\)', l)]
    w = next((j for j in waits if j > i), None)
    if w is not None:
        return list(range(i + 1, w)), {w}
    for k in range(i + 1, len(L)):
        m2 = re.match(r'\s+s_c?branch\w*\s+(\.LBB\d+_\d+)', L[k])
        if m2 and labels.get(m2.group(1), len(L)) < i:
            h = labels[m2.group(1)]
            w = next(j for j in waits if j > h)
            return list(range(i + 1, k + 1)) + list(range(h, w)), {w}
    return [], set()


def regs(tok):
    m = re.match(r'v\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', tok)
    return {int(m.group(1))} if m else set()


def all_regs(line):
    out = set()
    for t in re.findall(r'v\[\d+:\d+\]|\bv\d+\b', line):
        out |= regs(t)
    return out


def benign(line, hit):
    """A read that cannot observe the in-flight value: hipcc forms 32-bit
    address arithmetic as v_mad_u64_u32 dst, sdst, a, b, v[lo:hi] and uses only
    dst's low half, so the addend's high register is read but never affects
    the result."""
    m = re.match(r'v_mad_u64_u32 v\[(\d+):(\d+)\], \S+, \S+, \S+, v\[(\d+):(\d+)\]', line)
    return bool(m) and hit == {int(m.group(4))} and int(m.group(4)) not in \
        (set(range(int(m.group(1)), int(m.group(2)) + 1)) - {int(m.group(2))})


def flight(L, labels, i):
    """Instruction lines reachable from line i + 1 before an s_waitcnt vmcnt
    (on every path), following branches; returns (lines, waits reached)."""
    seen, waits, todo = set(), set(), [i + 1]
    while todo:
        k = todo.pop()
        while k < len(L):
            if k in seen:
                break
            seen.add(k)
            line = L[k].strip()
            if re.search(r's_waitcnt\s+vmcnt\(\d+\)', line):
                waits.add(k)
                break
            m = re.match(r's_(c?)branch\w*\s+(\.LBB\d+_\d+)', line)
            if m:
                todo.append(labels[m.group(2)])
                if not m.group(1):  # unconditional: no fall-through
                    break
            if line.startswith('s_endpgm'):
                break
            k += 1
    return sorted(seen - waits), waits


def min_vmem_to_waits(L, labels, i, skip=0):
    """0-1 BFS from line i + 1: the fewest VMEM instructions (loads, stores)
    issued on any path from the load at line i to each vmcnt wait it reaches
    after passing `skip` earlier waits (an LDS-DMA ring slot is consumed
    `skip` steps after the one that issues it).  A wait vmcnt(N) only covers
    the load if every path issues >= N of them."""
    from collections import deque
    best, res = {}, {}
    dq = deque([(i + 1, 0, 0)])
    while dq:
        k, c, w = dq.popleft()
        if k >= len(L) or best.get((k, w), 1 << 30) <= c:
            continue
        best[(k, w)] = c
        line = L[k].strip()
        m = re.search(r's_waitcnt\s+vmcnt\((\d+)\)', line)
        if m and int(m.group(1)) > 0 and w < skip:
            w += 1
        elif m:
            res[k] = min(res.get(k, 1 << 30), c)
            continue
        wt = 1 if re.match(r'(buffer|global)_(load|store)', line) else 0
        nxt = []
        mb = re.match(r's_(c?)branch\w*\s+(\.LBB\d+_\d+)', line)
        if mb:
            nxt.append(labels[mb.group(2)])
            if mb.group(1):
                nxt.append(k + 1)
        elif not line.startswith('s_endpgm'):
            nxt.append(k + 1)
        for n in nxt:
            (dq.append if wt else dq.appendleft)((n, c + wt, w))
    return res


def check(src, kname, method):
    asm = f'/tmp/{kname}_check.s'
    subprocess.check_call(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950', '-ffp-contract=off',
                           '-fno-slp-vectorize', '-I' + os.path.join(ROOT, 'include'),
                           '-I' + os.path.join(ROOT, 'sift-gpu_amd', 'build'), '--cuda-device-only', '-S',
                           os.path.join(ROOT, 'sift-gpu_amd', 'csrc', src), '-o', asm], stderr=subprocess.DEVNULL)
    s = open(asm).read()
    bad = 0
    found = 0
    for m in re.finditer(r'^(_ZN4sift\S*%s\S*):' % kname, s, re.M):
        found += 1
        start = m.end()
        L = s[start:s.index('.Lfunc_end', start)].split('\n')
        tag = kname + re.search(r'I(L\S+?)EEv', m.group(1)).group(1)
        labels = {l.split(':')[0]: k for k, l in enumerate(L) if re.match(r'^\.LBB\d+_\d+:', l)}
        # the asm loads: inside ;;#ASMSTART ... ;;#ASMEND blocks
        loads = []
        in_asm = False
        for k, l in enumerate(L):
            if ';;#ASMSTART' in l:
                in_asm = True
            elif ';;#ASMEND' in l:
                in_asm = False
            elif in_asm and re.match(r'\s+(global_load_dword|buffer_load_dword.*\blds\b)', l):
                loads.append(k)
        n = 0
        groups = {}
        for i in loads:
            span, waits = (flight if method == 'cfg' else flight_linear)(L, labels, i)
            if not waits:
                print(f'  {tag}: the load at line {i} reaches no vmcnt wait')
                n += 1
            # an LDS-DMA load writes no register (its first operand is the offset)
            d = set() if re.search(r'\blds\b', L[i]) else regs(L[i].split()[1].rstrip(','))
            for j in span:
                line = L[j].strip()
                if not line or line.startswith(';') or line.startswith('.'):
                    continue
                hit = all_regs(line) & d
                if hit and benign(line, hit):
                    continue
                if hit:
                    n += 1
                    print(f'  {tag}: line {j} touches prefetch register of line {i}: {line}')
            stores = sum(1 for j in span if re.match(r'\s+(buffer|global)_store', L[j]))
            if method == 'cfg':
                # pyramid_pair's LDS-DMA ring: a step's rows are issued two
                # steps ahead of the wait that covers them (the vmcnt(0) at
                # the end covers everything)
                skip = 1 if re.search(r'\blds\b', L[i]) else 0
                for w, c in min_vmem_to_waits(L, labels, i, skip).items():
                    need = int(re.search(r'vmcnt\((\d+)\)', L[w]).group(1))
                    if c < need:
                        n += 1
                        print(f'  {tag}: load at line {i}: a path reaches {L[w].strip()} (line {w}) with only {c} '
                              f'VMEM instructions after the load')
            groups.setdefault(tuple(sorted(waits)), []).append((i, stores))
        for w, ls in sorted(groups.items()):
            print(f'{tag}: loads at {[i for i, _ in ls]} -> waits at {list(w)} '
                  f'({[L[x].strip() for x in w]}), {max(st for _, st in ls)} store instructions on the way')
        print(f'{tag}: {len(loads)} asm loads, {n} violations')
        bad += n
    if not found:
        print(f'{kname}: not found in {src}')
        bad += 1
    return bad


def main():
    bad = sum(check(src, k, m) for src, k, m in SRCS)
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()

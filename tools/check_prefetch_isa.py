"""ISA check for pyramid_fast.hip's untracked prefetch (ld2_async / ld1_async).

Compiles the file to gfx950 assembly and, per pyr_fast_kernel instance, checks
that no instruction touches a prefetch destination register between the
asm load and the explicit `s_waitcnt vmcnt(N)` that ends the column passes,
and reports the VMEM stores in between.  Exit status 1 on a violation.

    python tools/check_prefetch_isa.py
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'sift-gpu_amd', 'csrc', 'pyramid_fast.hip')


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


def main():
    asm = '/tmp/pyramid_fast_check.s'
    subprocess.check_call(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950', '-ffp-contract=off',
                           '-fno-slp-vectorize', '-I' + os.path.join(ROOT, 'include'), '--cuda-device-only', '-S',
                           SRC, '-o', asm], stderr=subprocess.DEVNULL)
    s = open(asm).read()
    bad = 0
    for m in re.finditer(r'^(_ZN4sift\S*pyr_fast_kernel\S*):', s, re.M):
        start = m.end()
        L = s[start:s.index('.Lfunc_end', start)].split('\n')
        tag = re.search(r'ILb(\d)ELb(\d)', m.group(1)).group(0)
        waits = [i for i, l in enumerate(L) if re.search(r's_waitcnt vmcnt\(\d+\)', l)]
        loads = [i for i, l in enumerate(L) if re.search(r'global_load_dword', l)]
        n = 0
        labels = {l.split(':')[0]: k for k, l in enumerate(L) if re.match(r'^\.LBB\d+_\d+:', l)}

        def flight(i):
            """Lines a load's destination stays in flight over, up to its wait.
            A rotated loop puts the loads after the wait: follow the first
            backward branch after the load to its header."""
            w = next((j for j in waits if j > i), None)
            if w is not None:
                return w, list(range(i + 1, w))
            for k in range(i + 1, len(L)):
                m2 = re.match(r'\s+s_c?branch\w*\s+(\.LBB\d+_\d+)', L[k])
                if m2 and labels.get(m2.group(1), len(L)) < i:
                    h = labels[m2.group(1)]
                    w = next(j for j in waits if j > h)
                    return w, list(range(i + 1, k + 1)) + list(range(h, w))
            raise RuntimeError(f'{tag}: no wait for the load at line {i}')

        for i in loads:
            w, span = flight(i)
            d = regs(L[i].split()[1].rstrip(','))
            for j in span:
                line = L[j].strip()
                if line.startswith(';'):
                    continue
                if all_regs(line) & d:
                    n += 1
                    print(f'  {tag}: line {j} touches prefetch register of line {i}: {line}')
        groups = {}
        for i in loads:
            w, span = flight(i)
            groups.setdefault(w, []).append((i, span))
        for w, ls in sorted(groups.items()):
            stores = sum('buffer_store' in L[j] for j in ls[0][1])
            print(f'{tag}: loads at {[i for i, _ in ls]} -> {L[w].strip()} at {w}, '
                  f'{stores} store instructions in between (all paths)')
        print(f'{tag}: {n} violations')
        bad += n
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()

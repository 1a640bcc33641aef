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
        for i in loads:
            w = next(j for j in waits if j > i)  # the explicit wait that ends this load's flight
            d = regs(L[i].split()[1].rstrip(','))
            for j in range(i + 1, w):
                line = L[j].strip()
                if line.startswith(';'):
                    continue
                if all_regs(line) & d:
                    n += 1
                    print(f'  {tag}: line {j} touches prefetch register of line {i}: {line}')
        groups = sorted(set(next(j for j in waits if j > i) for i in loads))
        for w in groups:
            first = min(i for i in loads if next(j for j in waits if j > i) == w)
            stores = sum('buffer_store' in L[j] for j in range(first, w))
            print(f'{tag}: loads at {[i for i in loads if next(j for j in waits if j > i) == w]} -> '
                  f'{L[w].strip()} at {w}, {stores} store instructions in between (all paths)')
        print(f'{tag}: {n} violations')
        bad += n
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()

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
        w0 = [i for i in waits if 'vmcnt(0)' in L[i]][-1]
        loop_waits = [i for i in waits if i > w0]
        loads = [i for i, l in enumerate(L) if re.search(r'global_load_dword', l) and w0 < i < loop_waits[0]]
        n = 0
        for i in loads:
            d = regs(L[i].split()[1].rstrip(','))
            for j in range(i + 1, loop_waits[-1]):
                line = L[j].strip()
                if line.startswith(';') or 's_waitcnt vmcnt' in line:
                    continue
                if all_regs(line) & d:
                    n += 1
                    print(f'  {tag}: line {j} touches prefetch register of line {i}: {line}')
        stores = sum('buffer_store' in L[j] for j in range(loads[-1], loop_waits[0]))
        print(f'{tag}: {len(loads)} prefetch loads, waits {[L[i].strip() for i in loop_waits]}, '
              f'{stores} store instructions in between (all paths), {n} violations')
        bad += n
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()

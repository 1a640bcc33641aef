"""ISA check for pyr_pc_kernel (sift-gpu_amd/csrc/pyramid_pc.hip).

The producer wave waits for its own LDS-DMA source rows with hand-counted
`s_waitcnt vmcnt(N)` (vmcnt counts loads, stores and LDS-DMA together, in
issue order), and the consumers must never wait on vmcnt at all (their plane
stores are fire and forget).  Those counts are only right if the compiler adds
no vector-memory traffic of its own, so this compiles pyramid_pc.hip to gfx950
assembly and checks, for both shipped instances (octave 0 and octave > 0;
the test-hook instances with a zero wait bound are skipped), that

  * no register is spilled and the kernel uses no scratch;
  * the only vmcnt waits are the producer's: octave 0 {16 (prologue: step
    -1's rows, 2 DMA instructions per image row), 2 (a step's rows behind the
    previous step's 2 plane-0 stores), 0}; octave > 0 {16 (step s's rows
    behind step s + 1's), 0};
  * there is exactly one s_barrier (the counters' initialisation): the waves
    synchronise through the LDS counters only;
  * the register transposes are there (v_permlane32_swap / v_permlane16_swap).

Exit status 1 on any violation.

    python tools/check_pc_isa.py [asm-file]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'sift-gpu_amd', 'csrc', 'pyramid_pc.hip')
WAITS = {'true': {16, 2, 0}, 'false': {16, 0}}


def compile_asm(out='/tmp/pyramid_pc_check.s'):
    subprocess.check_call(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950', '-ffp-contract=off',
                           '-fno-slp-vectorize', '-Wno-inline-asm', '-I' + os.path.join(ROOT, 'sift-gpu_amd', 'csrc'),
                           '--cuda-device-only', '-S', SRC, '-o', out], stderr=subprocess.DEVNULL)
    return out


def main():
    asm = sys.argv[1] if len(sys.argv) > 1 else compile_asm()
    s = open(asm).read()
    bad, found = [], 0
    for m in re.finditer(r'^(_ZN4sift\S*pyr_pc_kernelILb(\d)ELi(\d+)EE\S*):', s, re.M):
        name, oct0 = m.group(1), 'true' if m.group(2) == '1' else 'false'
        if m.group(3) == '0':   # the pc_stall_once test-hook instances (every wait bound 0)
            continue
        body = s[m.end():s.index('.Lfunc_end', m.end())]
        found += 1
        mi = s.index('.name:           ' + name)
        meta = s[mi:s.index('.wavefront_size', mi)]
        errs = []
        for key in ('.private_segment_fixed_size', '.vgpr_spill_count'):
            mm = re.search(re.escape(key) + r':\s+(\d+)', meta)
            if mm is None or int(mm.group(1)) != 0:
                errs.append(f'{key} = {mm.group(1) if mm else "missing"}')
        if re.search(r'\bscratch_', body):
            errs.append('scratch access in the kernel body')
        waits = {int(w) for w in re.findall(r's_waitcnt vmcnt\((\d+)\)', body)}
        if not waits <= WAITS[oct0] or not {w for w in WAITS[oct0] if w} <= waits:
            errs.append(f'vmcnt waits {sorted(waits)} (expected {sorted(WAITS[oct0])})')
        nbar = len(re.findall(r'\bs_barrier\b', body))
        if nbar != 1:
            errs.append(f'{nbar} s_barrier (expected 1: the counters\' initialisation)')
        if 'v_permlane32_swap' not in body or 'v_permlane16_swap' not in body:
            errs.append('no v_permlane32_swap / v_permlane16_swap register transposes')
        print(f'{name}: vmcnt waits {sorted(waits)}, {nbar} s_barrier, {len(errs)} violations')
        bad += [f'{name}: {e}' for e in errs]
    if found != 2:
        bad.append(f'expected 2 pyr_pc_kernel instances, found {found}')
    for e in bad:
        print('  ' + e)
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()

"""ISA check for pyr_tri_kernel (sift-gpu_amd/csrc/pyramid_tri.hip).

The kernel waits for its LDS-DMA source rows with hand-counted
`s_waitcnt vmcnt(N)`: N = the plane stores a role issues after a step's DMA
(vmcnt counts loads, stores and LDS-DMA together, in issue order).  That count
is only right if the compiler adds no vector-memory traffic of its own, so
this compiles pyramid_tri.hip to gfx950 assembly and checks, for both
instances (octave 0 and octave > 0), that

  * no register is spilled and the kernel uses no scratch (a spill or reload
    is a vector-memory op the hand counts do not know);
  * the only vmcnt waits are the roles' step waits and the final vmcnt(0):
    each store covers 4 rows, 2 per plane and step; octave 0 {4, 8, 0}
    (role 1: plane 0 + plane 3; role 2: plane 0, planes 2 and 1, the
    decimated plane), octave > 0 {2, 6, 0};
  * every step marker `; pt_step R M` of each role appears (roles 0-2, the
    role's NC = P / 8 phases: 5, 4, 3).

Exit status 1 on any violation.

    python tools/check_tri_isa.py [asm-file]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'sift-gpu_amd', 'csrc', 'pyramid_tri.hip')
WAITS = {'true': {4, 8, 0}, 'false': {2, 6, 0}}
PHASES = {0: 5, 1: 4, 2: 3}


def compile_asm(out='/tmp/pyramid_tri_check.s'):
    subprocess.check_call(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950', '-ffp-contract=off',
                           '-fno-slp-vectorize', '-Wno-inline-asm', '-I' + os.path.join(ROOT, 'sift-gpu_amd', 'csrc'),
                           '--cuda-device-only', '-S', SRC, '-o', out], stderr=subprocess.DEVNULL)
    return out


def main():
    asm = sys.argv[1] if len(sys.argv) > 1 else compile_asm()
    s = open(asm).read()
    bad, found = [], 0
    for m in re.finditer(r'^(_ZN4sift\S*pyr_tri_kernelILb(\d)EE\S*):', s, re.M):
        name, oct0 = m.group(1), 'true' if m.group(2) == '1' else 'false'
        body = s[m.end():s.index('.Lfunc_end', m.end())]
        found += 1
        # amdhsa metadata: the fields after this kernel's .name up to its .wavefront_size
        mi = s.index('.name:           ' + name)
        meta = s[mi:s.index('.wavefront_size', mi)]
        errs = []
        for key in ('.private_segment_fixed_size', '.vgpr_spill_count'):
            mm = re.search(re.escape(key) + r':\s+(\d+)', meta)
            if mm is None or int(mm.group(1)) != 0:
                errs.append(f'{key} = {mm.group(1) if mm else "missing"}')
        if re.search(r'\bscratch_|buffer_(store|load)\S*\s.*\boffset:\d+\s+; \d+-byte Folded', body):
            errs.append('scratch access in the kernel body')
        waits = {int(w) for w in re.findall(r's_waitcnt vmcnt\((\d+)\)', body)}
        waits |= {int(w) for w in re.findall(r's_waitcnt vmcnt\((\d+)\) lgkmcnt', body)}
        if not waits <= WAITS[oct0] or not {w for w in WAITS[oct0] if w} <= waits:
            errs.append(f'vmcnt waits {sorted(waits)} (expected {sorted(WAITS[oct0])})')
        marks = set(re.findall(r'; pt_step (\d) (\d)', body))
        for r, nc in PHASES.items():
            for mphase in range(nc):
                if (str(r), str(mphase)) not in marks:
                    errs.append(f'missing step marker role {r} phase {mphase}')
        print(f'{name}: vmcnt waits {sorted(waits)}, {len(marks)} step markers, {len(errs)} violations')
        bad += [f'{name}: {e}' for e in errs]
    if found != 2:
        bad.append(f'expected 2 pyr_tri_kernel instances, found {found}')
    for e in bad:
        print('  ' + e)
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()

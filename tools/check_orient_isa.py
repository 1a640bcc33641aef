"""ISA check for the orientation histogram's ordered read-modify-write steps
(detect.hip, orient_slots_kernel; reference src/sift.cpp:429-437: every bin
receives its terms in window raster order).

Each batch of 8 samples is added by 8 steps; at step jj, lane jj of every
8-lane group adds its samples (one per slot) into its slots' histogram rows.
The order is held by an `asm volatile("; orient step jj")` memory barrier on
an opaque copy of the lane index: without it hipcc rebuilt the eight guarded
blocks as a switch on the lane index and ran them out of order (3 % of the
angles a few ulps off).  This compiles detect.hip to gfx950
assembly and checks, for every orient_slots_kernel instance, that

  * the markers appear in the sample loop as complete runs 0, 1, ..., 7;
  * step jj tests the opaque lane copy against the constant jj and masks
    exec on it (v_cmp_eq_u32 jj, then s_and_saveexec);
  * inside step jj's masked block there are exactly S ds_read_b32 and S
    ds_write_b32 (S = slots, the same for every step), every write goes to an
    address read in the same block (read-modify-write of the same bins), the
    reads come first, and no other LDS access sits in the block;
  * no LDS access lies between the end of one step's block and the next
    marker (nothing of step jj can drift into step jj + 1).

Exit status 1 on any violation (also when no marker is found: the barrier
is gone).

    python tools/check_orient_isa.py [asm-file]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'sift-gpu_amd', 'csrc', 'detect.hip')


def compile_asm(out='/tmp/detect_orient_check.s'):
    subprocess.check_call(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950', '-ffp-contract=off',
                           '-fno-slp-vectorize', '-I' + os.path.join(ROOT, 'include'),
                           '-I' + os.path.join(ROOT, 'sift-gpu_amd', 'build'), '--cuda-device-only', '-S', SRC,
                           '-o', out], stderr=subprocess.DEVNULL)
    return out


def ds_addr(line):
    """(address register, offset) of a ds_read_b32 / ds_write_b32 line."""
    t = line.split()
    op = t[0]
    ops = [x.rstrip(',') for x in t[1:]]
    off = 0
    for x in ops:
        if x.startswith('offset:'):
            off = int(x.split(':')[1])
    addr = ops[1] if op.startswith('ds_read') else ops[0]
    return addr, off


def check_kernel(name, lines):
    errs = []
    code = [(i, l.strip()) for i, l in enumerate(lines)]
    marks = [(i, int(m.group(1))) for i, l in code for m in [re.search(r'; orient step (\d+)', l)] if m]
    if not marks:
        return [f'{name}: no "; orient step" markers -- the ordering barrier is gone'], 0
    seq = [k for _, k in marks]
    if len(seq) % 8 or any(seq[j] != j % 8 for j in range(len(seq))):
        errs.append(f'{name}: markers out of order: {seq}')
        return errs, len(seq) // 8
    slots = None
    for n, (mi, k) in enumerate(marks):
        # the opaque copy: the register the marker's asm holds ("+v"), which
        # the guard compares; its last write before the marker must be the
        # v_mov that copies the lane index (the scheduler may hoist it)
        nxt = marks[n + 1][0] if n + 1 < len(marks) else len(lines)
        seg = [l for i, l in code if mi < i < nxt and l and not l.startswith(';') and not l.startswith('.')]
        cmp_i = next((j for j, l in enumerate(seg) if l.startswith('v_cmp_eq_u32')), None)
        m_cmp = re.search(rf'\b{k}, (v\d+)$', seg[cmp_i]) if cmp_i is not None else None
        if m_cmp is None:
            errs.append(f'{name}: step {k}: guard is not v_cmp_eq_u32 {k}, <lane copy> '
                        f'({seg[cmp_i] if cmp_i is not None else "missing"})')
            continue
        copy_reg = m_cmp.group(1)
        prev = [l for i, l in code if i < mi and l and not l.startswith(';') and not l.startswith('.')]
        writer = next((l for l in reversed(prev) if l.split()[0].startswith('v_') and len(l.split()) > 1 and
                       l.split()[1].rstrip(',') == copy_reg), None)
        if writer is None or not writer.startswith('v_mov_b32'):
            errs.append(f'{name}: step {k}: {copy_reg} is not an opaque lane copy ({writer})')
            continue
        if any(re.search(rf'\b{copy_reg}\b', l) and l.split()[1].rstrip(',') == copy_reg
               for l in seg[:cmp_i] if len(l.split()) > 1):
            errs.append(f'{name}: step {k}: {copy_reg} rewritten between the marker and the guard')
            continue
        sv = next((j for j in range(cmp_i, len(seg)) if seg[j].startswith('s_and_saveexec')), None)
        end = next((j for j in range(sv or 0, len(seg)) if seg[j].startswith('s_or_b64 exec')), None)
        if sv is None or end is None:
            errs.append(f'{name}: step {k}: no exec-masked block')
            continue
        block = seg[sv + 1:end]
        pre = [l for l in seg[:sv] if l.startswith('ds_')]
        post = [l for l in seg[end:] if l.startswith('ds_')]
        if pre or (post and n + 1 < len(marks) and marks[n + 1][1] != 0):
            errs.append(f'{name}: step {k}: LDS access outside its block: {pre + post}')
        reads = [l for l in block if l.startswith('ds_read')]
        writes = [l for l in block if l.startswith('ds_write')]
        other = [l for l in block if l.startswith('ds_') and l not in reads + writes]
        if other or any(not l.startswith('ds_read_b32') for l in reads) or \
                any(not l.startswith('ds_write_b32') for l in writes):
            errs.append(f'{name}: step {k}: unexpected LDS instructions {other or reads + writes}')
        if slots is None:
            slots = len(reads)
        if not (len(reads) == len(writes) == slots and slots > 0):
            errs.append(f'{name}: step {k}: {len(reads)} reads / {len(writes)} writes (expected {slots} each)')
        last_read = max(j for j, l in enumerate(block) if l.startswith('ds_read')) if reads else -1
        first_write = min(j for j, l in enumerate(block) if l.startswith('ds_write')) if writes else 1 << 30
        if last_read > first_write:
            errs.append(f'{name}: step {k}: a write precedes a read of the same step')
        raddr = {ds_addr(l) for l in reads}
        for w in writes:
            if ds_addr(w) not in raddr:
                errs.append(f'{name}: step {k}: write {w} is not to a bin read in this step')
    return errs, len(seq) // 8


def main():
    asm = sys.argv[1] if len(sys.argv) > 1 else compile_asm()
    s = open(asm).read()
    bad, found = [], 0
    for m in re.finditer(r'^(_ZN4sift\S*orient_(?:slots_)?kernel\S*):', s, re.M):
        body = s[m.end():s.index('.Lfunc_end', m.end())].split('\n')
        errs, runs = check_kernel(m.group(1), body)
        found += 1
        print(f'{m.group(1)}: {runs} run(s) of 8 ordered steps, {len(errs)} violations')
        bad += errs
    if not found:
        bad.append('no orientation kernel in the assembly')
    for e in bad:
        print('  ' + e)
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()

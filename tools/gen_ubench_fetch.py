#!/usr/bin/env python3
"""Writes tools/ubench_fetch.hip: long straight-line VALU bodies (1,536
instructions, no loop inside) of 8-byte literal multiplies, 4-byte VGPR
multiplies, and the scatter blur's 1 multiply : 2 adds mix with the multiplier
as a literal or an SGPR, timed at 1-4 waves per SIMD on every CU.
    python3 tools/gen_ubench_fetch.py && hipcc -O3 --offload-arch=gfx950 -Wno-unused-value \\
        tools/ubench_fetch.hip -o tools/ubench_fetch
"""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
N = 1536


def body(kind):
    out = []
    for i in range(N):
        j, k = i % 16, (i + 1) % 16
        if kind == 'lit':
            out.append(f'"v_mul_f32 %{j}, 0x3f7fbe77, %{j}\\n"')
        elif kind == 'vgpr':
            out.append(f'"v_mul_f32 %{j}, %16, %{j}\\n"')
        elif i % 3 == 0:
            m = '0x3f7fbe77' if kind == 'mix' else '%17'
            out.append(f'"v_mul_f32 %{j}, {m}, %{k}\\n"')
        else:
            out.append(f'"v_add_f32 %{j}, %{k}, %{j}\\n"')
    return '\n        '.join(out)


def main():
    path = os.path.join(HERE, 'ubench_fetch.hip')
    src = open(path).read()
    bodies = [body(k) for k in ('lit', 'vgpr', 'mix', 'mixs')]
    # replace the four asm bodies in place (between 'asm volatile(' and ': OUTS')
    parts = re.split(r'(asm volatile\(\n)(.*?)(\n        : OUTS)', src, flags=re.S)
    n = 0
    for i in range(2, len(parts), 4):
        parts[i] = '        ' + bodies[n]
        n += 1
    open(path, 'w').write(''.join(parts))


if __name__ == '__main__':
    main()

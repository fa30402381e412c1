"""Instruction-class counts per kernel of a hipcc -S output (gfx950 asm).

    python tools/isa_stats.py file.s [name-substring]"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", s, re.S):
        name, body = m.group(1), m.group(2)
        if want not in name:
            continue
        lines = [l.strip() for l in body.split('\n')
                 if l.strip() and not l.strip().startswith(('.', ';', '_'))]

        def cnt(p):
            return sum(1 for l in lines if re.match(p, l))
        print(name[-60:], 'insts', len(lines), 'mfma', cnt(r'v_mfma'), 'ds_read', cnt(r'ds_read'),
              'writelane', cnt(r'v_writelane'), 'readlane', cnt(r'v_readlane'),
              'scratch', cnt(r'scratch_'), 'waitcnt', cnt(r's_waitcnt'),
              'valu', cnt(r'v_(?!mfma)'), 'salu', cnt(r's_(?!waitcnt|barrier|nop|cbranch|branch)'),
              'glds', cnt(r'global_load_lds'))
    for m in re.finditer(r'\.name:\s+(\S+)\n(?:.*\n){0,40}?\s+\.private_segment_fixed_size:\s+(\d+)', s):
        if want in m.group(1):
            print('scratch bytes', m.group(1)[-40:], m.group(2))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel code-object metadata of the library's HIP sources (gfx950): registers, spills,
static LDS and scratch, read from the AMDGPU metadata of a ``hipcc -save-temps`` build.

    tools/kernel_meta.py [SOURCE.hip ...] [--filter SUBSTRING] [-D MACRO=V ...]

With no source, every mpc_blaster_amd/csrc/*.hip file.  Columns: VGPR / AGPR / SGPR counts, SGPR and
VGPR spill counts, static LDS (group_segment_fixed_size) and scratch (private_segment_fixed_size)
bytes per work-item.  Host-only: the compile cross-targets gfx950, nothing runs on a GPU.
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ['-O3', '-std=c++17', '-fPIC', '--offload-arch=gfx950', '-fno-slp-vectorize']
KEYS = ('.vgpr_count', '.agpr_count', '.sgpr_count', '.sgpr_spill_count', '.vgpr_spill_count',
        '.group_segment_fixed_size', '.private_segment_fixed_size')


def demangle(names):
    out = subprocess.run(['c++filt'], input='\n'.join(names),
                         capture_output=True, text=True).stdout.split('\n')
    return out[:len(names)]


def meta(src: str, defines: list[str]) -> list[dict]:
    with tempfile.TemporaryDirectory() as d:
        cmd = ['/opt/rocm/bin/hipcc', *FLAGS, *[f'-D{x}' for x in defines], '-c', os.path.abspath(src), '-o',
               os.path.join(d, 'x.o'), '-save-temps']
        r = subprocess.run(cmd, cwd=d, capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(f'{" ".join(cmd)}\n{r.stderr}')
        s = open(glob.glob(os.path.join(d, '*gfx950*.s'))[0]).read()
    md = s[s.index('amdhsa.kernels:'):]
    kernels = []
    for block in re.split(r'\n  - ', md)[1:]:
        k = {}
        for key in KEYS + ('.name',):
            m = re.search(r'^\s*' + re.escape(key) + r':\s+(\S+)', block, re.M)
            if m:
                k[key[1:]] = m.group(1)
        if 'name' in k:
            kernels.append(k)
    for k, dn in zip(kernels, demangle([k['name'] for k in kernels])):
        k['demangled'] = dn.split('(')[0].removeprefix('void ')
    return kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('sources', nargs='*')
    ap.add_argument('--filter', default='')
    ap.add_argument('-D', dest='defines', action='append', default=[])
    args = ap.parse_args()
    srcs = args.sources or sorted(glob.glob(os.path.join(REPO, 'mpc_blaster_amd', 'csrc', '*.hip')))
    print(f'{"kernel":64s} {"vgpr":>5s} {"agpr":>5s} {"sgpr":>5s} {"sspill":>6s} {"vspill":>6s} {"lds":>6s} {"scratch":>7s}')
    for src in srcs:
        for k in meta(src, args.defines):
            if args.filter not in k['demangled']:
                continue
            print(f'{k["demangled"][:64]:64s} {k.get("vgpr_count", "?"):>5s} {k.get("agpr_count", "?"):>5s} '
                  f'{k.get("sgpr_count", "?"):>5s} {k.get("sgpr_spill_count", "?"):>6s} '
                  f'{k.get("vgpr_spill_count", "?"):>6s} {k.get("group_segment_fixed_size", "?"):>6s} '
                  f'{k.get("private_segment_fixed_size", "?"):>7s}')
    return 0


if __name__ == '__main__':
    sys.exit(main())

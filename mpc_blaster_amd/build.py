"""Build libmpcblaster.so in-tree with hipcc for gfx950 (no JIT cache, no site-packages)."""
from __future__ import annotations

import os
import shlex
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
SOURCES = ['mpcb_solve.hip', 'mpcb_split.hip', 'mpcb_rollout.hip', 'mpcb_box.hip', 'mpcb_as.hip', 'mpcb_aux.hip', 'mpcb_full.hip', 'mpcb_r17.hip',
           'mpcb_poc.hip', 'mpcb_capi.hip']
OUT = os.path.join(HERE, 'libmpcblaster.so')
ARCH = os.environ.get('MPCB_OFFLOAD_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['-O3', '-std=c++17', '-fPIC', '-shared', f'--offload-arch={ARCH}',
         # SLP packing into v_pk_fma_f32 bloats register pressure ~2x in these kernels
         '-fno-slp-vectorize',
         '-Wall', '-Wno-unused-result', '-Wno-unused-variable']


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(os.path.dirname(HERE), 'include', 'mpcb.h'))
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print('[mpcb build]', ' '.join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f'hipcc failed ({r.returncode}): {cmd[-1]}')


def build(force: bool = False, verbose: bool = True, out: str | None = None, extra=()) -> str:
    """One hipcc -c per translation unit (in parallel), then one shared-object link."""
    from concurrent.futures import ThreadPoolExecutor
    out = out or OUT
    if out == OUT and not force and not needs_build():
        return OUT
    objdir = out + '.objs'
    os.makedirs(objdir, exist_ok=True)
    flags = [f for f in FLAGS if f != '-shared'] + list(extra)
    objs = [os.path.join(objdir, os.path.splitext(s)[0] + '.o') for s in SOURCES]
    cmds = [[HIPCC] + flags + ['-c', os.path.join(CSRC, s), '-o', o] for s, o in zip(SOURCES, objs)]
    jobs = max(1, min(len(cmds), int(os.environ.get('MAX_JOBS', '8'))))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), cmds))
    _run([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}'] + objs + ['-o', out + '.tmp'], verbose)
    os.replace(out + '.tmp', out)
    return out


if __name__ == '__main__':
    build(force='--force' in sys.argv)

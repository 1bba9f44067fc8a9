#!/usr/bin/env python3
"""Build an experimental variant of the library: mpc_blaster_amd/variants/lib_<name>.so with
extra hipcc flags (e.g. -DMPCB_P1_ULDS=0).  Variants are A/B'd on the GPU box with
MPCB_LIB=<path> (tools/ab_p2.sh); they are never shipped.

    tools/build_variant.py NAME [-DFLAG=V ...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpc_blaster_amd import build as b  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(b.HERE, 'variants', f'lib_{name}.so')
os.makedirs(os.path.dirname(out), exist_ok=True)
b.build(force=True, verbose=False, out=out, extra=flags)
print(out)

"""CPU-side checks of the drop-in boundary: the HIP library builds, loads and exports every
symbol include/mpcb.h declares; the ctypes struct mirrors ``mpcb_config``; the host-side
config validation mirrors the reference constructor's arguments."""
import ctypes
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, 'include', 'mpcb.h')


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r'\b(mpcb_[a-z_]+)\s*\(', txt)))


def test_library_exports_every_declared_symbol():
    from mpc_blaster_amd import _lib
    from mpc_blaster_amd.build import build
    build()
    lib = _lib.load()
    declared = _declared()
    assert len(declared) >= 11
    for name in declared:
        assert hasattr(lib, name), name
    assert set(_lib.EXPORTS) == set(declared)
    assert lib.mpcb_abi_version() == 5


def test_config_struct_layout_matches_header():
    from mpc_blaster_amd import _lib
    # 8 int32 (32 B) + 8 doubles + J[9] + Q[289] + R[36] + QN[289] + lbu[6] + ubu[6] + lbx[17] + ubx[17]
    n_doubles = 8 + 9 + 289 + 36 + 289 + 6 + 6 + 17 + 17
    assert ctypes.sizeof(_lib.MpcbConfig) == 32 + 8 * n_doubles
    # compile a tiny C program against the header and compare sizeof/offsetof
    import subprocess
    import tempfile
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "mpcb.h"
int main(void) { printf("%zu %zu %zu %zu %zu %zu\n", sizeof(mpcb_config), offsetof(mpcb_config, dt),
  offsetof(mpcb_config, Q), offsetof(mpcb_config, lbu), offsetof(mpcb_config, box_x),
  offsetof(mpcb_config, lbx)); return 0; }
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, 'm.c')
        open(c, 'w').write(src)
        exe = os.path.join(d, 'm')
        subprocess.check_call(['gcc', '-I', os.path.dirname(HEADER), c, '-o', exe])
        out = subprocess.check_output([exe]).decode().split()
    C = _lib.MpcbConfig
    assert [int(v) for v in out] == [ctypes.sizeof(C), C.dt.offset, C.Q.offset, C.lbu.offset, C.box_x.offset,
                                     C.lbx.offset]


def test_create_without_gpu_fails_cleanly():
    """On a GPU-less host mpcb_create reports an error instead of crashing."""
    torch = pytest.importorskip('torch')
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from mpc_blaster_amd import MPCConfig, _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    c = MPCConfig().to_c()
    rc = lib.mpcb_create(ctypes.byref(c), 0, 16, ctypes.byref(h))
    assert rc != 0 and not h.value
    assert lib.mpcb_last_error()


def test_config_validation():
    from mpc_blaster_amd import MPCConfig
    with pytest.raises(ValueError):
        MPCConfig(Q=np.eye(17))
    with pytest.raises(ValueError):
        MPCConfig(lbu=np.zeros(4))
    c = MPCConfig(N=30, lbu=np.zeros(4), ubu=np.full(4, 65.0))
    cc = c.to_c()
    assert cc.box_u == 1 and cc.N == 30 and abs(cc.cost_scale - 1 / 30) < 1e-15
    assert list(cc.ubu)[:4] == [65.0] * 4


def test_config_defaults_equal_reference_json_slice():
    """MPCConfig defaults = the 12/4 slice of acados_ocp_blasterModel.json (fixture)."""
    import json
    import os
    from mpc_blaster_amd import MPCConfig
    pin = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'ocp_json_pin.json')))
    c = MPCConfig()
    W = np.asarray(pin['W'])
    assert np.array_equal(c.Q, W[:12, :12])
    assert np.array_equal(c.R, W[17:21, 17:21])
    assert np.array_equal(c.QN, np.asarray(pin['W_e'])[:12, :12])
    assert abs(c.dt - pin['solver_options']['time_steps'][0]) < 1e-15
    b = MPCConfig(lbu=np.asarray(pin['lbu'][:4]), ubu=np.asarray(pin['ubu'][:4]))
    assert b.to_c().box_u == 1


def test_packed_value_function_record_covers_every_entry():
    """The PS2 record (mpcb_kernels.h): lane j stores P[j][(j + d) % 12] for d = 0..6
    (mpcb_split.hip riccati_body, the store after the symmetric publish), and the active-set
    kernel's restart reads P[i][j] from lane i's slot (j - i) % 12 when that is <= 6, else from
    lane j's slot (i - j) % 12 (mpcb_as.hip).  Restated here on a random symmetric P: the read
    rule recovers all 144 entries from the 12 x 7 stored slots."""
    hdr = open(os.path.join(REPO, 'mpc_blaster_amd', 'csrc', 'mpcb_kernels.h')).read()
    ps2_w = int(re.search(r'PS2_W\s*=\s*(\d+)', hdr).group(1))
    nx = 12
    rng = np.random.default_rng(7)
    a = rng.standard_normal((nx, nx))
    P = a + a.T
    rec = np.full((nx, ps2_w), np.nan)
    for j in range(nx):
        for d in range(7):
            o = (j + d) % nx
            rec[j, d] = P[max(o, j), min(o, j)]   # the lower triangle the kernel reads
    assert not np.isnan(rec[:, :7]).any() and ps2_w >= 8   # slot 7 holds p_k[j]
    for jx in range(nx):        # reader lane jx rebuilds column jx: Pc[i] = P[i][jx]
        for i in range(nx):
            dd = (jx - i) % nx
            v = rec[i, dd] if dd <= 6 else rec[jx, nx - dd]
            assert v == P[i, jx]

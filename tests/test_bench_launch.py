"""bench.py's own multi-rank launcher (``--gpus N`` without torchrun): the parent starts N ranks
under torch.distributed.run before anything touches a GPU, rank 0 prints ONE JSON line with
n_gpus = N and global_batch = N*B, and the gathered u0 equals an unsharded solve.  Run here over
gloo with the CPU solver stub (tests/bench_stub.py) standing in for the HIP handle."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_cmd(workload, gpus, batch, steps, extra=()):
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get('PYTHONPATH', ''),
               OMP_NUM_THREADS='1')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT', 'BENCH_STUB_STALL_RANK'):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', str(gpus),
           '--steps', str(steps), '--warmup', '1', '--workload', workload,
           '--batch', str(batch), '--no-cpu-baseline', '--backend', 'gloo',
           '--solver-stub', 'tests.bench_stub'] + list(extra)
    return cmd, env


def _run_bench(tmp_path, workload, gpus, batch, steps=2, extra=()):
    dump = str(tmp_path / f'gather_{workload}.npy')
    cmd, env = _bench_cmd(workload, gpus, batch, steps, list(extra) + ['--dump-gather', dump])
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0]), np.load(dump)


@pytest.mark.parametrize('workload,gpus,batch', [('c2', 2, 12), ('c5', 2, 10)])
def test_bench_gpus_n_launches_n_ranks(tmp_path, workload, gpus, batch):
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec, mpc_solve
    line, got = _run_bench(tmp_path, workload, gpus, batch)
    assert line['n_gpus'] == gpus
    assert line['config']['global_batch'] == gpus * batch
    assert line['value'] > 0 and line['bad_status'] == 0
    N = 20 if workload == 'c2' else 40
    inp = make_inputs(workload, ids=np.arange(gpus * batch, dtype=np.uint64), N=N)
    ref = mpc_solve(inp['x0'], inp['xref'], inp['uref'], OcpSpec(N=N), wind=inp['wind'])['u0']
    if workload == 'c2':   # the RCCL/gloo all-gather of u0 in global id order
        assert got.shape == (gpus * batch, 4)
        assert np.array_equal(got, ref)
    else:                  # the all-reduced per-motor histogram
        b = np.clip(np.floor(ref * (64 / 65.0)), 0, 63).astype(np.int64)
        want = np.stack([np.bincount(b[:, m], minlength=64) for m in range(4)])
        assert np.array_equal(got, want)


def test_bench_gpus_1_runs_in_process(tmp_path):
    line, got = _run_bench(tmp_path, 'c2', 1, 8, steps=1)
    assert line['n_gpus'] == 1 and line['config']['global_batch'] == 8
    assert got.shape == (8, 4)


def test_bench_gpus_4_adds_the_c4_secondary(tmp_path):
    """At 4 ranks the line also times BASELINE configs[3] (c4: input box, instance-sharded over 4
    GPUs); the gathered c4 u0 equals the unsharded oracle's active-set solution."""
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec, mpc_solve
    sb = 3
    line, _ = _run_bench(tmp_path, 'c2', 4, 4, steps=1, extra=['--secondary-batch', str(sb)])
    assert line['n_gpus'] == 4 and line['config']['global_batch'] == 16
    sec = line['secondary']
    assert sec['workload'].startswith('c4') and sec['global_batch'] == 4 * sb and sec['n_gpus'] == 4
    assert sec['value'] > 0 and sec['bad_status'] == 0
    assert 'active_set' in sec['roofline']
    got = np.load(str(tmp_path / 'gather_c2.npy') + '.secondary.npy')
    inp = make_inputs('c4', ids=np.arange(4 * sb, dtype=np.uint64), N=30)
    ref = mpc_solve(inp['x0'], inp['xref'], inp['uref'],
                    OcpSpec(N=30, lbu=np.zeros(4), ubu=np.full(4, 65.0)))['u0']
    assert got.shape == (4 * sb, 4)
    assert np.array_equal(got, ref)


def test_bench_gpus_8_adds_the_c5_histogram_secondary(tmp_path):
    """At 8 ranks the line also times BASELINE configs[4] (c5: N = 40, fp32, wind, instance-sharded
    over 8 GPUs with only the u0* histogram reduced, bench.py sec_name): the all-reduced per-motor
    histogram equals the global oracle histogram of all 8 shards' instances, bit for bit."""
    from oracle.inputs import make_inputs
    from oracle.ocp import OcpSpec, mpc_solve
    sb = 3
    line, _ = _run_bench(tmp_path, 'c2', 8, 2, steps=1, extra=['--secondary-batch', str(sb)])
    assert line['n_gpus'] == 8 and line['config']['global_batch'] == 16
    sec = line['secondary']
    assert sec['workload'].startswith('c5') and sec['global_batch'] == 8 * sb and sec['n_gpus'] == 8
    assert sec['value'] > 0 and sec['bad_status'] == 0
    got = np.load(str(tmp_path / 'gather_c2.npy') + '.secondary.npy')
    inp = make_inputs('c5', ids=np.arange(8 * sb, dtype=np.uint64), N=40)
    ref = mpc_solve(inp['x0'], inp['xref'], inp['uref'], OcpSpec(N=40), wind=inp['wind'])['u0']
    b = np.clip(np.floor(ref * (64 / 65.0)), 0, 63).astype(np.int64)
    want = np.stack([np.bincount(b[:, m], minlength=64) for m in range(4)])
    assert got.shape == (4, 64) and got.sum() == 4 * 8 * sb
    assert np.array_equal(got, want)


def test_bench_stalled_rank_fails_fast():
    """A rank that never joins the rendezvous: the others give up after --init-timeout and the
    parent exits non-zero well before the driver's limit (no hang, no JSON line)."""
    import time
    cmd, env = _bench_cmd('c2', 2, 4, 1, ['--init-timeout', '8'])
    env['BENCH_STUB_STALL_RANK'] = '1'
    t0 = time.time()
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert time.time() - t0 < 200

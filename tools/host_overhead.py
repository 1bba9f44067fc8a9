#!/usr/bin/env python3
"""Host-side cost of one c2 step (the bench's timed loop is host-bound when it exceeds the device
time): issue time of K solve calls without synchronisation vs the device time per solve.

    python tools/host_overhead.py [K]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mpc_blaster_amd import BatchedMPC, MPCConfig  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
B, N = 4096, 20
mpc = BatchedMPC(MPCConfig(N=N, dtype='f64'), max_batch=B, device=0)
inp = mpc.gen_inputs(B, seed=1002, ref='hover')
outs = (torch.empty((B, 4), dtype=torch.float64, device=0), torch.empty((B, N + 1, 12), dtype=torch.float64, device=0),
        torch.empty((B, N, 4), dtype=torch.float64, device=0), torch.zeros((B,), dtype=torch.int32, device=0))
for _ in range(5):
    mpc.solve(inp['x0'], inp['xref'], inp['uref'], out=outs)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    mpc.solve(inp['x0'], inp['xref'], inp['uref'], out=outs)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(K):
    mpc.solve(inp['x0'], inp['xref'], inp['uref'], out=outs)
e1.record()
torch.cuda.synchronize()
print(f'host issue {1e6 * (t1 - t0) / K:.1f} us/step, wall {1e6 * (t2 - t0) / K:.1f} us/step, '
      f'device {1e3 * e0.elapsed_time(e1) / K:.1f} us/step')

# a K=20 window after a synchronisation (the driver's bench.py --steps 20): wall vs device time,
# and the device time of each step (events between steps, separate run)
for rep in range(3):
    torch.cuda.synchronize()
    e0.record()
    t0 = time.perf_counter()
    for _ in range(20):
        mpc.solve(inp['x0'], inp['xref'], inp['uref'], out=outs)
    e1.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'K=20 window: wall {1e6 * (t2 - t0) / 20:.1f} us/step, device {1e3 * e0.elapsed_time(e1) / 20:.1f} us/step')
evs = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
torch.cuda.synchronize()
evs[0].record()
for i in range(20):
    mpc.solve(inp['x0'], inp['xref'], inp['uref'], out=outs)
    evs[i + 1].record()
torch.cuda.synchronize()
print('per-step device us:', ' '.join(f'{1e3 * evs[i].elapsed_time(evs[i + 1]):.0f}' for i in range(20)))

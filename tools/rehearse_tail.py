"""Where a slow step of the two-rank config-4 rehearsal goes (bench.py --gpus 2
over gloo, both ranks on one GPU: the tail of VERDICT round 4 item 7).  Per
step and rank: the wall time, the native call's host phases (tpe_host_phases)
and the time inside the id-block gather (dist.gather_id_blocks).  Run as
python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
tools/rehearse_tail.py [steps]; writes gpurun_out/rehearse_tail_rank<r>.json."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import bench
    from hyperopt_amd import _native as N, dist as D, engine as E

    class _Args(object):
        dims, history5, appending, axis4 = 1000, 100000, False, 'ids'
    _, step, _ = bench.config_workload(4, rank, world, _Args())
    gather_s = []
    orig = D.gather_id_blocks

    def timed(*a, **k):
        s0 = time.perf_counter()
        try:
            return orig(*a, **k)
        finally:
            gather_s.append(time.perf_counter() - s0)
    D.gather_id_blocks = timed
    for i in range(2):
        step(i)
    eng = E._ENGINES[str(torch.device('cuda', 0))]
    buf = (ctypes.c_double * len(N.PHASES))()
    eng.lib.tpe_host_phases(1, None, 0)
    rows = []
    dist.barrier()
    for i in range(steps):
        g0 = len(gather_s)
        s0 = time.perf_counter()
        step(100 + i)
        wall = 1e3 * (time.perf_counter() - s0)
        eng.lib.tpe_host_phases(1, buf, len(N.PHASES))
        rows.append(dict(step=i, wall_ms=round(wall, 3),
                         gather_ms=round(1e3 * sum(gather_s[g0:]), 3),
                         phases_us={k: round(float(v), 1) for k, v in zip(N.PHASES, buf)}))
    eng.lib.tpe_host_phases(0, None, 0)
    os.makedirs('gpurun_out', exist_ok=True)
    with open('gpurun_out/rehearse_tail_rank%d.json' % rank, 'w') as f:
        json.dump(rows, f)
    walls = np.array([r['wall_ms'] for r in rows])
    th = ctypes.c_int32(0)
    eng.lib.tpe_host_threads(-1, ctypes.byref(th))
    print('rank %d: host threads %d' % (rank, th.value))
    slow = [r for r in rows if r['wall_ms'] > 2 * np.median(walls)]
    print('rank %d: p50 %.2f ms mean %.2f ms; slow steps:' % (rank, np.median(walls), walls.mean()))
    for r in slow:
        print('  ', json.dumps(r))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()

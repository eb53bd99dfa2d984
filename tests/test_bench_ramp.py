"""bench.py's untimed ramp on world_size 2 (gloo, CPU): ranks of different speed run the SAME number
of ramp chunks. Each sweep's ghost exchange pairs with the neighbours', so a rank that ran one chunk
more would post sends nobody answers (the multi-GPU bench would stall until the communicator's
timeout)."""
import multiprocessing as mp
import os
import socket
import sys
import time

import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, delays_ms, ramp_ms, q):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, REPO)
        import bench

        def any_rank(flag):
            t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return t.item() > 0

        def run(k):
            time.sleep(delays_ms[rank] / 1e3)

        n, ms = bench.ramp_sweeps(run, ramp_ms, any_rank, chunk=5)
        q.put((rank, n, ms, None))
    except Exception as e:  # reported to the parent
        q.put((rank, None, None, repr(e)))
    finally:
        dist.destroy_process_group()


def test_ramp_length_agreed_across_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    delays, ramp_ms = (1.0, 9.0), 60.0
    procs = [ctx.Process(target=_worker, args=(r, 2, port, delays, ramp_ms, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert all(r[3] is None for r in res), res
    counts = {r[1] for r in res}
    assert len(counts) == 1, res  # the fast rank waited for the slow one's verdict
    assert all(r[2] >= ramp_ms for r in res), res
    assert counts.pop() > 0


def test_ramp_single_rank_zero_budget():
    sys.path.insert(0, REPO)
    import bench
    calls = []
    n, _ = bench.ramp_sweeps(lambda k: calls.append(k), 0.0, lambda f: f)
    assert n == 0 and not calls

"""bench.py's agreement on a failed learner leg, on the CPU over gloo with two ranks:
a leg that fails on ONE rank is reported as failed on every rank (so all of them skip the rest
together), and a rank whose peer never reaches the agreement -- as when the peer is blocked in a
replayed collective that the failed rank will not join -- exits non-zero instead of hanging."""
import datetime
import multiprocessing as mp
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, port, mode, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    bench.CTRL = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=5))
    if mode == "one_fails":
        q.put((rank, bench.any_rank_failed(rank == 1), bench.any_rank_failed(False)))
        dist.destroy_process_group()
    else:  # "peer_stuck": rank 1 never arrives
        if rank == 1:
            time.sleep(30)
            os._exit(0)
        bench.any_rank_failed(False)
        q.put((rank, "returned", None))  # not reached: the agreement times out first


def _run(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rank, args=(r, port, mode, q)) for r in range(2)]
    for p in ps:
        p.start()
    return ps, q


def test_one_rank_failing_is_agreed_by_all():
    ps, q = _run("one_fails")
    for p in ps:
        p.join(60)
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert got == [(0, True, False), (1, True, False)]
    assert all(p.exitcode == 0 for p in ps)


def test_missing_peer_exits_nonzero():
    ps, q = _run("peer_stuck")
    ps[0].join(60)
    assert ps[0].exitcode == 3
    assert q.empty()
    ps[1].kill()
    ps[1].join(10)

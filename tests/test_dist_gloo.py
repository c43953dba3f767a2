"""Multi-process (world_size 2, gloo, CPU) checks of the data-parallel pieces: identical init by
broadcast, one flat-bucket gradient all-reduce == the mean of the per-rank gradients, replicas
in lockstep after Adam, and board sharding (board_offset) reproducing one big env."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "reinforcement-learning-2048_amd")]
    from g2048 import dqn_lib
    from g2048.dist import FlatGradBucket, broadcast_params, init_from_env
    from g2048.nets import make_net

    w, r, dev = init_from_env("gloo")
    assert (w, r, dev.type) == (world, rank, "cpu")
    torch.manual_seed(100 + rank)  # different init per rank -> broadcast must fix it
    m = make_net("conv", torch.float64)
    tg = make_net("conv", torch.float64)
    broadcast_params(m)
    broadcast_params(tg)
    bucket = FlatGradBucket(m)
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    g = torch.Generator().manual_seed(7 + rank)  # rank-local minibatch
    B = 64
    s = torch.randint(0, 10, (B, 1, 4, 4), generator=g).double()
    s2 = torch.randint(0, 10, (B, 1, 4, 4), generator=g).double()
    a = torch.randint(0, 4, (B,), generator=g)
    rew = torch.randint(0, 64, (B,), generator=g).double()
    d = (torch.rand(B, generator=g) < 0.1).double()
    bucket.zero_()
    loss, _, _ = dqn_lib.dqn_loss(m, tg, s, a, rew, s2, d, 0.8)
    loss.backward()
    local = bucket.flat.clone()
    bucket.allreduce_mean_()
    opt.step()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), local=local.numpy(), reduced=bucket.flat.numpy(),
             params=torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy(),
             init0=m._modules["0"].weight.detach().numpy())
    dist.destroy_process_group()


def test_two_rank_gradient_allreduce(tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r0, r1 = np.load(tmp_path / "r0.npz"), np.load(tmp_path / "r1.npz")
    assert not np.allclose(r0["local"], r1["local"])          # ranks saw different data
    np.testing.assert_allclose(r0["reduced"], (r0["local"] + r1["local"]) / 2, rtol=1e-12)
    assert np.array_equal(r0["reduced"], r1["reduced"])
    assert np.array_equal(r0["params"], r1["params"])          # replicas in lockstep


def test_board_sharding_oracle():
    """Rank r owns boards [r*N, (r+1)*N) through board_offset; the shards step exactly like the
    matching slices of one unsharded env (Philox subsequence = global board id)."""
    from oracle import oracle as O

    n, seed = 300, 11
    whole = O.OracleEnv(2 * n, seed=seed)
    shards = [O.OracleEnv(n, seed=seed, board_offset=r * n) for r in range(2)]
    for _ in range(50):
        whole.step(O.MODE_RANDOM)
        for sh in shards:
            sh.step(O.MODE_RANDOM)
    assert np.array_equal(whole.board, np.concatenate([sh.board for sh in shards]))
    assert np.array_equal(whole.meta, np.concatenate([sh.meta for sh in shards]))

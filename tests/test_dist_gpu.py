"""The data-parallel learner on the GPU: two ranks (gloo collectives -- RCCL refuses two ranks on
one device; the 8-GPU RCCL run is the driver's) each own a board shard and its replay ring, run
the fused graph-captured update with the flat-bucket all-reduce between the gradient and the
Adam launch, and must stay in lockstep bit for bit (online and target nets)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, net, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "reinforcement-learning-2048_amd")]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import g2048
    from g2048.learner import DQNLearner

    n = 2048
    env = g2048.VecEnv2048(n, seed=7, device=dev, board_offset=rank * n)
    rb = g2048.ReplayBuffer(8 * n, device=dev)
    env.rollout(8, replay=rb)
    L = DQNLearner(rb, net=net, dtype=torch.float32, batch_size=1024, target_sync_every=2,
                   seed=100 + rank)  # different seeds: the broadcast must equalise the init
    assert L.world == world and L.fused
    init = torch.cat([p.detach().reshape(-1).clone() for p in L.model.parameters()])
    for _ in range(3):
        L.update()
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1) for p in L.model.parameters()] +
                     [p.detach().reshape(-1) for p in L.target.parameters()]).cpu()
    got = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(got, flat)
    losses = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(losses, L.last_loss.detach().float().reshape(1).cpu())
    if rank == 0:
        same = all(torch.equal(got[0], g) for g in got[1:])
        moved = not torch.equal(init.cpu(), got[0][:init.numel()])
        finite = bool(torch.isfinite(got[0]).all())
        diff_loss = float(losses[0]) != float(losses[1])  # different shards, different minibatches
        torch.save({"same": same, "moved": moved, "finite": finite, "diff_loss": diff_loss},
                   os.path.join(out_dir, "res.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("net", ["conv", "dense64"])
def test_two_ranks_stay_in_lockstep(tmp_path, net):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    mp.spawn(_worker, args=(2, _free_port(), net, str(tmp_path)), nprocs=2, join=True)
    res = torch.load(os.path.join(tmp_path, "res.pt"), weights_only=True)
    assert res["finite"] and res["moved"]
    assert res["diff_loss"], "ranks should see different minibatches"
    assert res["same"], "replicas diverged"

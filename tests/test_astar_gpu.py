"""generate_replay_buffer_using_A_star (src/state_space_search.py:103-131) on the GPU: fresh
boards dealt by the env, host searches, transitions in the device ring (reference and fixed
formats)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("compat", [True, False])
def test_replay_ring_holds_the_paths(compat):
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    from g2048.astar import generate_replay_buffer_using_A_star

    rb, results = generate_replay_buffer_using_A_star(4, 10_000, device="cuda:0", seed=5,
                                                      goal_tile=64, compat=compat)
    n = sum(len(r["path_moves"]) for r in results)
    assert all(r["success"] for r in results) and n > 0
    assert int(rb.count) == n
    s, a, r, s2, d = (t[:n].cpu().numpy() for t in (rb.s, rb.a, rb.r, rb.s2, rb.d))
    k = 0
    for res in results:  # trace-back order: returned node first
        pb, pm, ps = res["path_boards"], res["path_moves"], res["path_scores"]
        for j in range(len(pm), 0, -1):
            if compat:  # (child, move, parent - child score, child, 0)
                assert np.array_equal(s[k], pb[j]) and np.array_equal(s2[k], pb[j])
                assert r[k] == ps[j - 1] - ps[j] and d[k] == 0
            else:       # (parent, move, gain, child, terminal(child))
                assert np.array_equal(s[k], pb[j - 1]) and np.array_equal(s2[k], pb[j])
                assert r[k] == ps[j] - ps[j - 1] == O.move(pb[j - 1], int(pm[j - 1]))[1]
                assert d[k] == int(O.legal_mask(pb[j]) == 0)
            assert a[k] == pm[j - 1]
            k += 1
    # the deque(maxlen) keeps the newest transitions
    rb2, _ = generate_replay_buffer_using_A_star(4, 7, device="cuda:0", seed=5, goal_tile=64,
                                                 compat=compat)
    assert int(rb2.count) == 7
    assert torch.equal(rb2.s[:7].cpu(), torch.from_numpy(s[n - 7:n]))

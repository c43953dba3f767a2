"""Round 4's stale bias-gradient failure, pinned down.

The torch-path learner's captured update returned wrong conv / fc bias gradients from its second
replay on, only when the fused float64 conv update ran between replays; its bias gradients were
torch's dim-0 sum (`gy.sum(0)`) then.  Two explanations were open:

  (1) torch's multi-block (global) reduction reads stale data inside a replayed graph -- a torch /
      ROCm issue (on ROCm, torch's Reduce.cuh writes the per-block partials with agent-scope
      atomic stores and lets the last block read them back with plain loads, no acquire);
  (2) a kernel of the fused update writes outside its buffers, into memory the torch graph's
      private pool owns -- a memory-safety bug on the product path.

test_captured_dim0_sum_replays captures such a reduction alone and replays it (a) back to back,
(b) with an unrelated kernel or torch graph between replays, (c) with the fused fp64 / fp32 conv
update between replays: all exact.  test_fused_learners_stay_in_bounds runs every fused learner
with every buffer it writes carved from one allocation between sentinel-filled margins: no margin
byte changes, so (2) is ruled out.  The original case on the old form fails exactly when another
GRAPH is replayed between the learner graph's replays (an unrelated torch graph suffices), and
never with HIP's graph packet capture off (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0): a runtime issue of
(1)'s kind, in HIP's pre-built graph packets.  The product path keeps torch's global reductions
out of its captured graphs, and test_torch_path_survives_interleaved_graph_replays guards that."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    import g2048
    g2048.load_native()
    return g2048


def _capture(fn):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def _between(G, kind):
    """The work run between two replays: nothing, an unrelated kernel, or a fused conv update."""
    if kind == "none":
        return lambda: None
    if kind == "torchcap":  # capture and replay an unrelated torch graph that allocates
        x = torch.randn(1 << 16, 64, dtype=torch.float64, device=DEV)
        st = {}

        def tc():
            if "g" not in st:
                def body():
                    st["y"] = (x @ x[:64].t()).relu().sum(1) * 2.0
                st["g"] = _capture(body)
            st["g"].replay()
        return tc
    if kind == "fill":
        big = torch.empty(4 << 20, dtype=torch.float64, device=DEV)  # 32 MB
        cnt = [0]

        def fill():
            cnt[0] += 1
            big.fill_(float(cnt[0]))
        return fill
    from g2048.learner import DQNLearner
    n = 2048
    env = G.VecEnv2048(n, seed=3, device=DEV)
    rb = G.ReplayBuffer(16 * n, device=DEV)
    env.rollout(16, replay=rb)
    dt = torch.float32 if kind == "conv32" else torch.float64
    L = DQNLearner(rb, net="conv", dtype=dt, batch_size=4096, target_sync_every=2, seed=9,
                   graph=kind != "conv64_eager")
    assert L.fused
    if kind == "conv64_captureonly":  # capture (+ warm-up) once, then nothing
        return lambda: L._capture() if L._graphs is None else None
    return L.update


@pytest.mark.parametrize("between", ["none", "fill", "torchcap", "conv64", "conv32"])
@pytest.mark.parametrize("rows", [16384, 36864, 73728])
def test_captured_dim0_sum_replays(G, rows, between):
    """x.sum(0) of an f64 [rows, 64] tensor produced inside the graph (the shape of the conv net's
    bias gradients at B = 4096 / 8192: conv2 [4B, 64], conv1 [9B, 64]), replayed 8 times with
    fresh inputs, each result against the float64 CPU sum (rounding-level tolerance)."""
    src = torch.zeros(rows, 64, dtype=torch.float64, device=DEV)
    out = torch.zeros(64, dtype=torch.float64, device=DEV)

    def fn():
        out.copy_((src * 1.0).sum(0))

    g = _capture(fn)
    work = _between(G, between)
    gen = torch.Generator(device=DEV).manual_seed(rows)
    errs = []
    for k in range(8):
        src.copy_(torch.randn(rows, 64, dtype=torch.float64, device=DEV, generator=gen))
        g.replay()
        torch.cuda.synchronize()
        x = src.cpu()
        ref = x.sum(0)
        scale = float(x.abs().sum(0).max())
        errs.append(float((out.cpu() - ref).abs().max()) / scale)
        work()
        torch.cuda.synchronize()
    assert max(errs) <= 1e-13, errs


class Arena:
    """One int64 allocation: [margin | piece | margin | piece | ... | margin], every piece
    256-byte aligned, everything outside the pieces' used bytes (margins and alignment tails)
    filled with a NaN-payload sentinel."""
    SENT = 0x7FF42048DEADBEEF  # a NaN payload as f64; an int64 < 2**63
    MARGIN = 8192  # int64 words = 64 KB

    def __init__(self, words):
        self.spans = []
        off = self.MARGIN
        for w in words:
            w = (int(w) + 31) // 32 * 32
            self.spans.append((off, w))
            off += w + self.MARGIN
        self.buf = torch.full((off,), self.SENT, dtype=torch.int64, device=DEV)
        self.used = [0] * len(self.spans)

    def piece(self, i, dtype, n, zero=True):
        off, w = self.spans[i]
        v = self.buf[off:off + w].view(dtype)[:n]
        assert v.numel() == n
        self.used[i] = n * v.element_size()
        if zero:
            v.zero_()
        return v

    def margins_clean(self):
        """[(region, first bad byte, last bad byte, bad bytes)] of every sentinel region that
        changed; region j is the gap after piece j - 1 (0: the leading margin)."""
        torch.cuda.synchronize()
        b = self.buf.cpu().numpy().view(np.uint8)
        pat = np.frombuffer(np.int64(self.SENT).tobytes(), dtype=np.uint8)
        bad = []
        regions = [(0, self.MARGIN * 8)] + [((o * 8) + u, (o + w + self.MARGIN) * 8)
                                            for (o, w), u in zip(self.spans, self.used)]
        for j, (lo, hi) in enumerate(regions):
            want = pat[np.arange(lo, hi) % 8]
            hit = np.nonzero(b[lo:hi] != want)[0]
            if hit.size:
                bad.append((j, int(hit[0]), int(hit[-1]), int(hit.size)))
        return bad


def _carve_net(arena, base, model, dt):
    for j, p in enumerate(model.parameters()):
        v = arena.piece(base + j, dt, p.numel(), zero=False).view_as(p)
        v.copy_(p.detach())
        p.data = v
    return base + len(list(model.parameters()))


@pytest.mark.parametrize("batch", [700, 3000, 4096, 8192, 65536])
@pytest.mark.parametrize("path", ["conv64", "conv32", "dense64_64", "dense64_32", "dense_64",
                                  "dense_32"])
def test_fused_learners_stay_in_bounds(G, path, batch):
    """Every buffer a fused update writes -- both nets' parameters (Adam, the target sync), Adam's
    moments, the workspace (packed operands, slabs, dZ2 / dM, pre), grad_out, y, idx, the loss and
    the step counter -- carved from one allocation between 64 KB sentinel margins: three updates
    with Adam folded in, then three gradient-only updates + the separate Adam step (the
    data-parallel form), and no margin byte changes."""
    from g2048 import qnet
    from g2048.nets import make_net
    from g2048.optim import FusedAdam

    net = path.rsplit("_", 1)[0] if path.startswith("dense") else "conv"
    f64 = path.endswith("64")
    dt = torch.float64 if f64 else torch.float32
    n = 2048
    env = G.VecEnv2048(n, seed=5, device=DEV)
    rb = G.ReplayBuffer(16 * n, device=DEV)
    env.rollout(16, replay=rb)
    torch.manual_seed(1)
    model = make_net(net, dt, DEV)
    target = copy.deepcopy(model)
    P = sum(p.numel() for p in model.parameters())
    from g2048 import _native as N
    wsn = {"conv64": N.load().g2048_convnet_update_f64_workspace,
           "conv32": N.load().g2048_convnet_train_workspace,
           "dense64_64": N.load().g2048_dense64_update_f64_workspace,
           "dense64_32": N.load().g2048_dense64_update_workspace,
           "dense_64": lambda b: N.load().g2048_densenet_update_workspace(b, N.F64),
           "dense_32": lambda b: N.load().g2048_densenet_update_workspace(b, N.F32)}[path](batch)
    assert wsn > 0
    words = lambda k: (k * (8 if f64 else 4) + 7) // 8  # noqa: E731  (int64 words of k elements)
    nparam = len(list(model.parameters()))
    sizes = ([words(p.numel()) for p in model.parameters()] * 2
             + [words(P), words(P), words(wsn), words(P), words(batch), batch, 1, 1])
    A = Arena(sizes)
    k = _carve_net(A, 0, model, dt)
    k = _carve_net(A, k, target, dt)
    adam = (qnet.Adam64 if f64 else FusedAdam)(model.parameters(), lr=1e-2)
    adam.exp_avg = A.piece(k, dt, P)
    adam.exp_avg_sq = A.piece(k + 1, dt, P)
    adam.attach_target(list(target.parameters()), 2)
    ws = A.piece(k + 2, dt, wsn)
    grad = A.piece(k + 3, dt, P)
    y = A.piece(k + 4, dt, batch)
    idx = A.piece(k + 5, torch.int64, batch)
    step = A.piece(k + 6, torch.int64, 1)
    loss = A.piece(k + 7, dt, 1).view(())
    cls = {"conv64": qnet.ConvUpdate64, "conv32": qnet.ConvUpdate,
           "dense64_64": qnet.Dense64Update64, "dense64_32": qnet.Dense64Update,
           "dense_64": qnet.DenseRefUpdate, "dense_32": qnet.DenseRefUpdate}[path]
    upd = cls(model, target, batch, adam=adam)
    upd.workspace = ws
    if hasattr(upd, "ensure_packed"):
        upd.ensure_packed(force=True)
    assert nparam in (4, 8)
    for _ in range(3):
        upd(rb, idx, y, step, 0.8, True, 77, None, grad_out=grad, loss_out=loss)
    bad = A.margins_clean()
    assert not bad, ("Adam folded", bad)
    assert torch.isfinite(loss).all() and int(step) == 3
    upd.adam = None
    for _ in range(3):
        upd(rb, idx, y, step, 0.8, True, 77, None, grad_out=grad, loss_out=loss)
        adam.step(grad, step)
    bad = A.margins_clean()
    assert not bad, ("gradient only + Adam step", bad)
    assert torch.isfinite(grad).all() and all(torch.isfinite(p).all() for p in model.parameters())


def _interleaved_errors(G, between, form):
    """Four updates of a torch-path learner's captured float64 conv update at B = 4096 against the
    same learner run eagerly (same rows and weights), with `between` run after each update; the
    bias gradients in `form` ("sum": torch's dim-0 sum, round 3; "gemm": the product path).
    Returns the per-update, per-tensor relative gradient errors."""
    from g2048 import nets
    from g2048.learner import DQNLearner

    n, B = 2048, 4096
    env = G.VecEnv2048(n, seed=3, device=DEV)
    rb = G.ReplayBuffer(16 * n, device=DEV)
    env.rollout(16, replay=rb)
    rows = torch.zeros(B, dtype=torch.int64, device=DEV)
    work = _between(G, between)
    old = nets.BIAS_GRAD_FORM
    nets.BIAS_GRAD_FORM = form
    try:
        kw = dict(net="conv", dtype=torch.float64, batch_size=B, target_sync_every=2, seed=7,
                  loss_fn=torch.nn.L1Loss(reduction="sum"), sampler=lambda b, r: rows)
        a = DQNLearner(rb, graph=True, **kw)
        b = DQNLearner(rb, graph=False, **kw)
        a.loss_fn = b.loss_fn = None
        b.model.load_state_dict(a.model.state_dict())
        b.target.load_state_dict(a.target.state_dict())
        gen = torch.Generator(device=DEV).manual_seed(3)
        sizes = [p.numel() for p in a.model.parameters()]
        errs = []
        for k in range(4):
            rows.copy_(torch.randint(0, 16 * n, (B,), device=DEV, generator=gen))
            a.update()
            b.update()
            torch.cuda.synchronize()
            off, e = 0, []
            for sz in sizes:
                ga, gb = a.grad_flat[off:off + sz], b.grad_flat[off:off + sz]
                e.append(float((ga - gb).norm()) / max(float(gb.norm()), 1e-300))
                off += sz
            errs.append(e)
            with torch.no_grad():
                for p, q in zip(list(a.model.parameters()) + list(a.target.parameters()),
                                list(b.model.parameters()) + list(b.target.parameters())):
                    p.copy_(q)
            work()
            torch.cuda.synchronize()
    finally:
        nets.BIAS_GRAD_FORM = old
    return errs


# interleavings: nothing, an eager torch kernel, another captured torch graph replayed, the fused
# conv learner's captured update (fp64 / fp32), the same run eagerly, its capture without replays
BETWEEN = ["none", "fill", "torchcap", "conv64", "conv64_eager", "conv64_captureonly", "conv32"]


@pytest.mark.parametrize("between", BETWEEN)
def test_torch_path_survives_interleaved_graph_replays(G, between):
    """The product path (bias gradients through the chunked GEMMs, nets.Linear) is exact in every
    interleaving -- in particular with other graphs replayed between the captured update's
    replays, where a torch global reduction inside the graph goes wrong (below).  A global
    reduction that re-enters the captured learner graph makes this test fail."""
    errs = _interleaved_errors(G, between, "gemm")
    assert max(max(e) for e in errs) <= 1e-9, errs


@pytest.mark.parametrize("between", ["torchcap", "conv64"])
def test_old_bias_form_packet_capture_repro(G, between):
    """Round 4's failure, reproduced on the old form: torch's dim-0 sum over the 36 864 rows of
    conv1's bias gradient, captured in the update graph, comes out wrong on every replay after
    ANOTHER graph was replayed in between (a torch graph of unrelated ops does it as well as the
    fused learner's: `torchcap`), never with eager work in between or without replays, and not
    with HIP's graph packet capture off (test_old_bias_form_without_packet_capture).  Expected to
    fail while the runtime has the bug: xfail then, a pass once it is fixed."""
    errs = _interleaved_errors(G, between, "sum")
    bad = max(max(e) for e in errs)
    if bad > 1e-9:
        assert max(errs[0]) <= 1e-9  # the first replay (before any interleaved graph) is right
        pytest.xfail(f"HIP graph packet capture: conv1 bias gradient off by {bad:.3g} (relative)")


def test_old_bias_form_without_packet_capture(tmp_path):
    """The same interleaving with DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 (HIP's graph launch without
    its pre-built AQL packets) is exact: the wrong sums come from the runtime's packet-capture
    path, not from the kernels of either learner (whose buffers stay in bounds, above)."""
    import json
    import os
    import subprocess
    import sys

    env = dict(os.environ, DEBUG_CLR_GRAPH_PACKET_CAPTURE="0")
    out = subprocess.run([sys.executable, __file__, "torchcap"], capture_output=True, text=True,
                         env=env, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    errs = json.loads(out.stdout.strip().splitlines()[-1])
    assert max(max(e) for e in errs) <= 1e-9, errs


def test_unpacked_workspace_refused(G):
    """ABI v4: an Adam-folded float64 conv update on a workspace g2048_convnet_pack_f64 never
    packed for these nets is refused (G2048_EINVAL) instead of training on uninitialised memory;
    packing it makes the same call succeed."""
    from g2048 import _native as N
    from g2048 import qnet
    from g2048.nets import make_net

    n = 1024
    env = G.VecEnv2048(n, seed=2, device=DEV)
    rb = G.ReplayBuffer(4 * n, device=DEV)
    env.rollout(4, replay=rb)
    m = make_net("conv", torch.float64, DEV)
    t = copy.deepcopy(m)
    upd = qnet.ConvUpdate64(m, t, 512, adam=qnet.Adam64(m.parameters()))
    upd.workspace = torch.empty_like(upd.workspace)  # a fresh workspace, never packed
    upd._packed_at = upd._versions()  # (so the host-side version check does not pack it)
    args = (rb, torch.zeros(512, dtype=torch.int64, device=DEV),
            torch.zeros(512, dtype=torch.float64, device=DEV),
            torch.zeros(1, dtype=torch.int64, device=DEV))
    with pytest.raises(N.NativeError, match="packed"):
        upd(*args)
    # the same workspace for other nets than the ones it was packed for: refused as well
    upd.ensure_packed(force=True)
    upd(*args)
    other = qnet.ConvUpdate64(make_net("conv", torch.float64, DEV), t, 512,
                              adam=qnet.Adam64(m.parameters()))
    other.workspace = upd.workspace
    other._packed_at = other._versions()
    with pytest.raises(N.NativeError, match="packed"):
        other(*args)
    torch.cuda.synchronize()


if __name__ == "__main__":  # test_old_bias_form_without_packet_capture's child: one interleaving
    import json
    import os
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "reinforcement-learning-2048_amd")]
    import g2048

    g2048.load_native()
    print(json.dumps(_interleaved_errors(g2048, sys.argv[1], "sum")))

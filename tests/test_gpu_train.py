"""Training step (training.rs:137-190, 277-292) on the GPU against the
torch-CPU float64 oracle (oracle/train_ref.py).  The step computes in f32 (the reference's
precision) on v_mfma_f32_16x16x4_f32.  Tolerances:
  losses                 |d| <= 1e-5 * (1 + |ref|)
  gradient tensors       relative norm error ||g - g_ref|| / ||g_ref|| <= 1e-4 per parameter
                         tensor, with the oracle's ReLUs taking the GPU's branch (its masks, read
                         back through az_trainer_relu_output): a pre-activation within f32 rounding
                         of 0 can otherwise take the other branch in float64, and that one element
                         moves dbeta of the BatchNorm below it by ~1/(64*B) relative, propagating
                         to every earlier layer (measured 8e-4 at B=2, 20x256, without masks).
                         Without masks: <= 1e-2.  Biases of convs followed by BatchNorm have exact
                         gradient 0: max |g| <= 1e-5 (rounding noise of a sum that cancels).
  running statistics     |d| <= 1e-5 * (1 + |ref|)
  AdamW + clipping       bit-exact against the float32 restatement, given the GPU gradients
"""
import numpy as np
import pytest

import azchess as A
import train_ref as T

pytestmark = pytest.mark.gpu


def batch(n, seed):
    """Positions from random playouts (to_tensor planes), sparse target policies over legal
    moves (visit distributions), target values in [-1, 1]."""
    rng = np.random.default_rng(seed)
    planes, pol, val = [], [], []
    while len(planes) < n:
        gs = A.GameState()
        for _ in range(int(rng.integers(0, 60))):
            idx = gs.position.legal_indices()
            if len(idx) == 0 or int(A.play_move(gs, int(rng.choice(idx)))) != 0:
                break
        idx = np.unique(gs.position.legal_indices())
        if len(idx) == 0:
            continue
        visits = rng.integers(0, 20, len(idx)).astype(np.float32)
        visits[0] += 1
        p = np.zeros(4096, np.float32)
        p[idx] = visits / np.float32(visits.sum())
        planes.append(A.to_tensor(gs.position).reshape(19 * 64))
        pol.append(p)
        val.append(np.float32(rng.uniform(-1, 1)))
    return np.stack(planes), np.stack(pol), np.array(val, np.float32)


def bn_fed_biases(blocks):
    names = ["input_conv.bias", "policy_conv_1.bias", "value_conv.bias"]
    for b in range(blocks):
        names += ["res_blocks.%d.conv1.bias" % b, "res_blocks.%d.conv2.bias" % b]
    return set(names)


@pytest.mark.parametrize("blocks,filters,n", [(2, 32, 16), (6, 64, 8), (20, 256, 2)])
def test_grads_losses_and_running_stats_match_oracle(require_gpu, blocks, filters, n):
    w = A.random_weights(blocks, filters, seed=7)
    planes, tpol, tval = batch(n, seed=blocks * 100 + n)
    tr = A.Trainer(blocks, filters, weights=w, max_batch=max(n, 4))
    pl, vl = tr.compute_gradients(planes, tpol, tval)
    g = tr.grads()
    masks = tr.relu_masks(n)
    ref = T.TrainRef(blocks, filters, w)
    rg, (rpl, rvl) = ref.grads(planes, tpol, tval, masks)
    ug, _ = T.TrainRef(blocks, filters, w).grads(planes, tpol, tval)     # the oracle's own branches
    assert abs(pl - rpl) <= 1e-5 * (1 + abs(rpl)), (pl, rpl)
    assert abs(vl - rvl) <= 1e-5 * (1 + abs(rvl)), (vl, rvl)
    zero_bias = bn_fed_biases(blocks)
    seg, _ = T.segments(blocks, filters)
    for name, (o, shape, bn) in seg.items():
        size = int(np.prod(shape))
        if bn:
            C = shape[1]
            parts = [(name + ".gamma", o, C), (name + ".beta", o + C, C)]
        else:
            parts = [(name, o, size)]
        for pname, off, cnt in parts:
            a, r, u = g[off:off + cnt].astype(np.float64), rg[off:off + cnt], ug[off:off + cnt]
            if pname in zero_bias:
                assert np.abs(a).max() <= 1e-5, (pname, np.abs(a).max())
                continue
            nr = max(np.linalg.norm(r), 1e-30)
            assert np.linalg.norm(a - r) / nr <= 1e-4, (pname, np.linalg.norm(a - r) / nr)
            assert np.linalg.norm(a - u) / nr <= 1e-2, (pname, np.linalg.norm(a - u) / nr)
    p = tr.params()
    rs = ref.running_stats_flat(w)
    mask = T.trainable_mask(blocks, filters)
    stats = ~mask
    assert np.all(np.abs(p[stats] - rs[stats]) <= 1e-5 * (1 + np.abs(rs[stats])))
    assert np.array_equal(p[mask], w[mask])    # compute_gradients does not move parameters


def test_adamw_and_clipping_bit_exact(require_gpu):
    blocks, filters = 2, 32
    w = A.random_weights(blocks, filters, seed=3)
    tr = A.Trainer(blocks, filters, weights=w, max_batch=16)
    mask = T.trainable_mask(blocks, filters)
    m = np.zeros_like(w)
    v = np.zeros_like(w)
    p = tr.params()
    for step, it in enumerate([5, 13, 1002]):
        planes, tpol, tval = batch(16, seed=step)
        tr.compute_gradients(planes, tpol, tval)
        g = tr.grads()
        p = tr.params()                     # running statistics moved during the forward
        lr = A.get_cyclical_lr(it)
        assert lr == T.cyclical_lr(it)
        tr.apply(lr)
        p, m, v = T.adamw_step(p, g, m, v, mask, step + 1, lr)
        got = tr.params()
        assert np.array_equal(got, p), np.abs(got - p).max()
    # clipping engaged: some gradient entries exceed 1 in magnitude on this batch
    assert np.abs(g).max() > 0


def test_step_is_deterministic_and_comm_world1_is_identity(require_gpu):
    blocks, filters = 2, 64
    w = A.random_weights(blocks, filters, seed=11)
    planes, tpol, tval = batch(8, seed=5)
    a = A.Trainer(blocks, filters, weights=w, max_batch=8)
    b = A.Trainer(blocks, filters, weights=w, max_batch=8)
    b.set_comm(A.comm_unique_id(), 0, 1)     # RCCL all-reduce over a 1-rank communicator
    for it in range(3):
        la = a.step(planes, tpol, tval, A.get_cyclical_lr(it))
        lb = b.step(planes, tpol, tval, A.get_cyclical_lr(it))
        assert la == lb
    assert np.array_equal(a.params(), b.params())
    assert np.array_equal(a.grads(), b.grads())


def test_training_reduces_the_loss(require_gpu):
    blocks, filters = 2, 32
    tr = A.Trainer(blocks, filters, max_batch=32)
    planes, tpol, tval = batch(32, seed=9)
    first = sum(tr.step(planes, tpol, tval, 1e-3))
    for _ in range(20):
        last = sum(tr.step(planes, tpol, tval, 1e-3))
    assert last < 0.8 * first, (first, last)
    # the trained weights drive the inference engine (model.valid(), training.rs:83)
    net = tr.model(dtype="f32")
    pol, val = net.forward(planes[:4])
    assert np.allclose(pol.sum(1), 1.0, atol=1e-4) and np.all(np.abs(val) <= 1)


def test_full_loop_selfplay_replay_train(require_gpu):
    """training.rs train(): self-play -> memory.rs replay -> training steps -> new model, twice."""
    logs = []
    tr, replay, hist = A.train(2, blocks=2, filters=32, games=16, sims=8, min_replay=200, train_steps=3,
                               batch_size=64, dtype="f32", log=logs.append)
    assert len(hist) == 2 and len(replay) >= 200
    assert all(np.isfinite(h["policy_loss"]) and np.isfinite(h["value_loss"]) for h in hist)
    assert hist[1]["lr"] == A.get_cyclical_lr(1)
    step_ms, ar_ms, n = tr.timing()
    assert n == 6 and step_ms > 0 and ar_ms < 1.0


def test_c5_full_loop_20x256(require_gpu):
    """C5 (BASELINE.json configs[4]) at its network size on one GPU: one iteration of train()
    (training.rs:71-200) with the 20x256 f32 net -- 256 self-play games played to the end on the
    Winograd tower, memory.rs replay, 2 AdamW steps on 512-position batches -- at 8 sims/move so
    that it fits a test.  Checks: every game ends and every searched move becomes an EpisodeStep;
    the replay holds >= 512 positions; losses finite; one more AdamW step at 20x256 bit-exact
    against the float32 restatement (T.adamw_step, fresh moments); the trained net's forward within
    the f32 tolerance of the oracle on 4 replay positions."""
    import oracle as O
    B, F, G = 20, 256, 256
    tr, replay, hist = A.train(1, blocks=B, filters=F, games=G, sims=8, min_replay=512, train_steps=2,
                               batch_size=512, dtype="f32")
    h = hist[0]
    assert h["games_finished"] == h["selfplay_games"] == G
    assert h["episode_steps"] == h["moves"] > G
    assert len(replay) >= 512
    assert np.isfinite(h["policy_loss"]) and np.isfinite(h["value_loss"])
    # one AdamW step at 20x256 from the trained weights, bit-exact
    planes, pol, val, _ = replay.sample_arrays(512, seed=99)
    t2 = A.Trainer(B, F, weights=tr.params(), max_batch=512)
    t2.compute_gradients(planes, pol, val)
    g = t2.grads()
    p = t2.params()
    lr = A.get_cyclical_lr(1)
    t2.apply(lr)
    mask = T.trainable_mask(B, F)
    want, _, _ = T.adamw_step(p, g, np.zeros_like(p), np.zeros_like(p), mask, 1, lr)
    got = t2.params()
    assert np.array_equal(got, want), np.abs(got - want).max()
    # the trained network on the inference engine (model.valid(), training.rs:83) vs the oracle
    net = tr.model(dtype="f32")
    assert net.winograd                  # the headline's f32 Winograd tower
    x = planes[:4].reshape(4, 19, 8, 8)
    gp, gv = net.forward(x)
    rp, rv = O.RefNet(B, F, tr.params()).forward(x)
    assert np.all(np.abs(gv - rv) <= 1e-5), np.abs(gv - rv).max()
    assert np.all(np.abs(gp - rp) <= 1e-4 * rp + 1e-8)


def test_winograd_training_convs_match_direct(require_gpu, monkeypatch):
    """The 20x256 training step's residual convs (forward and data grad) as Winograd F(2x2,3x3)
    (conv_wino_train_kernel, the inference tower's core) and as implicit-GEMM direct convs
    (AZ_TRAIN_WINOGRAD=0) on the same batch, each against the float64 oracle following that path's
    own ReLU masks: losses within 1e-5, every gradient tensor within 1e-4 relative norm.  The two
    paths round differently, so a pre-activation within f32 rounding of 0 can take different ReLU
    branches in them: path against path is held to the unmasked tolerance, 1e-2 (module docstring)."""
    blocks, filters, n = 20, 256, 4
    w = A.random_weights(blocks, filters, seed=5)
    planes, tpol, tval = batch(n, seed=77)
    seg, _ = T.segments(blocks, filters)
    zero_bias = bn_fed_biases(blocks)
    stats = ~T.trainable_mask(blocks, filters)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("AZ_TRAIN_WINOGRAD", flag)
        tr = A.Trainer(blocks, filters, weights=w, max_batch=n)
        (pl, vl), g, p = tr.compute_gradients(planes, tpol, tval), tr.grads(), tr.params()
        ref = T.TrainRef(blocks, filters, w)
        rg, (rpl, rvl) = ref.grads(planes, tpol, tval, tr.relu_masks(n))
        assert abs(pl - rpl) <= 1e-5 * (1 + abs(rpl)) and abs(vl - rvl) <= 1e-5 * (1 + abs(rvl)), (flag, pl, rpl, vl, rvl)
        for name, (o, shape, bn) in seg.items():
            size = int(np.prod(shape))
            parts = [(name + ".gamma", o, shape[1]), (name + ".beta", o + shape[1], shape[1])] if bn else [(name, o, size)]
            for pname, off, cnt in parts:
                if pname in zero_bias:
                    continue
                a, r = g[off:off + cnt].astype(np.float64), rg[off:off + cnt]
                err = np.linalg.norm(a - r) / max(np.linalg.norm(r), 1e-30)
                assert err <= 1e-4, (flag, pname, err)
        rs = ref.running_stats_flat(w)
        assert np.all(np.abs(p[stats] - rs[stats]) <= 1e-5 * (1 + np.abs(rs[stats]))), flag
        out[flag] = g
    g1, g0 = out["1"].astype(np.float64), out["0"].astype(np.float64)
    for name, (o, shape, bn) in seg.items():
        if name in zero_bias:
            continue
        cnt = 2 * shape[1] if bn else int(np.prod(shape))
        r = g0[o:o + cnt]
        assert np.linalg.norm(g1[o:o + cnt] - r) <= 1e-2 * max(np.linalg.norm(r), 1e-30), name


@pytest.mark.parametrize("knob,fuse,n", [("AZ_TRAIN_ORC", "1", 300), ("AZ_TRAIN_ORC", "0", 37)])
def test_round6_conv_changes_are_bit_identical(require_gpu, monkeypatch, knob, fuse, n):
    """Round 6, AZ_TRAIN_ORC: for a BatchNorm with no residual
    (BN 0, every block's BN1) the data-grad conv recomputes O > 0 as ((Y - mean) / std) * gamma +
    beta > 0 (the forward's own float expression) instead of reading O, in the BN-backward staging
    and in the STATS 2 epilogue (fused and unfused BN paths; n = 300: the persistent one-board
    kernel, 44 workgroups take two boards; n = 37: the half-channel kernel, which reads O either
    way).  Losses, running statistics and every gradient bit-identical over two steps (the second
    from the AdamW-updated weights)."""
    blocks = 3
    w = A.random_weights(blocks, 256, seed=29)
    planes, tpol, tval = batch(n, seed=501)
    monkeypatch.setenv("AZ_TRAIN_FUSE_BN", fuse)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv(knob, flag)
        tr = A.Trainer(blocks, 256, weights=w, max_batch=n)
        rec = []
        for it in range(2):
            rec.append((tr.compute_gradients(planes, tpol, tval), tr.grads(), tr.params()))
            tr.apply(A.get_cyclical_lr(it))
        out[flag] = rec
    for (l1, g1, p1), (l0, g0, p0) in zip(out["1"], out["0"]):
        assert l1 == l0
        assert np.array_equal(p1, p0)
        assert np.array_equal(g1, g0), np.abs(g1 - g0).max()


@pytest.mark.parametrize("blocks,n", [(2, 300), (3, 13)])
def test_bn_staging_matches_separate_bn_kernels(require_gpu, monkeypatch, blocks, n):
    """The BatchNorm apply / backward staged in the Winograd convs (the default) against the same
    step with separate BN kernels (AZ_TRAIN_FUSE_BN=0: bn_apply4 / bn_back4 and the convs' plain
    staging): the staging does their arithmetic element for element and both take the statistics
    from the convs' per-board partials, so losses, running statistics and every gradient but the
    BN-fed conv biases are bit-identical (those biases' exact gradient is 0: their partial sums
    are added in another order, |g| <= 1e-5 either way).  n = 300 boards: the persistent convs'
    256 workgroups take two boards each for 44 of them; n = 13: fewer boards than workgroups."""
    w = A.random_weights(blocks, 256, seed=23)
    planes, tpol, tval = batch(n, seed=400 + n)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("AZ_TRAIN_FUSE_BN", flag)
        tr = A.Trainer(blocks, 256, weights=w, max_batch=n)
        losses = tr.compute_gradients(planes, tpol, tval)
        out[flag] = (losses, tr.grads(), tr.params())
    (l1, g1, p1), (l0, g0, p0) = out["1"], out["0"]
    assert l1 == l0
    assert np.array_equal(p1, p0)                 # running statistics
    seg, _ = T.segments(blocks, 256)
    zero_bias = bn_fed_biases(blocks)
    checked = 0
    for name, (o, shape, bn) in seg.items():
        cnt = 2 * shape[1] if bn else int(np.prod(shape))
        a, b = g1[o:o + cnt], g0[o:o + cnt]
        if name in zero_bias:
            assert np.abs(a).max() <= 1e-5 and np.abs(b).max() <= 1e-5, name
            continue
        assert np.array_equal(a, b), (name, np.abs(a - b).max())
        checked += 1
    assert checked > 4 * blocks


@pytest.mark.parametrize("blocks,n,fuse,parts", [(20, 4, "1", "4"), (2, 80, "1", "2"), (2, 80, "0", "4"),
                                                 (3, 13, "0", "2"), (2, 64, "1", "4"), (2, 128, "1", "2")])
def test_part_workgroup_convs_bit_identical(require_gpu, monkeypatch, blocks, n, fuse, parts):
    """Round 6: at small batches (the 512 / world shard of a sharded step) the Winograd convs run as
    two half-channel or four quarter-channel workgroups per board (conv_wino_part_kernel: the
    default when 2B or 4B <= 256, so that 2x / 4x the CUs work); against the persistent one-board
    kernel (AZ_TRAIN_HALF=0): the same MFMA accumulation order per accumulator (the quarters
    interleave two steps' chains), transforms, BatchNorm staging and per-board statistics, so two
    steps give bit-identical losses, gradients and parameters.  n = 64 / 80 / 128 map a board's
    parts to one XCD (n % 8 == 0), n = 4 / 13 take the plain board order; fuse = "0" runs the convs
    without BatchNorm staging (AZ_TRAIN_FUSE_BN=0)."""
    w = A.random_weights(blocks, 256, seed=17)
    planes, tpol, tval = batch(n, seed=300 + n)
    monkeypatch.setenv("AZ_TRAIN_FUSE_BN", fuse)
    out = {}
    for flag in (parts, "0"):
        monkeypatch.setenv("AZ_TRAIN_HALF", flag)
        tr = A.Trainer(blocks, 256, weights=w, max_batch=n)
        losses = [tr.step(planes, tpol, tval, A.get_cyclical_lr(it)) for it in range(2)]
        out[flag] = (losses, tr.grads(), tr.params())
    (l1, g1, p1), (l0, g0, p0) = out[parts], out["0"]
    assert l1 == l0
    assert np.array_equal(g1, g0), np.abs(g1 - g0).max()
    assert np.array_equal(p1, p0), np.abs(p1 - p0).max()


@pytest.mark.parametrize("blocks,n", [(2, 81), (2, 512), (3, 64), (2, 4)])
def test_weight_grad_one_wave_per_simd_bit_identical(require_gpu, monkeypatch, blocks, n):
    """Round 6: the default Winograd weight grad (wino_wgrad_gemm4_kernel: one wave per SIMD,
    accumulators in AGPRs, the next board transformed and the one after loaded between single
    MFMAs) against the 8-wave kernel (AZ_TRAIN_WGRAD4=0): the same MFMA sequence per accumulator
    and the same transform operations, so two steps give bit-identical losses, gradients and
    parameters.  n = 81: 14 splits of 6 boards, the last of 3; 64: 16 splits of 4 boards (a world-8
    shard); 4: splits of one board.  (The output-channel split of small batches is off here: its
    own test pins it against this kernel.)"""
    w = A.random_weights(blocks, 256, seed=19)
    planes, tpol, tval = batch(n, seed=400 + n)
    monkeypatch.setenv("AZ_TRAIN_WGRAD_COSPLIT", "0")
    monkeypatch.setenv("AZ_TRAIN_WGRAD_COSPLIT4", "0")
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("AZ_TRAIN_WGRAD4", flag)
        tr = A.Trainer(blocks, 256, weights=w, max_batch=n)
        losses = [tr.step(planes, tpol, tval, A.get_cyclical_lr(it)) for it in range(2)]
        out[flag] = (losses, tr.grads(), tr.params())
    (l1, g1, p1), (l0, g0, p0) = out["1"], out["0"]
    assert l1 == l0
    assert np.array_equal(g1, g0), np.abs(g1 - g0).max()
    assert np.array_equal(p1, p0), np.abs(p1 - p0).max()


@pytest.mark.parametrize("parts", ["AZ_TRAIN_WGRAD_COSPLIT", "AZ_TRAIN_WGRAD_COSPLIT4"])
@pytest.mark.parametrize("blocks,n,rows", [(2, 64, 128), (3, 81, 176), (2, 4, 16)])
def test_weight_grad_output_channel_split_bit_identical(require_gpu, monkeypatch, blocks, n, rows, parts):
    """Round 6: the one-wave weight grad with its output channels split over two or four
    workgroups (wino_wgrad_gemm4_kernel<2> / <4>, AZ_TRAIN_WGRAD_COSPLIT / _COSPLIT4: half / a quarter
    of the split partials at small batches) against one workgroup per (split, point), at the same
    split size (AZ_TRAIN_WGRAD_ROWS): each
    output channel's accumulator takes the same MFMAs in the same order, so two steps give
    bit-identical losses, gradients and parameters."""
    w = A.random_weights(blocks, 256, seed=29)
    planes, tpol, tval = batch(n, seed=600 + n)
    monkeypatch.setenv("AZ_TRAIN_WGRAD_ROWS", str(rows))
    monkeypatch.setenv("AZ_TRAIN_WGRAD_COSPLIT", "0")
    monkeypatch.setenv("AZ_TRAIN_WGRAD_COSPLIT4", "0")
    out = {}
    for flag in (str(n), "0"):
        monkeypatch.setenv(parts, flag)
        tr = A.Trainer(blocks, 256, weights=w, max_batch=n)
        losses = [tr.step(planes, tpol, tval, A.get_cyclical_lr(it)) for it in range(2)]
        out[flag] = (losses, tr.grads(), tr.params())
    (l1, g1, p1), (l0, g0, p0) = out[str(n)], out["0"]
    assert l1 == l0
    assert np.array_equal(g1, g0), np.abs(g1 - g0).max()
    assert np.array_equal(p1, p0), np.abs(p1 - p0).max()


def test_winograd_weight_grad_multi_split(require_gpu):
    """the production Winograd weight grad (wino_wgrad_gemm_kernel, at most 16 splits of
    whole boards, summed by wino_wgrad_reduce_out_kernel) with a partial last split: 81 boards =
    14 splits of 6 boards, the last one of 3.  Every gradient tensor against
    the float64 oracle under the GPU's ReLU masks (1e-4 relative norm), at F = 256 where that kernel
    runs.  The same batch pins the per-board BatchNorm statistics of the Winograd conv epilogues
    (round 4: forward sums / squared deviations combined over 81 boards, backward dz sums): the
    BN gamma / beta grads above and the running statistics below."""
    blocks, filters, n = 2, 256, 81
    w = A.random_weights(blocks, filters, seed=13)
    planes, tpol, tval = batch(n, seed=81)
    tr = A.Trainer(blocks, filters, weights=w, max_batch=n)
    tr.compute_gradients(planes, tpol, tval)
    g = tr.grads()
    ref = T.TrainRef(blocks, filters, w)
    rg, _ = ref.grads(planes, tpol, tval, tr.relu_masks(n))
    p = tr.params()
    rs = ref.running_stats_flat(w)
    stats = ~T.trainable_mask(blocks, filters)
    assert np.all(np.abs(p[stats] - rs[stats]) <= 1e-5 * (1 + np.abs(rs[stats])))
    seg, _ = T.segments(blocks, filters)
    zero_bias = bn_fed_biases(blocks)
    checked = 0
    for name, (o, shape, bn) in seg.items():
        size = int(np.prod(shape))
        parts = [(name + ".gamma", o, shape[1]), (name + ".beta", o + shape[1], shape[1])] if bn else [(name, o, size)]
        for pname, off, cnt in parts:
            if pname in zero_bias:
                continue
            a, r = g[off:off + cnt].astype(np.float64), rg[off:off + cnt]
            err = np.linalg.norm(a - r) / max(np.linalg.norm(r), 1e-30)
            assert err <= 1e-4, (pname, err)
            checked += "res_blocks" in pname and pname.endswith("weight")
    assert checked == 2 * blocks


def test_data_parallel_world2_bit_exact(require_gpu):
    """The world > 1 arithmetic of the data-parallel step (training.rs:137-200 sharded over ranks)
    without a second GPU: two trainers on the two halves of a batch, their gradients summed by a
    host reducer (az_trainer_set_host_reducer: the all-reduce RCCL would do, sum of two operands =
    the same float32 sum in either order), then AdamW with world = 2 (gradient scale 1/2 before the
    clip) and the BatchNorm running statistics averaged.  Both ranks end bit-identical, and equal
    to the float32 restatement T.adamw_step(p, g0 + g1, ..., world=2) with averaged statistics.
    Note the reference trains one batch of 512 on one device (training.rs:138): with 512 per rank
    the global batch is 512 x world and BatchNorm sees per-rank statistics."""
    import threading
    blocks, filters, n = 2, 64, 16
    w = A.random_weights(blocks, filters, seed=21)
    planes, tpol, tval = batch(2 * n, seed=22)
    ranks = [A.Trainer(blocks, filters, weights=w, max_batch=n) for _ in range(2)]
    slots, bar = [None, None], threading.Barrier(2, timeout=30)

    def reducer(rank):
        def reduce(buf):
            slots[rank] = buf.copy()
            bar.wait()
            buf[:] = slots[0] + slots[1]
            bar.wait()
        return reduce

    for r, tr in enumerate(ranks):
        tr.set_host_reducer(reducer(r), r, 2)
    mask = T.trainable_mask(blocks, filters)
    m = np.zeros_like(w)
    v = np.zeros_like(w)
    want = w.copy()
    for step, it in enumerate([3, 12]):
        gs, ps = [], []
        for r, tr in enumerate(ranks):
            tr.compute_gradients(planes[r * n:(r + 1) * n], tpol[r * n:(r + 1) * n], tval[r * n:(r + 1) * n])
            gs.append(tr.grads())
            ps.append(tr.params())           # running statistics moved by this rank's forward
        lr = A.get_cyclical_lr(it)
        errs = []
        th = [threading.Thread(target=lambda tr=tr: errs.append(tr.apply(lr))) for tr in ranks]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert errs == [None, None]
        assert np.array_equal(ps[0][mask], want[mask]) and np.array_equal(ps[1][mask], want[mask])
        want, m, v = T.adamw_step(want, gs[0] + gs[1], m, v, mask, step + 1, lr, world=2)
        stats = ~mask
        want[stats] = (ps[0][stats] + ps[1][stats]) * np.float32(0.5)
        got0, got1 = ranks[0].params(), ranks[1].params()
        assert np.array_equal(got0, got1)
        assert np.array_equal(got0, want), np.abs(got0 - want).max()
    assert not np.array_equal(gs[0], gs[1])     # the ranks saw different data


def _run_ranks(fns):
    """Run one callable per rank in its own thread (the ranks meet inside the host reducer);
    re-raise the first failure."""
    import threading
    res, errs = [None] * len(fns), []

    def run(i):
        try:
            res[i] = fns[i]()
        except BaseException as e:          # noqa: B902 -- reported below
            errs.append(e)
    th = [threading.Thread(target=run, args=(i,), daemon=True) for i in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung"
    if errs:
        raise errs[0]
    return res


def _host_reducer_pair():
    import threading
    slots, bar = [None, None], threading.Barrier(2, timeout=60)

    def reducer(rank):
        def reduce(buf):
            slots[rank] = buf.copy()
            bar.wait()
            buf[:] = slots[0] + slots[1]
            bar.wait()
        return reduce
    return reducer


@pytest.mark.parametrize("blocks,filters", [(2, 64), (2, 256)])
def test_sharded_world1_rccl_is_the_plain_step(require_gpu, blocks, filters):
    """az_trainer_set_sharded over a 1-rank RCCL communicator: every BatchNorm's statistics and
    backward sums, the losses and the gradients go through ncclAllReduce, and the step is the
    plain step bit for bit (F = 64: column-sum statistics; F = 256: the Winograd epilogues'
    per-board statistics)."""
    w = A.random_weights(blocks, filters, seed=31)
    planes, tpol, tval = batch(16, seed=32)
    a = A.Trainer(blocks, filters, weights=w, max_batch=16)
    b = A.Trainer(blocks, filters, weights=w, max_batch=16)
    b.set_comm(A.comm_unique_id(), 0, 1)
    b.set_sharded(True)
    for it in range(2):
        la = a.compute_gradients(planes, tpol, tval)
        lb = b.compute_gradients(planes, tpol, tval)
        assert np.allclose(la, lb, rtol=1e-6, atol=0), (la, lb)
        assert np.array_equal(a.grads(), b.grads())
        assert np.array_equal(a.params(), b.params())
        a.apply(A.get_cyclical_lr(it))
        b.apply(A.get_cyclical_lr(it))
        assert np.array_equal(a.params(), b.params())
    # az_trainer_step: the losses ride in the gradient all-reduce; the two head BatchNorms share one
    # exchange per direction -> 2 per tower BN + 2 + 1 collectives per step
    b.exchange_stats(reset=True)
    b.time_exchanges(True)
    for it in range(2, 4):
        la = a.step(planes, tpol, tval, A.get_cyclical_lr(it))
        lb = b.step(planes, tpol, tval, A.get_cyclical_lr(it))
        assert np.allclose(la, lb, rtol=1e-6, atol=0), (la, lb)
        assert np.array_equal(a.params(), b.params())
    n, steps, ms = b.exchange_stats()
    assert steps == 2 and n == 2 * (2 * (1 + 2 * blocks) + 2 + 1), n
    assert ms > 0.0


@pytest.mark.parametrize("split", [256, 200])
def test_sharded_world2_host_reducer_matches_single_batch(require_gpu, split):
    """the reference trains ONE batch of 512 (training.rs:137-159,
    parameters.rs:17) with batch-512 BatchNorm statistics (agent.rs:37,41,115).  Two ranks in
    sharded mode (az_trainer_set_sharded, exchanges through the host reducer), 256 positions each,
    against one rank on all 512, both against the float64 oracle on the 512-position batch under
    each path's own ReLU masks (the two ranks' masks concatenated):
      losses (global means)            |d| <= 1e-5 (1 + |ref|), and against the 1-rank step
      every gradient tensor            <= 1e-4 relative norm vs the oracle (sharded: g0 + g1)
      sharded vs 1-rank, per tensor    <= 1e-2 relative norm (different ReLU branches near 0)
      running statistics               <= 1e-5 vs the oracle; bit-identical on the two ranks
    then the AdamW step: both ranks bit-identical and equal to T.adamw_step(p, g0 + g1, world=1).
    split = 200: unequal shards (200 + 312 positions; the Chan combine weights each rank by its rows,
    the loss and BN backward divide by the global count)."""
    blocks, filters, n = 2, 256, 512
    cuts = [0, split, n]
    w = A.random_weights(blocks, filters, seed=41)
    planes, tpol, tval = batch(n, seed=42)
    one = A.Trainer(blocks, filters, weights=w, max_batch=n)
    l1 = one.compute_gradients(planes, tpol, tval)
    g1, p1, m1 = one.grads(), one.params(), one.relu_masks(n)
    ranks = [A.Trainer(blocks, filters, weights=w, max_batch=cuts[r + 1] - cuts[r]) for r in range(2)]
    red = _host_reducer_pair()
    for r, tr in enumerate(ranks):
        tr.set_host_reducer(red(r), r, 2)
        tr.set_sharded(True)
    sl = [slice(cuts[r], cuts[r + 1]) for r in range(2)]
    ls = _run_ranks([lambda r=r, tr=tr: tr.compute_gradients(planes[sl[r]], tpol[sl[r]], tval[sl[r]])
                     for r, tr in enumerate(ranks)])
    assert ls[0] == ls[1]                     # global means on both ranks
    gs = [tr.grads() for tr in ranks]
    ps = [tr.params() for tr in ranks]
    ms = [tr.relu_masks(cuts[r + 1] - cuts[r]) for r, tr in enumerate(ranks)]
    msh = [np.concatenate([a, b]) for a, b in zip(ms[0], ms[1])]
    gsh = gs[0].astype(np.float64) + gs[1].astype(np.float64)
    stats = ~T.trainable_mask(blocks, filters)
    assert np.array_equal(ps[0][stats], ps[1][stats])
    seg, _ = T.segments(blocks, filters)
    zero_bias = bn_fed_biases(blocks)
    for name_path, (loss, g, p, masks) in {"1-rank": (l1, g1, p1, m1), "sharded": (ls[0], gsh, ps[0], msh)}.items():
        ref = T.TrainRef(blocks, filters, w)
        rg, (rpl, rvl) = ref.grads(planes, tpol, tval, masks)
        assert abs(loss[0] - rpl) <= 1e-5 * (1 + abs(rpl)) and abs(loss[1] - rvl) <= 1e-5 * (1 + abs(rvl)), \
            (name_path, loss, rpl, rvl)
        rs = ref.running_stats_flat(w)
        assert np.all(np.abs(p[stats] - rs[stats]) <= 1e-5 * (1 + np.abs(rs[stats]))), name_path
        for name, (o, shape, bn) in seg.items():
            parts = [(name + ".gamma", o, shape[1]), (name + ".beta", o + shape[1], shape[1])] if bn else \
                [(name, o, int(np.prod(shape)))]
            for pname, off, cnt in parts:
                a = np.asarray(g[off:off + cnt], np.float64)
                if pname in zero_bias:
                    assert np.abs(a).max() <= 1e-5, (name_path, pname)
                    continue
                r = rg[off:off + cnt]
                err = np.linalg.norm(a - r) / max(np.linalg.norm(r), 1e-30)
                assert err <= 1e-4, (name_path, pname, err)
    assert abs(ls[0][0] - l1[0]) <= 1e-5 * (1 + abs(l1[0])) and abs(ls[0][1] - l1[1]) <= 1e-5 * (1 + abs(l1[1]))
    for name, (o, shape, bn) in seg.items():
        if name in zero_bias:
            continue
        cnt = 2 * shape[1] if bn else int(np.prod(shape))
        r = g1[o:o + cnt].astype(np.float64)
        assert np.linalg.norm(gsh[o:o + cnt] - r) <= 1e-2 * max(np.linalg.norm(r), 1e-30), name
    # the optimizer step: gradients summed by the reducer, applied unscaled (global-mean loss)
    lr = A.get_cyclical_lr(4)
    _run_ranks([lambda tr=tr: tr.apply(lr) for tr in ranks])
    mask = T.trainable_mask(blocks, filters)
    want, _, _ = T.adamw_step(ps[0], gs[0] + gs[1], np.zeros_like(w), np.zeros_like(w), mask, 1, lr, world=1)
    got0, got1 = ranks[0].params(), ranks[1].params()
    assert np.array_equal(got0, got1)
    assert np.array_equal(got0, want), np.abs(got0 - want).max()


def _allgather_pair():
    import threading
    slots, bar = [None, None], threading.Barrier(2, timeout=120)

    def allgather(rank):
        def ag(payload):
            slots[rank] = payload
            bar.wait()
            out = list(slots)
            bar.wait()
            return out
        return ag
    return allgather


def _host_reducer_n(world):
    """In-process host reducer for `world` ranks as threads: the element-wise sum in rank order."""
    import threading
    slots, bar = [None] * world, threading.Barrier(world, timeout=60)

    def reducer(rank):
        def reduce(buf):
            slots[rank] = buf.copy()
            bar.wait()
            acc = slots[0].copy()
            for r in range(1, world):
                acc += slots[r]
            buf[:] = acc
            bar.wait()
        return reduce
    return reducer


def test_sharded_world4_host_reducer_matches_single_batch(require_gpu):
    """The sharded step at world 4 (round 6: gathers, rank-order sums): four ranks as threads on one
    GPU with unequal shards 100 + 156 + 128 + 128 of one 512 batch (the 100 / 128 shards take the
    quarter-channel convs, 156 the one-board kernel), against one rank on all 512: losses <= 1e-5,
    every gradient tensor summed over the ranks <= 1e-2 relative norm (ReLU branches near 0),
    running statistics <= 1e-5 and bit-identical on the four ranks, and the AdamW step leaves the
    four ranks bit-identical."""
    blocks, filters, n = 2, 256, 512
    cuts = [0, 100, 256, 384, 512]
    w = A.random_weights(blocks, filters, seed=43)
    planes, tpol, tval = batch(n, seed=44)
    one = A.Trainer(blocks, filters, weights=w, max_batch=n)
    l1 = one.compute_gradients(planes, tpol, tval)
    g1, p1 = one.grads().astype(np.float64), one.params()
    red = _host_reducer_n(4)
    ranks = [A.Trainer(blocks, filters, weights=w, max_batch=cuts[r + 1] - cuts[r]) for r in range(4)]
    for r, tr in enumerate(ranks):
        tr.set_host_reducer(red(r), r, 4)
        tr.set_sharded(True)
    sl = [slice(cuts[r], cuts[r + 1]) for r in range(4)]
    ls = _run_ranks([lambda r=r, tr=tr: tr.compute_gradients(planes[sl[r]], tpol[sl[r]], tval[sl[r]])
                     for r, tr in enumerate(ranks)])
    assert all(l == ls[0] for l in ls)
    assert abs(ls[0][0] - l1[0]) <= 1e-5 * (1 + abs(l1[0])) and abs(ls[0][1] - l1[1]) <= 1e-5 * (1 + abs(l1[1]))
    gs = [tr.grads().astype(np.float64) for tr in ranks]
    gsum = gs[0] + gs[1] + gs[2] + gs[3]
    ps = [tr.params() for tr in ranks]
    stats = ~T.trainable_mask(blocks, filters)
    for p in ps[1:]:
        assert np.array_equal(p[stats], ps[0][stats])
    assert np.all(np.abs(ps[0][stats] - p1[stats]) <= 1e-5 * (1 + np.abs(p1[stats])))
    seg, _ = T.segments(blocks, filters)
    zero_bias = bn_fed_biases(blocks)
    for name, (o, shape, bn) in seg.items():
        if name in zero_bias:
            continue
        cnt = 2 * shape[1] if bn else int(np.prod(shape))
        r = g1[o:o + cnt]
        assert np.linalg.norm(gsum[o:o + cnt] - r) <= 1e-2 * max(np.linalg.norm(r), 1e-30), name
    lr = A.get_cyclical_lr(3)
    _run_ranks([lambda tr=tr: tr.apply(lr) for tr in ranks])
    after = [tr.params() for tr in ranks]
    for p in after[1:]:
        assert np.array_equal(p, after[0])


def test_train_loop_one_global_buffer_two_ranks(require_gpu, tmp_path):
    """train() at world 2 computes the reference's train() (training.rs:81-159,
    memory.rs:41-96) -- two ranks as threads on one GPU, gradient / BatchNorm exchanges through a host
    reducer, EpisodeSteps through an in-process allgather:
      * each rank plays its own games, and both replicas of the ONE replay buffer end byte-identical
        (every rank's steps added in (rank, drain) order) and hold both ranks' steps;
      * every step both ranks draw the same global batch of 64 (shared sample seed) and train the
        two contiguous halves of it (sharded BatchNorm, the default at world > 1);
      * the two trainers end bit-identical, and within the sharded tolerance of ONE trainer stepped
        on the same global batches: losses <= 1e-5 (1 + |l|), BatchNorm running statistics
        <= 1e-5, the AdamW parameter update <= 1e-2 relative norm (sign flips of near-zero
        gradients under different ReLU branches, as in the single-step test)."""
    red, ag = _host_reducer_pair(), _allgather_pair()
    logs = [[], []]
    steps, gb, seed = 2, 64, 5

    def run(r):
        def lb(it, b, planes, pol, val, lo, hi):
            logs[r].append((planes.copy(), pol.copy(), val.copy(), lo, hi))
        return A.train(1, blocks=2, filters=256, games=16, sims=8, min_replay=64, train_steps=steps, batch_size=gb,
                       seed=seed, reducer=(red(r), r, 2), allgather=ag(r), log_batch=lb)
    out = _run_ranks([lambda r=r: run(r) for r in range(2)])
    (t0, rep0, h0), (t1, rep1, h1) = out
    rep0.save(tmp_path / "r0")
    rep1.save(tmp_path / "r1")
    assert (tmp_path / "r0").read_bytes() == (tmp_path / "r1").read_bytes()
    assert h0[0]["shared_replay"] and h0[0]["shard_batch"]
    assert h0[0]["episode_steps_global"] == h1[0]["episode_steps_global"] == \
        h0[0]["episode_steps"] + h1[0]["episode_steps"]
    assert h0[0]["new_unique"] == h1[0]["new_unique"] == len(rep0) >= 64
    assert h0[0]["policy_loss"] == h1[0]["policy_loss"] and h0[0]["value_loss"] == h1[0]["value_loss"]
    assert len(logs[0]) == len(logs[1]) == steps
    for a, b in zip(logs[0], logs[1]):
        for x, y in zip(a[:3], b[:3]):
            assert np.array_equal(x, y)                       # the same global batch on both ranks
        assert a[0].shape[0] == gb and (a[3], a[4], b[3], b[4]) == (0, gb // 2, gb // 2, gb)
    p0, p1 = t0.params(), t1.params()
    assert np.array_equal(p0, p1)
    w0 = A.random_weights(2, 256, seed)
    one = A.Trainer(2, 256, weights=w0, max_batch=gb)
    lone = [one.step(pl, po, va, A.get_cyclical_lr(0)) for pl, po, va, _, _ in logs[0]]
    pone = one.params()
    for k, name in ((0, "policy_loss"), (1, "value_loss")):
        want = sum(l[k] for l in lone) / steps
        assert abs(h0[0][name] - want) <= 1e-5 * (1 + abs(want)), (name, h0[0][name], want)
    mask = T.trainable_mask(2, 256)
    st = ~mask
    assert np.all(np.abs(p0[st] - pone[st]) <= 1e-5 * (1 + np.abs(pone[st])))
    d_sh, d_one = (p0 - w0)[mask].astype(np.float64), (pone - w0)[mask].astype(np.float64)
    assert np.linalg.norm(d_sh - d_one) <= 1e-2 * np.linalg.norm(d_one), np.linalg.norm(d_sh - d_one) / np.linalg.norm(d_one)


def test_train_loop_per_rank_opt_in_two_ranks(require_gpu):
    """The labelled opt-ins (shared_replay=False, shard_batch=False): each rank its own buffer and
    its own batch of batch_size, per-rank BatchNorm, averaged gradients -- the trainers still end
    bit-identical and the losses are finite."""
    red = _host_reducer_pair()
    out = _run_ranks([lambda r=r: A.train(1, blocks=2, filters=256, games=16, sims=8, min_replay=64, train_steps=2,
                                          batch_size=32, seed=5, reducer=(red(r), r, 2), shard_batch=False,
                                          shared_replay=False)
                      for r in range(2)])
    (t0, rep0, h0), (t1, rep1, h1) = out
    assert not h0[0]["shared_replay"] and not h0[0]["shard_batch"]
    assert np.isfinite(h0[0]["policy_loss"]) and np.isfinite(h0[0]["value_loss"])
    assert np.array_equal(t0.params(), t1.params())
    assert len(rep0) >= 64 and len(rep1) >= 64


def test_winograd_trainer_more_than_1024_positions(require_gpu):
    """the fused BN backward keeps per-board bias partials (B x [2][F]) in slots sized for
    max_batch, so a Winograd trainer takes more than 1024 positions per step; its gradients equal
    the unfused backward's (AZ_TRAIN_FUSE_BN=0) within 1e-5 relative norm."""
    import os
    w = A.random_weights(1, 256, seed=61)
    planes, tpol, tval = batch(1100, seed=62)
    a = A.Trainer(1, 256, weights=w, max_batch=1100)
    la = a.compute_gradients(planes, tpol, tval)
    old = os.environ.get("AZ_TRAIN_FUSE_BN")
    os.environ["AZ_TRAIN_FUSE_BN"] = "0"
    try:
        b = A.Trainer(1, 256, weights=w, max_batch=1100)
    finally:
        if old is None:
            del os.environ["AZ_TRAIN_FUSE_BN"]
        else:
            os.environ["AZ_TRAIN_FUSE_BN"] = old
    lb = b.compute_gradients(planes, tpol, tval)
    assert np.allclose(la, lb, rtol=1e-6), (la, lb)
    ga, gb = a.grads().astype(np.float64), b.grads().astype(np.float64)
    assert np.all(np.isfinite(ga))
    assert np.linalg.norm(ga - gb) <= 1e-5 * np.linalg.norm(gb), np.linalg.norm(ga - gb) / np.linalg.norm(gb)

"""The N > 1 rank path of bench.py with the REAL engine on a one-GPU box (--same-device maps every
rank to device 0 and skips the RCCL training leg).  It exercises the spawn, per-rank seeds, barrier,
max-over-ranks timing and counter sums with libaz doing the self-play -- not a scaling measurement
(no scaling curve has been measured: the driver had no 8-GPU node)."""
import pytest

from test_dist import _bench

pytestmark = pytest.mark.gpu


def test_bench_two_ranks_real_engine_on_one_gpu(require_gpu):
    G, S, K, steps = 32, 16, 8, 2     # the window ends mid-move: root visits non-zero
    rc, lines, err = _bench(["--gpus", "2", "--same-device", "--steps", str(steps), "--warmup", "1",
                             "--games", str(G), "--sims", str(S), "--sims-per-step", str(K), "--blocks", "2",
                             "--filters", "64", "--bf16-steps", "0", "--no-cpu-baseline", "--train-steps", "0",
                             "--games-leg", "0"], timeout=300)
    assert rc == 0, err[-3000:]
    assert len(lines) == 1
    r = lines[0]
    assert r["n_gpus"] == 2 and r["steps"] == steps and r["dtype"] == "f32"
    sims = r["value"] * r["ms_per_step"] * 1e-3 * steps
    assert abs(sims - 2 * G * K * steps) < 1e-6 * sims
    assert r["evals_per_sim"] > 0.5
    d = r["rank_root_digests"]
    assert len(d) == 2 and d[0] != d[1]          # distinct games per rank (per-rank seeds)
    assert "TEST MODE" in r["config"]["parallelism"]

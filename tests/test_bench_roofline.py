"""bench.py's roofline bookkeeping against the committed hardware counters (CPU only): the executed
MFMA FLOPs per row that `roofline.frac` divides by the f32 peak must be the work the kernel really
issues -- PMC SQ_INSTS_MFMA x 2048 FLOP (v_mfma_f32_16x16x4_f32) / 2048 rows per launch -- and the
HBM traffic figure must come from the PMC summary of the current tower."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_executed_flops_equal_pmc_mfma_count():
    path = bench.PMC_SUMMARY["f32"]
    with open(path) as f:
        s = json.load(f)
    per_row_pmc = s["SQ_INSTS_MFMA"] * 2048.0 / 2048.0          # 2048 FLOP per MFMA, 2048 rows per launch
    assert bench.tower_exec_flop_per_row(20, 256, "f32", True) == per_row_pmc


def test_traffic_comes_from_the_current_summary():
    traffic, src = bench.pmc_traffic(2048, 20, 256, "f32", True)
    with open(os.path.join(ROOT, src)) as f:
        s = json.load(f)
    assert traffic == s["traffic_bytes"] and traffic > 0
    # other workloads have no PMC figure
    assert bench.pmc_traffic(256, 6, 64, "f32", True) == (None, None)


def test_executed_training_flops_use_winograd_at_256():
    direct = bench.net_flop_per_eval(20, 256)
    wino = bench.executed_flop_per_eval(20, 256, True)
    # the 40 residual convs execute 16 x 16 instead of 64 x 9 multiply-adds per output channel pair
    resid = 2.0 * 64.0 * 18.0 * 20 * 256 * 256
    assert abs((direct - wino) - resid * (1 - 256.0 / 576.0)) < 1.0
    assert bench.executed_flop_per_eval(6, 64, False) == bench.net_flop_per_eval(6, 64)

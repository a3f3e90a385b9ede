"""Summarise tools/pmc_run.sh output for one kernel (per-launch averages).
HBM bytes per MI355X_MICROARCH.md 'HBM': FETCH_SIZE reads half the bytes of wide coalesced
streaming reads on gfx950 (x2 correction), WRITE_SIZE exact for 16-B stores; both in KB.
Usage: python tools/pmc_summary.py <outdir> [kernel-name substring, default tower_kernel] [MFMA cycles/SIMD:
16 for v_mfma_f32_16x16x32_bf16 (default), 32 for v_mfma_f32_16x16x4_f32]"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "tower_kernel"
mfma_cyc = float(sys.argv[3]) if len(sys.argv) > 3 else 16.0
res = {"kernel_pattern": pat}
durs = []
for sub in ("fetch", "write", "sq", "tcc", "cyc"):
    f = os.path.join(d, sub, sub + "_counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, v in agg.items():
        res[c] = sum(v.values()) / len(v)
        res[c + "_launches"] = len(v)
    for kt in glob.glob(os.path.join(d, sub, "*kernel_trace.csv")):
        for r in csv.DictReader(open(kt)):
            if pat in r["Kernel_Name"]:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
if durs:
    res["profiled_avg_launch_s"] = sum(durs) / len(durs)
if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
    res["hbm_read_bytes_corrected"] = res["FETCH_SIZE"] * 1024 * 2
    res["hbm_write_bytes"] = res["WRITE_SIZE"] * 1024
    res["traffic_bytes"] = res["hbm_read_bytes_corrected"] + res["hbm_write_bytes"]
if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
    res["l2_hit_rate"] = res["TCC_HIT_sum"] / max(res["TCC_HIT_sum"] + res["TCC_MISS_sum"], 1)
if "SQ_LDS_IDX_ACTIVE" in res:
    res["lds_conflict_frac"] = res["SQ_LDS_BANK_CONFLICT"] / max(res["SQ_LDS_IDX_ACTIVE"], 1)
if "SQ_WAVE_CYCLES" in res:
    res["wait_frac"] = res["SQ_WAIT_ANY"] / res["SQ_WAVE_CYCLES"]
    res["wait_inst_frac"] = res["SQ_WAIT_INST_ANY"] / res["SQ_WAVE_CYCLES"]
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs on the chip
    res["mfma_busy_frac"] = res["SQ_VALU_MFMA_BUSY_CYCLES"] / (res["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if durs:
        res["effective_clock_ghz"] = res["GRBM_GUI_ACTIVE"] / 8 / res["profiled_avg_launch_s"] / 1e9
if "SQ_INSTS_MFMA" in res and "GRBM_GUI_ACTIVE" in res:
    # v_mfma_f32_16x16x32_bf16 = 16 cycles, v_mfma_f32_16x16x4_f32 = 32 (MI355X_MICROARCH.md cycle constants)
    res["mfma_issue_frac"] = res["SQ_INSTS_MFMA"] * mfma_cyc / (res["GRBM_GUI_ACTIVE"] / 8 * 1024)
print(json.dumps(res, indent=1))

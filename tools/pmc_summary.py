"""Summarise tools/pmc.sh output: mean per-dispatch counter values of the conv
kernel (skipping the first, cold dispatch) plus derived ratios."""
import csv
import glob
import json
import os
import sys


def load(d):
    vals = {}
    for f in glob.glob(os.path.join(d, "g*", "run_counter_collection.csv")):
        rows = list(csv.DictReader(open(f)))
        by = {}
        for r in rows:
            by.setdefault(r["Counter_Name"], []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        for k, v in by.items():
            v.sort()
            v = v[1:] if len(v) > 1 else v
            vals[k] = sum(x for _, x in v) / len(v)
    return vals


def main(d, mfma_gflop=None):
    """mfma_gflop: the useful bf16 MFMA work of one dispatch (GFLOP, bf16x3 = 3x the conv's
    FLOPs): adds the matrix pipe's busy fraction of the SIMD-cycles and the useful part of it
    (one v_mfma_f32_16x16x32_bf16 = 16384 FLOP in 16 cycles)."""
    v = load(d)
    out = {k: round(x, 1) for k, x in sorted(v.items())}
    if "SQ_WAVE_CYCLES" in v:
        wc = v["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in v:
                out["frac_" + k] = round(v[k] / wc, 3)
    if "FETCH_SIZE" in v:
        out["hbm_read_bytes_x2_corrected"] = v["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in v:
        out["hbm_write_bytes"] = v["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
        out["l2_hit_rate"] = round(v["TCC_HIT_sum"] / max(1.0, v["TCC_HIT_sum"] + v["TCC_MISS_sum"]), 3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in v and "GRBM_GUI_ACTIVE" in v:
        simd_cycles = 1024 * v["GRBM_GUI_ACTIVE"] / 8  # GRBM_GUI_ACTIVE sums the 8 XCDs
        out["mfma_busy_frac"] = round(v["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles, 3)
        if mfma_gflop:
            out["mfma_useful_gflop"] = mfma_gflop  # the argument the useful fraction is computed from
            out["mfma_useful_frac"] = round(mfma_gflop * 1e9 / 16384 * 16 / simd_cycles, 3)
    if "SQ_LDS_BANK_CONFLICT" in v and "SQ_LDS_IDX_ACTIVE" in v:
        out["lds_conflict_frac"] = round(v["SQ_LDS_BANK_CONFLICT"] / max(1.0, v["SQ_LDS_IDX_ACTIVE"]), 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)

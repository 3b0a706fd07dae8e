"""Summarise the PMC passes of tools/pmc_passes.sh into profiles/valu_pmc.json and
profiles/traffic_k_decompress.json (the files bench.py folds into its roofline object).

  python tools/pmc_summary.py gpurun_out   # reads gpurun_out/pmc_{valu,int,fetch,write}/run_counter_collection.csv
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 1 << 20
KERNELS = ["k_decompress", "k_challenge", "k_msm_accum_dma", "k_msm_scatter", "k_coef"]
MAD_CYC, OTHER_CYC, SIMDS = 4.46, 2.5, 1024     # profiles/r01_valu_rates.txt; 256 CU x 4 SIMD


def medians(path):
    """{kernel short name: {counter: median over this kernel's dispatches with its most frequent grid}}
    (the bench's steady-state batch launches)"""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("edc::", "")
            if name in KERNELS:
                rows.append((name, int(r["Grid_Size"]), r["Counter_Name"], float(r["Counter_Value"])))
    # the steady-state dispatches: the grid size seen most often per kernel (the first batch of a
    # context runs without a key-ratio hint, so its MSM plan and grids differ)
    seen = defaultdict(lambda: defaultdict(int))
    for name, g, _, _ in rows:
        seen[name][g] += 1
    top = {name: max(gs.items(), key=lambda x: (x[1], x[0]))[0] for name, gs in seen.items()}
    per = defaultdict(lambda: defaultdict(list))
    for name, g, c, v in rows:
        if g == top[name]:
            per[name][c].append(v)
    return {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in per.items()}


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
    p = {x: medians(os.path.join(d, f"pmc_{x}", "run_counter_collection.csv")) for x in ("valu", "int", "fetch", "write")}
    out = {"method": "rocprofv3 --pmc, two passes (SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES "
                     "GRBM_GUI_ACTIVE; SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS) over bench.py "
                     "--steps 2 --inflight 1 (tools/pmc_passes.sh, tools/pmc_summary.py), median over launches, "
                     "n = 2^20 (configs[2]); counters are wave-instructions summed over the chip; GRBM_GUI_ACTIVE is "
                     "summed over the 8 XCDs. INT64 wave-instructions are almost all v_mad_u64_u32. issue_bound = "
                     "INT64 x 4.46 + (VALU - INT64) x 2.5 cycles (profiles/r01_valu_rates.txt) over 1024 SIMDs.",
           "n": N, "kernels": {}}
    for k in KERNELS:
        if k not in p["valu"] or k not in p["int"]:
            continue
        a, b = p["valu"][k], p["int"][k]
        waves, valu, i64 = a["SQ_WAVES"], a["SQ_INSTS_VALU"], b["SQ_INSTS_VALU_INT64"]
        cyc = a["GRBM_GUI_ACTIVE"] / 8
        bound = (i64 * MAD_CYC + (valu - i64) * OTHER_CYC) / SIMDS
        out["kernels"][k] = {
            "waves": waves, "valu_insts": valu, "int64_insts": i64, "int32_insts": b["SQ_INSTS_VALU_INT32"],
            "salu_insts": b["SQ_INSTS_SALU"], "lds_insts": b["SQ_INSTS_LDS"], "kernel_cycles": round(cyc),
            "valu_per_wave": round(valu / waves), "cycles_per_valu_per_simd": round(cyc / (valu / SIMDS), 3),
            "issue_bound_cycles": round(bound), "valu_issue_frac": round(bound / cyc, 3),
            "int64_lane_ops_per_cycle_per_simd": round(i64 * 64 / SIMDS / cyc, 2)}
    with open(os.path.join(ROOT, "profiles", "valu_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    fk, wk = p["fetch"]["k_decompress"]["FETCH_SIZE"], p["write"]["k_decompress"]["WRITE_SIZE"]
    t = {"kernel": "k_decompress (ZIP215 decode of every R_i -> affine Niels records)", "n": N,
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/pmc_passes.sh: "
                   "bench.py --steps 2 --inflight 1), median over launches; FETCH_SIZE x2 per the gfx950 correction "
                   "(MI355X_MICROARCH.md HBM section); units KB",
         "fetch_size_kb_raw": fk, "write_size_kb": wk, "fetch_bytes": int(fk * 1024 * 2), "write_bytes": int(wk * 1024),
         "hbm_bytes_per_launch": int(fk * 1024 * 2 + wk * 1024), "algorithmic_bytes_per_launch": N * (32 + 112),
         "note": "reads cover whole 64-byte signature records (R shares the cache line with s); writes are whole "
                 "128-byte point records"}
    with open(os.path.join(ROOT, "profiles", "traffic_k_decompress.json"), "w") as f:
        json.dump(t, f, indent=1)
    # MSM traffic: the scatter writes 8-byte entries (8 windows x n R digits at configs[2]); the
    # accumulation gathers one 112-byte row per entry
    entries = 8 * N
    msm = {"n": N, "entries": entries, "entry_bytes": entries * 8,
           "k_msm_scatter": {"write_bytes": int(p["write"].get("k_msm_scatter", {}).get("WRITE_SIZE", 0) * 1024),
                             "fetch_bytes": int(p["fetch"].get("k_msm_scatter", {}).get("FETCH_SIZE", 0) * 1024 * 2)},
           "k_msm_accum_dma": {"fetch_bytes": int(p["fetch"].get("k_msm_accum_dma", {}).get("FETCH_SIZE", 0) * 1024 * 2),
                               "write_bytes": int(p["write"].get("k_msm_accum_dma", {}).get("WRITE_SIZE", 0) * 1024),
                               "algorithmic_gather_bytes": entries * 112}}
    msm["k_msm_scatter"]["write_over_entry_bytes"] = round(msm["k_msm_scatter"]["write_bytes"] / (entries * 8), 3)
    if "k_msm_accum_dma" in out["kernels"]:
        msm["k_msm_accum_dma"]["cycles_per_valu_per_simd"] = out["kernels"]["k_msm_accum_dma"]["cycles_per_valu_per_simd"]
    with open(os.path.join(ROOT, "profiles", "traffic_msm.json"), "w") as f:
        json.dump(msm, f, indent=1)
    print(json.dumps(msm, indent=1))
    print(json.dumps(out["kernels"], indent=1))
    print(json.dumps(t, indent=1))


if __name__ == "__main__":
    main()

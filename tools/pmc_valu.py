#!/usr/bin/env python3
"""VALU utilisation per kernel from tools/pmc_valu.sh output.

    python tools/pmc_valu.py C4 gpurun_out profiles/r03/pmc_valu_C4.json [pairs_json]

Per kernel dispatch (rocprofv3 counter_collection.csv, one row per counter):
  clock          = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs,
                   MI355X_MICROARCH.md 'DVFS give-back') / kernel wall time
  valu_issue_frac = SQ_INSTS_VALU wave-instructions / (1024 SIMDs x cycles / 2):
                   a wave64 VALU instruction issues over 2 cycles on a SIMD32
                   (cdna_hip_programming.md), so 1024 SIMDs sustain one
                   instruction per SIMD every 2 cycles -- the issue roofline the
                   FP32 vector peak (157.3 TF) is quoted on;
  valu_busy      = SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (1024 x cycles);
  insts_per_pair = SQ_INSTS_VALU x 64 / VRL pairs (lanes per instruction /
                   pairs), given the pair count of the dispatch;
  pair_rate_at_valu_peak = 1024 x 32 lanes x clock / insts_per_pair.
"""
import csv
import glob
import json
import os
import sys

KEYS = {"k_refine": "refine", "k_gather_clustered": "render", "k_gather_brute": "render",
        "k_build_R_blocks": "rbuild", "k_build_R_strict": "rbuild"}
NSIMD = 1024


def main():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pmc_summary import build_id_of_run
    cfg, root, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    bid = build_id_of_run(os.path.join(root, f"pmc_{cfg}_VALU.log"))
    pairs = json.load(open(sys.argv[4])) if len(sys.argv) > 4 else {}
    rows = {}
    for fn in glob.glob(os.path.join(root, f"pmc_{cfg}_VALU", "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"]
                key = next((v for k, v in KEYS.items() if k + "(" in name or k + "<" in name), None)
                if key is None:
                    continue
                d = rows.setdefault((key, r["Dispatch_Id"]), {"kernel": name.split("(")[0]})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                if "Start_Timestamp" in r:
                    d["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = {}
    for (key, _), d in rows.items():
        ns = d.get("ns")
        cyc = d["GRBM_GUI_ACTIVE"] / 8.0
        rec = {"kernel": d["kernel"], "config": cfg, "build_id": bid, "ms": ns / 1e6 if ns else None,
               "clock_ghz": cyc / ns if ns else None,
               "valu_insts": d["SQ_INSTS_VALU"], "valu_trans_f32": d.get("SQ_INSTS_VALU_TRANS_F32"),
               "salu_insts": d.get("SQ_INSTS_SALU"), "lds_insts": d.get("SQ_INSTS_LDS"),
               "waves": d.get("SQ_WAVES"),
               "valu_issue_frac": d["SQ_INSTS_VALU"] / (NSIMD * cyc / 2.0),
               "valu_busy": d["SQ_ACTIVE_INST_VALU"] * 4.0 / (NSIMD * cyc)}
        if key in pairs:
            p = pairs[key]
            rec["pairs"] = p
            rec["insts_per_pair"] = d["SQ_INSTS_VALU"] * 64.0 / p
            if ns:
                rec["pair_rate"] = p / (ns * 1e-9)
                rec["pair_rate_at_valu_peak"] = NSIMD * 32 * (cyc / ns * 1e9) / rec["insts_per_pair"]
        out.setdefault(key, []).append(rec)
    res = {k: v[-1] for k, v in out.items()}
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    for k, r in res.items():
        print(k, json.dumps({x: (round(y, 4) if isinstance(y, float) else y) for x, y in r.items()}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where the waves of the step's kernels spend their cycles, from the two
rocprofv3 --pmc passes of tools/pmc_wait2.sh (C4, one bench step):

    python tools/pmc_wait_summary.py TAG gpurun_out out.json [tree]

Counters are summed over the launches of each kernel; the ratios are to
SQ_WAVE_CYCLES (wait on anything, on an instruction dependency, issuing any /
VALU / LDS), and the LDS bank-conflict cycles per wave cycle."""
import csv
import glob
import json
import os
import sys

KEYS = ("k_refine", "k_gather_clustered", "k_gather_brute", "k_build_R_strict", "k_build_R_blocks")
RATIOS = ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
          "SQ_WAIT_INST_LDS")


def collect(d, acc):
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                key = next((k for k in KEYS if k + "(" in name or k + "<" in name), None)
                if key is None:
                    continue
                c = acc.setdefault(key, {})
                c[row["Counter_Name"]] = c.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])


def main():
    tag, root, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    tree = sys.argv[4] if len(sys.argv) > 4 else None
    acc = {}
    for p in (1, 2):
        collect(os.path.join(root, f"pmc_{tag}_{p}"), acc)
    out = {"source": f"tools/pmc_wait2.sh {tag} (C4, bench.py --steps 1, two --pmc passes, counters summed over "
                     "the launches of each kernel)", "tree": tree, "kernels": {}}
    for key, c in sorted(acc.items()):
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        out["kernels"][key] = {
            "counters": c,
            "ratios_to_SQ_WAVE_CYCLES": {r: (c[r] / wc if wc and r in c else None) for r in RATIOS},
            "lds_bank_conflict_per_wave_cycle": (c["SQ_LDS_BANK_CONFLICT"] / wc
                                                 if wc and "SQ_LDS_BANK_CONFLICT" in c else None),
        }
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v["ratios_to_SQ_WAVE_CYCLES"] for k, v in out["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()

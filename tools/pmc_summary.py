#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch from tools/pmc_traffic.sh output.

    python tools/pmc_summary.py C4 gpurun_out profiles/r01_pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are kB per dispatch.  MI355X_MICROARCH.md (HBM): on
gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane coalesced streaming
reads, so the read bytes are doubled; tools/pmc_calib.hip confirms the same
factor for the refinement's 8-B-per-lane loads (1 GiB read: 536.9 MB
reported) and shows that an agent-scope atomic counts 64 B of WRITE_SIZE.  The
bench reads the "hbm_bytes_per_launch" of the record whose config and
kernel_key match."""
import csv
import glob
import json
import os
import sys

KEYS = {"k_refine": "refine", "k_gather_clustered": "render", "k_gather_brute": "render",
        "k_build_R_blocks": "rbuild", "k_build_R_strict": "rbuild"}


def per_kernel(d, counter):
    out = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != counter:
                    continue
                name = row["Kernel_Name"]
                key = next((v for k, v in KEYS.items() if k + "(" in name or k + "<" in name), None)
                if key is None:
                    continue
                out.setdefault(key, []).append(float(row["Counter_Value"]) * 1024.0)
    return out


def build_id_of_run(*logs):
    """alvrl_build_id() of the library the profiled bench run loaded (its JSON
    line's build_mode), so that bench.py can refuse counters of another tree."""
    ids = set()
    for lg in logs:
        try:
            with open(lg) as f:
                for line in f:
                    if line.startswith("{") and "build_mode" in line:
                        ids.add(json.loads(line)["build_mode"]["build_id"])
        except (OSError, ValueError, KeyError):
            pass
    return ids.pop() if len(ids) == 1 else None


def main():
    cfg, root, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    bid = build_id_of_run(os.path.join(root, f"pmc_{cfg}_FETCH_SIZE.log"), os.path.join(root, f"pmc_{cfg}_WRITE_SIZE.log"))
    fetch = per_kernel(os.path.join(root, f"pmc_{cfg}_FETCH_SIZE"), "FETCH_SIZE")
    write = per_kernel(os.path.join(root, f"pmc_{cfg}_WRITE_SIZE"), "WRITE_SIZE")
    try:
        with open(dst) as f:
            recs = json.load(f)
        recs = recs if isinstance(recs, list) else [recs]
    except (OSError, ValueError):
        recs = []
    recs = [r for r in recs if r.get("config") != cfg]
    for key in sorted(fetch):
        fb = sum(fetch[key]) / len(fetch[key])
        wb = sum(write.get(key, [0.0])) / max(1, len(write.get(key, [])))
        recs.append({
            "config": cfg, "kernel_key": key, "launches": len(fetch[key]), "build_id": bid,
            "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE, separate passes",
            "FETCH_SIZE_bytes": fb, "WRITE_SIZE_bytes": wb,
            "correction": "FETCH_SIZE x2 (gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md HBM;"
                          " the same factor for 8-B-per-lane loads, tools/pmc_calib.hip)",
            "hbm_bytes_per_launch": 2.0 * fb + wb,
        })
    with open(dst, "w") as f:
        json.dump(recs, f, indent=1)
    print(json.dumps([r for r in recs if r["config"] == cfg], indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""bench.py's records_mode() alone (the plugin's records mode at C4: the
host-cast ABI with renderBlock-sized host calls from 16 threads), block sizes
128 and 32.  Session tool.

    python tools/records_mode_bench.py [--config C4] [--blocks 128,32]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mitsuba-alvrl_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--blocks", default="128,32")
    a = ap.parse_args()
    import bench
    import alvrl
    cfg = bench.CONFIGS[a.config]
    scene = alvrl.scene_default(cfg["w"], cfg["h"])
    vrls, pc = alvrl.trace_vrls(scene, cfg["nvrl"], seed=bench.SEED_VRL)
    r = bench.records_mode(cfg, vrls, pc, 10, 0, blocks=tuple(int(b) for b in a.blocks.split(",")))
    print(json.dumps(dict(r, build_id=alvrl.build_info()["build_id"])), flush=True)


if __name__ == "__main__":
    main()

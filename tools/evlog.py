"""Reads the developer event log of a -DALVRL_EVLOG build (ALVRL_EVLOG=file,
refine.hip EVLOG): per launch, the leaders' setup phases, the phases of every
split of at least --min columns, and the divided splits' parts.  Times in us
from the launch's first event (the wall clock runs at 100 MHz).

  python tools/evlog.py gpurun_out/ev.log [--launch -1] [--min 16384] [--rows 214]
"""
import argparse
import collections

LEAD = {1: "start", 2: "colw", 3: "init", 4: "uncl", 5: "end"}
SPLIT = {11: "samp", 12: "dir", 13: "proj", 14: "sort", 15: "var", 16: "argmin"}
KIND = {0: "var", 1: "proj", 2: "colw", 3: "init"}


def launches(path):
    cur = None
    for line in open(path):
        if line.startswith("#"):
            cur = []
            yield_ = cur
            launches.acc.append(yield_)
            continue
        t, tag, blk, a, b = map(int, line.split())
        cur.append((t, tag, blk, a, b))
    return launches.acc


launches.acc = []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--launch", type=int, default=-1)
    ap.add_argument("--min", type=int, default=16384)
    ap.add_argument("--rows", type=int, default=0, help="only leaders/splits of jobs with this many rows (0: all)")
    args = ap.parse_args()
    L = launches(args.path)
    ev = sorted(L[args.launch])
    t0 = ev[0][0]
    us = lambda t: (t - t0) / 100.0
    rows_of = {}
    print(f"{len(L)} launches; launch {args.launch}: {len(ev)} events, {us(ev[-1][0]):.0f} us")
    print("-- leaders (us): start colw init uncl end")
    lead = collections.defaultdict(dict)
    for t, tag, blk, a, b in ev:
        if tag in LEAD:
            lead[blk][LEAD[tag]] = us(t)
            rows_of[blk] = a
    for blk in sorted(lead, key=lambda k: -rows_of[k]):
        if args.rows and rows_of[blk] != args.rows:
            continue
        d = lead[blk]
        print(f"  b{blk:<4} R{rows_of[blk]:<4}", " ".join(f"{k} {d.get(k, float('nan')):8.0f}" for k in LEAD.values()))
    print(f"-- splits of >= {args.min} columns: start, phase durations (us)")
    open_ = {}
    for t, tag, blk, a, b in ev:
        if tag == 10:
            open_[blk] = [us(t), a, b, {}]
        elif tag in SPLIT and blk in open_:
            st = open_[blk]
            last = st[0] + sum(st[3].values())
            st[3][SPLIT[tag]] = us(t) - last
            if tag == 16:
                s0, m, beg, ph = open_.pop(blk)
                if m >= args.min:
                    print(f"  b{blk:<4} m{m:<7} beg{beg:<7} start {s0:8.0f} end {s0 + sum(ph.values()):8.0f} |",
                          " ".join(f"{k} {v:6.0f}" for k, v in ph.items()))
    print("-- divided variance passes (owner): gather->parts->reduce (us)")
    sp = {}
    for t, tag, blk, a, b in ev:
        if tag == 20:
            sp[blk] = [us(t), a, b]
        elif tag == 21 and blk in sp:
            sp[blk].append(us(t))
        elif tag == 22 and blk in sp:
            s = sp.pop(blk)
            if s[1] >= args.min:
                print(f"  b{blk:<4} m{s[1]:<7} R{s[2]:<4} at {s[0]:8.0f} parts {s[3] - s[0]:7.0f} reduce {us(t) - s[3]:6.0f}")
    print("-- parts: count, mean / max duration (us) by kind and cluster size")
    ps = {}
    dur = collections.defaultdict(list)
    for t, tag, blk, a, b in ev:
        if tag == 30:
            ps[blk] = (us(t), a, b)
        elif tag == 31 and blk in ps:
            s0, kind, p = ps.pop(blk)
            if b >= args.min:
                dur[(KIND.get(kind, kind), b)].append(us(t) - s0)
    for (k, m), v in sorted(dur.items(), key=lambda x: (x[0][0], -x[0][1])):
        print(f"  {k:5} m{m:<7} n{len(v):<3} mean {sum(v) / len(v):7.0f} max {max(v):7.0f}")


if __name__ == "__main__":
    main()

"""Attribute the VALU instructions of the brute gather's VRL loop to source
lines (line tables from -gline-tables-only), to see where the issue budget
goes.  Usage: python tools/isa_lines.py [kernel-substring] [top-N]"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "mitsuba-alvrl_amd", "csrc", "gather.hip")


def main():
    kname = sys.argv[1] if len(sys.argv) > 1 else "k_gather_bruteILi2ELi2E"
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    out = "/tmp/isa_lines.s"
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-I" + os.path.join(ROOT, "include"),
                           "-fno-hip-fp32-correctly-rounded-divide-sqrt",
                           "-fgpu-flush-denormals-to-zero", "-gline-tables-only",
                           "--cuda-device-only", "-S", SRC, "-o", out],
                          stderr=subprocess.DEVNULL)
    s = open(out).read()
    files = {}
    for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s):
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
    sym = [n for n in re.findall(r"^(_Z\S+):", s, re.M) if kname in n][0]
    body = s[s.index(sym + ":"):]
    body = body[:body.index(".Lfunc_end")]
    lines = body.split("\n")
    # the VRL loop: from the loop header to the last backward branch into it
    head = next(i for i, l in enumerate(lines) if "Loop Header" in l)
    hlabel = lines[head].split(":")[0].strip()
    labels = {l.split(":")[0].strip(): i for i, l in enumerate(lines) if re.match(r"\s*\.LBB\S+:", l)}
    end = head
    for i, l in enumerate(lines):
        m = re.match(r"\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and labels.get(m.group(1), 1 << 30) <= head and i > end:
            end = i
    cur = None
    cnt, tr, sal = collections.Counter(), collections.Counter(), 0
    for l in lines[head:end + 1]:
        l = l.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        if not l or l.startswith((".", ";")):
            continue
        op = l.split()[0]
        if op.startswith("v_"):
            cnt[cur] += 1
            if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_", op):
                tr[cur] += 1
        elif op.startswith("s_"):
            sal += 1
    print(f"{sym}: loop {hlabel}, VALU {sum(cnt.values())} (trans {sum(tr.values())}), scalar {sal}")
    for (f, ln), n in sorted(cnt.items(), key=lambda x: -x[1])[:top]:
        src = ""
        if f == "vrl_device.hpp":
            src = open(os.path.join(ROOT, "mitsuba-alvrl_amd", "csrc", f)).read().split("\n")[ln - 1].strip()[:90]
        print(f"{n:4d} tr={tr[(f, ln)]:2d} {f}:{ln}  {src}")


if __name__ == "__main__":
    main()

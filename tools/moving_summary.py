#!/usr/bin/env python3
"""Summary table of tools/moving_ab.py's JSON lines: per (scene, lib, policy, slots, camera) the mean one-frame-at-
a-time rate, wall ms per frame and render-kernel ms over the reps."""
import collections
import json
import sys

rows = collections.defaultdict(list)
for line in open(sys.argv[1]):
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    rows[(d["scene"] + ":" + d.get("mode", ""), d["lib"], d["policy"], d["fif"], d["camera"])].append(d)
print(f"{'scene':13} {'library':22} {'policy':7} {'slots':5} {'camera':7} {'Mrays/s':>9} {'wall ms':>8} {'kernel ms':>9}  lpt")
for k in sorted(rows):
    v = rows[k]
    mr = sum(x["mrays_per_s_one_at_a_time"] for x in v) / len(v)
    wm = sum(x["frame_ms_wall"] for x in v) / len(v)
    km = sum(x["kernel_ms"] for x in v) / len(v)
    lpt = v[-1].get("lpt", "")
    print(f"{k[0]:13} {k[1]:22} {k[2]:7} {k[3]:5} {k[4]:7} {mr:9.1f} {wm:8.4f} {km:9.4f}  {lpt}")

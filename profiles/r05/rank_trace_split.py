#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of profiles/r05/rank_trace.py (3 kernels per frame: tile
pass, crawl pass, RGB8 pack) into its warm / pipelined / lone phases.
  python profiles/r05/rank_trace_split.py <kernel_trace.csv> [steps warm lone]"""
import csv
import sys

path = sys.argv[1]
steps, warm, lone = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (100, 20, 30)
rows = [r for r in csv.DictReader(open(path)) if any(k in r["Kernel_Name"] for k in ("march_kernel", "crawl_kernel", "pack_rgb8"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
per = 3
assert len(ev) == per * (warm + steps + lone), (len(ev), per * (warm + steps + lone))
pipe = ev[per * warm: per * (warm + steps)]
t0 = min(s for s, _, _ in pipe)
t1 = max(e for _, e, _ in pipe)
busy, cur_s, cur_e = 0, None, None
for s, e, _ in sorted(pipe):
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s


def short(n):
    return "march" if "march_kernel" in n else ("crawl" if "crawl_kernel" in n else ("pack" if "pack" in n else n[:30]))


print(f"pipelined: {steps} frames, span {(t1 - t0) / 1e3:.1f} us = {(t1 - t0) / steps / 1e3:.2f} us/frame, "
      f"GPU busy (union of kernels) {busy / (t1 - t0):.3f}")
for kind in ("march", "crawl", "pack"):
    d = [e - s for s, e, n in pipe if short(n) == kind]
    print(f"  {kind:5s}: mean dispatch {sum(d) / len(d) / 1e3:8.2f} us (overlapping)")
# what runs when: the pipelined span split by the set of kernel kinds active
pts = sorted([(s_, 1, short(n)) for s_, _, n in pipe] + [(e_, -1, short(n)) for _, e_, n in pipe])
act = {"march": 0, "crawl": 0, "pack": 0}
mix = {}
prev = pts[0][0]
for t, d, k in pts:
    state = "+".join(x for x in ("march", "crawl", "pack") if act[x]) or "idle"
    mix[state] = mix.get(state, 0) + (t - prev)
    prev = t
    act[k] += d
tot = sum(mix.values())
print("  active kinds over the span: " + ", ".join(f"{k} {v / tot:.3f}" for k, v in sorted(mix.items(), key=lambda kv: -kv[1])))
lo = ev[per * (warm + steps):]
tm, tc, tp, gaps = [], [], [], []
for i in range(0, len(lo), per):
    f = sorted(lo[i:i + per])
    d = {short(n): (s, e) for s, e, n in f}
    tm.append((d["march"][1] - d["march"][0]) / 1e3)
    tc.append((d["crawl"][1] - d["crawl"][0]) / 1e3)
    tp.append((d["pack"][1] - d["pack"][0]) / 1e3)
    gaps.append((f[-1][1] - f[0][0]) / 1e3)


def med(x):
    x = sorted(x)
    return x[len(x) // 2]


print(f"lone frames ({lone}): median tile pass {med(tm):.1f} us, crawl pass {med(tc):.1f} us, pack {med(tp):.1f} us, "
      f"first start -> last end {med(gaps):.1f} us")

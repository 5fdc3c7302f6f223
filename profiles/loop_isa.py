#!/usr/bin/env python3
"""Print the innermost loops that hold a global_load_dwordx2 in one kernel of
an ISA listing (hipcc -S / --save-temps), with VALU/SALU instruction counts.
  python profiles/loop_isa.py build/isa_vr_march-hip-amdgcn-amd-amdhsa-gfx950.s march_kernelILi0ELi1ELb0E [--print]"""
import re
import sys

path, kname = sys.argv[1], sys.argv[2]
show = "--print" in sys.argv
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + kname + r"\w*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
for i, l in enumerate(body):
    if "global_load_dwordx2" not in l:
        continue
    # innermost loop containing i: the closest back-edge branch after i to a label before i
    best = None
    for j in range(i, len(body)):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", body[j])
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] <= i:
                best = (labels[tgt], j)
                break
    if not best:
        continue
    a, b = best
    ins = [x.strip() for x in body[a:b + 1] if x.strip() and not x.strip().startswith((";", ".", "//"))]
    valu = [x for x in ins if x.startswith("v_")]
    salu = [x for x in ins if x.startswith("s_") and not x.startswith(("s_waitcnt", "s_nop"))]
    print(f"loop {body[a].split(':')[0]} (lines {start + a + 1}-{start + b + 1}): {len(ins)} instructions, "
          f"{len(valu)} VALU, {len(salu)} SALU/branch, {sum('global_load' in x for x in ins)} loads")
    if show:
        print("\n".join("   " + x for x in ins))

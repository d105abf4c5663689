#!/usr/bin/env python3
"""Instruction mix of each loop (label .. backward branch to it) of one kernel in a device .s file.
usage: scripts/isa_loops.py file.s mangled_kernel_name"""
import collections, re, sys
s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
lines = s[i:j].splitlines()
labels = {}
for k, ln in enumerate(lines):
    m = re.match(r"^(\.LBB\S+):", ln.strip())
    if m:
        labels[m.group(1)] = k
for k, ln in enumerate(lines):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", ln)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    if tgt in labels and labels[tgt] < k:
        body = lines[labels[tgt]:k + 1]
        c = collections.Counter()
        for b in body:
            t = b.strip().split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            c[t[0]] += 1
        g = collections.Counter()
        for op, v in c.items():
            key = ("fp64" if op.endswith(("_f64", "_f64_e32", "_f64_e64")) else "agpr" if "accvgpr" in op else
                   "dpp" if "dpp" in op else "v_mov" if op.startswith("v_mov") else "cndmask" if "cndmask" in op else
                   "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "salu" if op.startswith("s_") else "valu-other")
            g[key] += v
        print(f"loop {tgt} lines {labels[tgt]}-{k} total {sum(c.values())}: {dict(g)}")
        if sum(c.values()) > 300:
            for op, v in c.most_common(14):
                print(f"   {v:5d} {op}")

#!/usr/bin/env python3
"""Static instruction mix of one kernel in a device assembly file (hipcc --offload-device-only -S).
usage: scripts/isa_mix.py file.s mangled_kernel_name [top]"""
import collections, sys
s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
c = collections.Counter()
for ln in s[i:j].splitlines():
    t = ln.strip().split()
    if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
        continue
    c[t[0]] += 1
print("total", sum(c.values()))
groups = collections.Counter()
for k, v in c.items():
    g = ("fp64" if k.endswith(("_f64", "_f64_e32", "_f64_e64")) else "agpr" if "accvgpr" in k else
         "dpp" if "dpp" in k else "mov" if k.startswith("v_mov") else "cndmask" if "cndmask" in k else
         "vmem" if k.startswith(("global_", "buffer_", "flat_")) else "salu" if k.startswith("s_") else "valu-other")
    groups[g] += v
print(dict(groups))
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 25):
    print(f"{v:6d} {k}")

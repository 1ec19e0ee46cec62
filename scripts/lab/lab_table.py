"""Pivot a gemm_lab log: best (max) TF/s per (variant, shape) over the passes."""
import re
import sys
rows, order = {}, []
for l in open(sys.argv[1]):
    m = re.match(r'(.{18}) m=.*?k=\s*\d+\s+(.*?)\s+([\d.]+) ms\s+([\d.]+) TF/s', l)
    if not m:
        continue
    s, v, tf = m.group(1).strip(), m.group(2).strip(), float(m.group(4))
    d = rows.setdefault(v, {})
    d[s] = max(d.get(s, 0), tf)
    if s not in order:
        order.append(s)
print("%-40s" % "variant" + "".join("%11s" % o[:10] for o in order))
for v, d in rows.items():
    print("%-40s" % v + "".join("%11.1f" % d.get(o, 0) for o in order))

"""From a rocprofv3 kernel trace of bench.py: GPU kernel time inside the timed steps vs the wall time
of those steps (is the step GPU-bound or launch-bound?).  Usage: step_time_split.py trace.csv steps"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# the timed region: the last `steps` occurrences of the step's first kernel (the embedding forward)
starts = [s for s, e, n in ev if "embed_fwd" in n]
first_per_step = starts[::2]          # two embed_fwd launches per step (text, PV)
t0 = first_per_step[-steps]
t1 = ev[-1][1]
busy = 0
cur_s, cur_e = None, None
n = 0
for s, e, name in ev:
    if s < t0:
        continue
    n += 1
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
wall = t1 - t0
print("timed steps %d: wall %.2f ms/step, GPU busy %.2f ms/step (%.1f%%), %d kernels/step" % (
    steps, wall / 1e6 / steps, busy / 1e6 / steps, 100.0 * busy / wall, n // steps))

# per-kernel-family time inside the timed steps
import collections
import re
fam = collections.defaultdict(lambda: [0, 0])
for s, e, name in ev:
    if s < t0:
        continue
    key = name.replace("void ", "").replace("(anonymous namespace)::", "")
    key = re.sub(r"\(.*", "", key)[:90]
    fam[key][0] += e - s
    fam[key][1] += 1
tot = sum(v[0] for v in fam.values())
for k, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print("%-90s %5d/step %8.3f ms/step %5.1f%%" % (k, c // steps, t / 1e6 / steps, 100.0 * t / tot))

# the largest (kernel, grid) classes: which launches of a family cost most
if len(sys.argv) > 4:
    cls = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        s = int(r["Start_Timestamp"])
        if s < t0:
            continue
        key = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", ""))[:70]
        g = "%sx%sx%s/%s lds%s" % (r.get("Grid_Size_X", "?"), r.get("Grid_Size_Y", "?"), r.get("Grid_Size_Z", "?"),
                                  r.get("Workgroup_Size_X", "?"), r.get("LDS_Block_Size", r.get("Lds_Size", "?")))
        cls[(key, g)][0] += int(r["End_Timestamp"]) - s
        cls[(key, g)][1] += 1
    print("\ntop (kernel, grid) classes")
    for (k, g), (t, c) in sorted(cls.items(), key=lambda kv: -kv[1][0])[:int(sys.argv[4])]:
        print("%-70s %-28s %4d/step %7.3f ms/step  %7.1f us avg" % (k, g, c // steps, t / 1e6 / steps, t / 1e3 / c))

# optimizer time NOT hidden behind other kernels (the per-block AdamW runs on a side stream): the length of
# the union of adamw intervals minus its intersection with the union of every other kernel's intervals


def _union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _length(iv):
    return sum(e - s for s, e in iv)


def _intersect(a, b):
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


adam = _union([(s, e) for s, e, name in ev if s >= t0 and "adamw" in name])
other = _union([(s, e) for s, e, name in ev if s >= t0 and "adamw" not in name])
if adam:
    busy_adam = _length(adam)
    exposed = busy_adam - _length(_intersect(adam, other))
    print("\nAdamW: %.3f ms/step of kernel-union time, %.3f ms/step exposed (not overlapped by another kernel)" % (
        busy_adam / 1e6 / steps, exposed / 1e6 / steps))

"""Idle gaps of the GPU inside the timed steps of a rocprofv3 kernel trace (bench.py): every interval in which
no kernel runs, classified by the kernels on either side -- where the step's non-busy time goes (host waits,
stream synchronisation, launch boundaries).  Usage: step_gaps.py trace.csv steps [min_us] [top]"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))
    return n[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
top = int(sys.argv[4]) if len(sys.argv) > 4 else 25
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
starts = [s for s, e, n in ev if "embed_fwd" in n]
t0 = starts[::2][-steps]
ev = [x for x in ev if x[0] >= t0]
gaps = []
cur_e, cur_n = ev[0][1], ev[0][2]
for s, e, n in ev[1:]:
    if s > cur_e:
        gaps.append((s - cur_e, cur_n, n))
    if e > cur_e:
        cur_e, cur_n = e, n
tot = sum(g for g, _, _ in gaps)
hist = collections.Counter()
for g, _, _ in gaps:
    b = "<2us" if g < 2000 else "2-5us" if g < 5000 else "5-20us" if g < 20000 else "20-100us" if g < 100000 else ">100us"
    hist[b] += g
print("idle %.3f ms/step in %d gaps/step; by gap size (ms/step): %s" % (
    tot / 1e6 / steps, len(gaps) // steps,
    ", ".join("%s %.3f" % (k, hist[k] / 1e6 / steps) for k in ("<2us", "2-5us", "5-20us", "20-100us", ">100us"))))
pairs = collections.defaultdict(lambda: [0, 0])
for g, a, b in gaps:
    if g >= min_us * 1000:
        pairs[(short(a), short(b))][0] += g
        pairs[(short(a), short(b))][1] += 1
print("gaps >= %.1f us by (kernel before -> kernel after):" % min_us)
for (a, b), (t, c) in sorted(pairs.items(), key=lambda kv: -kv[1][0])[:top]:
    print("  %8.3f ms/step %4d/step  %s -> %s" % (t / 1e6 / steps, c // steps, a, b))

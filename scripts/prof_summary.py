"""Summarise a rocprofv3 --kernel-trace --stats CSV (per-step ms by kernel)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("%-100s %7s %10s %6s %10s" % ("kernel", "calls", "ms/step", "%", "avg_us"))
for r in rows[:40]:
    print("%-100s %7d %10.3f %5.1f%% %10.1f" % (r["Name"][:100], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6 / steps,
                                              100 * float(r["TotalDurationNs"]) / tot, float(r["AverageNs"]) / 1e3))
print("total kernel time per step: %.2f ms (%d kernel names)" % (tot / 1e6 / steps, len(rows)))

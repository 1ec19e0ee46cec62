"""Summarise lab PMC passes: per kernel name substring, mean counter value per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

tag, sub = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
for path in sorted(glob.glob("gpurun_out/pmc_%s_*/**/*counter_collection.csv" % tag, recursive=True)):
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print("%-28s %16.1f  (n=%d)" % (k, sum(v) / len(v), len(v)))

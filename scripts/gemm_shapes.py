"""Per-(kernel, grid) duration table from a rocprofv3 kernel trace: shows where GEMM time goes."""
import csv
import collections
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    if "gemm" not in name and "attn" not in name:
        continue
    key = (name.replace("void ", "").replace("(anonymous namespace)::", "").replace("k3m_x6::", "").split("(K3m")[0].split("(float")[0][:60], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]),
           int(r["Grid_Size_Y"]))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print("%-62s blocks=%5d y=%3d n=%4d avg=%8.1fus total=%8.1fms %4.1f%%" % (k[0], k[1], k[2], len(v), sum(v) / len(v), sum(v) / 1e3, 100 * sum(v) / tot))

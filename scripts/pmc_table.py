"""Counter table of one kernel from scripts/pmc_gemm.sh passes: mean per dispatch + derived rates.
usage: pmc_table.py <tag> <kernel-name substring> [flops_per_dispatch] [algorithmic_bytes] [M,N,K]
(bench.py reads traffic_bytes of the newest record whose shape and full kernel name match the kernel it runs)"""
import csv
import glob
import json
import sys
from collections import defaultdict

tag, sub = sys.argv[1], sys.argv[2]
flops = float(sys.argv[3]) if len(sys.argv) > 3 else None
alg_bytes = float(sys.argv[4]) if len(sys.argv) > 4 else None
shape = [int(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else None
vals = defaultdict(list)
names = set()
durs = []
for path in sorted(glob.glob("gpurun_out/pmc_%s_*/**/*counter_collection.csv" % tag, recursive=True)):
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            names.add(r["Kernel_Name"])
for path in sorted(glob.glob("gpurun_out/pmc_%s_*/**/*kernel_trace.csv" % tag, recursive=True)):
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
out = {"tag": tag, "kernel": sorted(names)[0] if len(names) == 1 else sub, "kernel_names": sorted(names),
       "shape": shape, "counters_mean_per_dispatch": m,
       "dispatches": {k: len(v) for k, v in vals.items()}}
if durs:
    # profiled dispatches only (clocks differ from un-profiled runs: MI355X_MICROARCH.md DVFS item 2)
    d = sorted(durs)[len(durs) // 2] * 1e-9
    out["median_dispatch_s"] = d
    if "GRBM_GUI_ACTIVE" in m:
        out["effective_clock_GHz"] = m["GRBM_GUI_ACTIVE"] / 8 / d / 1e9
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            # SQ_VALU_MFMA_BUSY_CYCLES summed over every SIMD of the chip (1024)
            out["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc)
    if flops:
        out["achieved_TFs_profiled"] = flops / d / 1e12
        out["mfma_cycles_expected_32x32x16"] = flops / 32768 * 32
if "SQ_WAVE_CYCLES" in m:
    w = m["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
              "SQ_WAIT_INST_LDS"):
        if k in m:
            out[k + "_frac_of_wave_cycles"] = m[k] / w
if "SQ_LDS_IDX_ACTIVE" in m and "SQ_LDS_BANK_CONFLICT" in m:
    out["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / max(1.0, m["SQ_LDS_IDX_ACTIVE"])
if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
    # FETCH_SIZE in KB, x2 on gfx950 for wide streaming reads; WRITE_SIZE in KB (MI355X_MICROARCH.md HBM)
    rd = 2 * m.get("FETCH_SIZE", 0) * 1024
    wr = m.get("WRITE_SIZE", 0) * 1024
    out["hbm_read_bytes"] = rd
    out["hbm_write_bytes"] = wr
    out["traffic_bytes"] = rd + wr
    if alg_bytes:
        out["traffic_over_algorithmic"] = (rd + wr) / alg_bytes
print(json.dumps(out, indent=1, sort_keys=True))

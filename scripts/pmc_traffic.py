"""Per-launch HBM traffic of one kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; each its
own run, MI355X_MICROARCH.md §HBM): FETCH_SIZE (kB) x 2 (gfx950 tallies 128-B read requests at 64 B)
+ WRITE_SIZE (kB), x 1024 bytes.  Writes the JSON bench.py reads as roofline.traffic.

    python scripts/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> M N K <epilogue> <out.json>
"""
import csv
import glob
import json
import sys


def per_launch(d, counter, substr):
    path = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and substr in r["Kernel_Name"]]
    names = {r["Kernel_Name"] for r in csv.DictReader(open(path)) if substr in r["Kernel_Name"]}
    assert vals, "no %s samples for %s in %s" % (counter, substr, path)
    return sum(vals) / len(vals), len(vals), sorted(names)[0]


def main():
    fdir, wdir, sub, M, N, K, epi, out = sys.argv[1:9]
    M, N, K = int(M), int(N), int(K)
    f, nf, name = per_launch(fdir, "FETCH_SIZE", sub)
    w, nw, _ = per_launch(wdir, "WRITE_SIZE", sub)
    rd, wr = 2.0 * f * 1024, w * 1024
    # algorithmic bytes: A + B read once, C (+ aux for BIAS_GELU) written once, fp32
    alg = 4 * (M * K + N * K + M * N * (2 if epi == "BIAS_GELU" else 1))
    d = {"kernel": name, "shape": [M, N, K], "epilogue": epi,
         "FETCH_SIZE_kB_per_launch": f, "FETCH_SIZE_launches": nf,
         "WRITE_SIZE_kB_per_launch": w, "WRITE_SIZE_launches": nw,
         "read_bytes_corrected": rd, "write_bytes": wr, "traffic_bytes": rd + wr, "algorithmic_bytes": alg,
         "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, --kernel-trace; "
                   "scripts/gemm_bench.py; FETCH_SIZE x2 per MI355X_MICROARCH.md gfx950 correction; kB x 1024",
         "source": "%s, %s (scripts/gpu_steps.sh pmc)" % (fdir, wdir)}
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(d, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()

"""Per-kernel ISA statistics of a hipcc -S device assembly file: scratch (spill) instructions in
total and inside basic blocks that also hold MFMAs (i.e. in the main loops), MFMA and VALU counts.
usage: python scripts/isa_stats.py file.s [name-regex]"""
import re
import sys


def main(path, pat="."):
    txt = open(path).read()
    parts = re.split(r"\n(_Z[^\s:]*):[^\n]*\n", txt)
    for i in range(1, len(parts), 2):
        name, body = parts[i], parts[i + 1].split(".Lfunc_end")[0]
        if not re.search(pat, name):
            continue
        blocks, cur = [], []
        for l in body.split("\n"):
            if re.match(r"^\.LBB", l):
                blocks.append(cur)
                cur = []
            cur.append(l)
        blocks.append(cur)
        sc = sum(1 for b in blocks for l in b if "scratch_" in l)
        insc = sum(sum(1 for l in b if "scratch_" in l) for b in blocks if any("v_mfma" in l for l in b))
        mf = sum(1 for b in blocks for l in b if "v_mfma" in l)
        short = re.sub(r"^_ZN.*?(gemm\w*?kernel)I", r"\1<", name)[:90]
        print("%-90s scratch %4d  in-mfma-blocks %4d  mfma %5d" % (short, sc, insc, mf))


if __name__ == "__main__":
    main(*sys.argv[1:])

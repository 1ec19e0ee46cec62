"""vmcnt waits, global stores and loads after the last MFMA of a kernel (its epilogue) in a hipcc -S
device assembly file.  usage: python scripts/epi_vmcnt.py file.s kernel-name-regex [...]"""
import re
import sys


def funcs(path):
    txt = open(path).read()
    parts = re.split(r"\n(_Z[^\s:]*):[^\n]*\n", "\n" + txt)
    for i in range(1, len(parts), 2):
        yield parts[i], parts[i + 1].split(".Lfunc_end")[0].split("\n")


def main(path, *pats):
    for name, body in funcs(path):
        if not any(re.search(p, name) for p in pats):
            continue
        mf = [n for n, l in enumerate(body) if "v_mfma" in l]
        if not mf:
            continue
        tail = body[mf[-1]:]
        w0 = sum(1 for l in tail if re.search(r"s_waitcnt vmcnt\(0\)", l))
        wn = sum(1 for l in tail if re.search(r"s_waitcnt vmcnt\([1-9]", l))
        st = sum(1 for l in tail if "global_store" in l)
        ld = sum(1 for l in tail if "global_load" in l and "lds" not in l)
        print("%-96s vmcnt(0) %3d  vmcnt(N>0) %3d  stores %4d  loads %3d" % (name[:96], w0, wn, st, ld))


if __name__ == "__main__":
    main(*sys.argv[1:])

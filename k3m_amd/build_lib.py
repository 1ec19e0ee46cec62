"""Build libk3m_hip.so (gfx950) in-tree with hipcc — no torch headers, C ABI only."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libk3m_hip.so")
SOURCES = ["gemm.hip", "gemm_x6p.hip", "gemm_bf16.hip", "norm.hip", "attention.hip", "attention_bf16.hip", "loss.hip", "fusion.hip", "struct.hip", "adamw.hip", "data.hip", "align.hip", "attention_long.hip", "attention_flash_long.hip"]
# -fno-slp-vectorize: no packed-f32 (v_pk_*_f32) code from paired scalar math.  Beside MFMAs packed f32
# VALU costs more than the scalar pair (MI355X_MICROARCH.md cycle constants), and in the GEMM epilogues
# the packed alpha/beta form  v_pk_fma_f32 s[alpha:beta], op_sel  dropped the beta*C term for
# scattered lane groups (scripts/debug/dgrad_beta.py: C = alpha*AB on ~1e-5 of the elements).
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-mcode-object-version=5", "-Wno-unused-result",
         "-fno-slp-vectorize"]


def hipcc():
    for p in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if p and os.path.exists(p):
            return p
    return "hipcc"


def build(force=False, jobs=8, verbose=False):
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    deps = [os.path.join(CSRC, "common.h"), os.path.join(CSRC, "gemm_f32_tile.h"), os.path.join(CSRC, "gemm_x6_tile.h"), os.path.join(CSRC, "gemm_b16_tile.h"), os.path.join(CSRC, "flash_frag.h"), os.path.join(os.path.dirname(HERE), "include", "k3m_hip.h")]
    dep_m = max(os.path.getmtime(d) for d in deps)

    # headers only one translation unit includes
    own = {"gemm_bf16.hip": [os.path.join(CSRC, "gemm_b16_ws.h")]}

    def one(src):
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, src + ".o")
        dm = max([dep_m] + [os.path.getmtime(d) for d in own.get(src, [])])
        if not force and os.path.exists(o) and os.path.getmtime(o) >= max(os.path.getmtime(s), dm):
            return o
        cmd = [hipcc()] + FLAGS + ["-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed for %s:\n%s" % (src, r.stderr[-4000:]))
        if verbose:
            print("built", src, file=sys.stderr)
        return o

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(one, srcs))
    if force or not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(o) for o in objs):
        cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s" % r.stderr[-4000:])
    return OUT


DATA_SRC = os.path.join(HERE, "host", "preprocess.cpp")
DATA_OUT = os.path.join(HERE, "libk3m_data.so")
# -ffp-contract=off: every fp32 expression rounds as the numpy array expression it restates
DATA_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall"]


def build_data(force=False):
    """Build the host data-path library libk3m_data.so (plain g++, no GPU code)."""
    hdr = os.path.join(os.path.dirname(HERE), "include", "k3m_data.h")
    if not force and os.path.exists(DATA_OUT) and os.path.getmtime(DATA_OUT) >= max(
            os.path.getmtime(DATA_SRC), os.path.getmtime(hdr)):
        return DATA_OUT
    r = subprocess.run(["g++"] + DATA_FLAGS + [DATA_SRC, "-o", DATA_OUT], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("g++ failed for %s:\n%s" % (DATA_SRC, r.stderr[-4000:]))
    return DATA_OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_data(force="--force" in sys.argv))

"""ctypes binding of libk3m_hip.so (the C ABI declared in include/k3m_hip.h).

The library is loaded AFTER ``import torch`` so it binds to the HIP runtime torch already loaded
(same SONAME libamdhip64.so.7): device pointers and streams are shared with torch's allocator and
stream pool.  There is no fallback: if the library is missing or a call fails, a RuntimeError is
raised — the product path never silently runs something else.
"""
import ctypes as C
import os

import torch  # noqa: F401  (loads the HIP runtime first)

from . import debug as _debug

_HERE = os.path.dirname(os.path.abspath(__file__))
# K3M_LIB: another build of the same library (same-box A/B of two builds, scripts/ab_lib.sh)
LIB_PATH = os.environ.get("K3M_LIB") or os.path.join(_HERE, "libk3m_hip.so")

F32, BF16 = 0, 1
EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_DGELU, EPI_BIAS_SIGMOID = 0, 1, 2, 3, 4
GEMM_SLABS_ONLY = 0x100   # K3M_GEMM_SLABS_ONLY: split-K slabs left for k3m_slab_reduce_batch
GEMM_COLSUM_SLABS = 0x200   # K3M_GEMM_COLSUM_SLABS: dGELU output column sums as 32-row slabs in ws
F32_SPLIT_BF16X6, F32_MFMA_F32 = 0, 1
ADAM_ZERO_GRAD, ADAM_APEX, ADAM_APEX_BIAS_CORRECTION = 1, 2, 4
GRAPH_SEED = 1 << 63   # K3M_GRAPH_SEED | address: the kernels read the seed from that device word

vp, i32, i64, f32, u64 = C.c_void_p, C.c_int, C.c_longlong, C.c_float, C.c_uint64


class K3mGemm(C.Structure):
    _fields_ = [("m", i32), ("n", i32), ("k", i32), ("a_trans", i32), ("b_trans", i32), ("epilogue", i32),
                ("dtype", i32), ("splitk", i32), ("c_dtype", i32), ("lda", i64), ("ldb", i64), ("ldc", i64), ("ldaux", i64),
                ("a", vp), ("b", vp), ("c", vp), ("bias", vp), ("aux", vp), ("ws", vp), ("alpha", f32),
                ("beta", f32), ("f32_algo", i32), ("a_planes", i64), ("b_planes", i64)]


# name -> argtypes (restype is always int status)
SIGNATURES = {
    "k3m_gemm": [C.POINTER(K3mGemm), vp],
    "k3m_colsum": [vp, i64, i32, i32, vp, i32, vp, i32, vp],
    "k3m_ln_fwd": [vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, f32, u64, u64, u64, i32, vp],
    "k3m_ln_bwd": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, u64, u64, u64, i32, vp, i32, vp],
    "k3m_ln_bwd_nslab": [i32, vp],
    "k3m_ln_bwd_slabs": [vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, u64, u64, u64, i32, i32, vp, i32, vp],
    "k3m_colsum_nslab": [i32, vp],
    "k3m_colsum_slabs": [vp, i64, i32, i32, vp, i32, vp],
    "k3m_slab_reduce_batch": [vp, vp, vp, vp, vp, i32, vp],
    "k3m_embed_fwd": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, f32, u64, u64, i32, vp],
    "k3m_embed_bwd": [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp],
    "k3m_attn_fwd": [vp, i64, vp, i64, vp, i64, vp, vp, i64, vp, i32, i32, i32, i32, i32, f32, f32, u64, u64, i32, vp],
    "k3m_attn_bwd": [vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, vp, vp, vp, i64, i64, i64, i32, i32, i32, i32,
                     i32, f32, f32, u64, u64, i32, vp],
    "k3m_flash_attn_fwd": [vp, i64, vp, i64, vp, i64, vp, vp, i64, vp, i32, i32, i32, i32, i32, f32, f32, u64, u64,
                           vp],
    "k3m_flash_attn_bwd": [vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, vp, vp, vp, vp, i64, i64, i64, i32, i32,
                           i32, i32, i32, f32, f32, u64, u64, vp],
    "k3m_flash_attn_long_fwd": [vp, i64, vp, i64, vp, i64, vp, vp, i64, vp, i32, i32, i32, i32, i32, f32, f32, u64,
                                u64, vp],
    "k3m_flash_attn_long_ws_bytes": [i32, i32, i32, i32, i32, vp],
    "k3m_flash_attn_long_bwd": [vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, vp, vp, vp, vp, i64, i64, i64, vp, i64,
                                i32, i32, i32, i32, i32, f32, f32, u64, u64, vp],
    "k3m_dgelu": [vp, vp, vp, i64, i32, vp],
    "k3m_gather_rows": [vp, i64, vp, i32, i32, vp, i64, i32, vp],
    "k3m_scatter_add_rows": [vp, i64, vp, i32, i32, vp, i64, i32, vp],
    "k3m_compact_labels_ex": [vp, i32, i64, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp],
    "k3m_ce_fwd_bwd": [vp, i64, vp, vp, i32, i32, vp, vp],
    "k3m_kl_fwd_bwd": [vp, i64, vp, i64, vp, vp, i32, i32, vp, vp],
    "k3m_loss_reduce": [vp, vp, vp, i32, vp, vp],
    "k3m_scale_rows_by_slot": [vp, i64, vp, i32, i32, f32, f32, vp],
    "k3m_nsp_loss": [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, vp],
    "k3m_relu_cat3": [vp, vp, vp, vp, i32, i32, i32, vp],
    "k3m_gate_fwd": [vp, vp, vp, vp, vp, vp, i32, i32, u64, u64, i32, vp],
    "k3m_gate_bwd": [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp],
    "k3m_relu_split3_bwd": [vp, vp, vp, vp, vp, i32, i32, i32, i32, vp],
    "k3m_mean3": [vp, vp, vp, vp, i64, i32, vp],
    "k3m_mean3_bwd": [vp, vp, vp, vp, i64, i32, i32, vp],
    "k3m_seq_mean": [vp, i32, i32, i32, i32, f32, vp, i32, i32, vp],
    "k3m_seq_mean_bwd": [vp, i32, i32, i32, i32, f32, vp, i32, vp],
    "k3m_sa_gather": [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
    "k3m_sa_attn_fwd": [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp],
    "k3m_sa_attn_bwd": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp],
    "k3m_lpm_fwd": [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, f32, vp, vp, vp],
    "k3m_lpm_bwd": [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, f32, vp, vp, vp, vp],
    "k3m_lpm_sample": [vp, i32, i32, i32, i32, u64, u64, vp, vp, vp],
    "k3m_sa_gather_bwd": [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
    "k3m_embed_bwd_det": [vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, i32, vp],
    "k3m_sa_attn_bwd_det": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp],
    "k3m_lpm_bwd_det": [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp],
    "k3m_sa_gather_bwd_det": [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
    "k3m_adamw": [vp, vp, vp, vp, vp, i64, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, i32, f32, vp],
    "k3m_adamw_ex": [vp, vp, vp, vp, vp, i64, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, i32, f32,
                     i32, vp],
    "k3m_adamw_ex_dev": [vp, vp, vp, vp, vp, i64, vp, C.c_double, C.c_double, C.c_double, f32, i32, vp],
    "k3m_adamw_scalars_n": [i32, vp, vp, C.c_double, C.c_double, i32, i32, vp],
    "k3m_cast_f32_bf16": [vp, vp, i64, vp],
    "k3m_convert": [vp, i32, vp, i32, i64, i32, f32, vp],
    "k3m_add_inplace": [vp, vp, i64, f32, i32, vp],
    "k3m_gemm_grouped": [vp, i32, vp],
    "k3m_collate_regions": [vp, i64, vp, vp, vp, i32, i32, i32, vp, vp],
    "k3m_attn_long_fwd": [vp, i64, vp, i64, vp, i64, vp, vp, i64, vp, i32, i32, i32, i32, i32, f32, f32, u64, u64, i32,
                          vp],
    "k3m_attn_long_bwd": [vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, vp, vp, vp, vp, i64, i64, i64, i32, i32, i32,
                          i32, i32, f32, f32, u64, u64, i32, vp],
    "k3m_adamw_torch": [vp, vp, vp, vp, vp, i64, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, i32, f32,
                        vp],
    "k3m_align_pair_cat": [vp, i32, i32, f32, u64, u64, vp, vp],
    "k3m_align_pair_cat_bwd": [vp, i32, i32, f32, u64, u64, vp, vp],
    "k3m_align_ce_fwd_bwd": [vp, vp, vp, vp, i32, i32, f32, u64, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "k3m_align_cosine_fwd_bwd": [vp, vp, i32, i32, f32, vp, vp, vp, vp, vp],
}

_lib = None


def load(path=LIB_PATH):
    """Load (once) and type the library; raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError("libk3m_hip.so not found at %s — build it with `python -m k3m_amd.build_lib` "
                           "(or __graft_entry__.build()); there is no CPU fallback" % path)
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_int
    _lib = lib
    return lib


def exported_symbols(path=LIB_PATH):
    lib = C.CDLL(path)
    return [n for n in SIGNATURES if hasattr(lib, n)]


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


try:   # the raw current-stream handle without building a torch.cuda.Stream (1,400 launches per step)
    _raw_stream = torch._C._cuda_getCurrentRawStream
    _cur_dev = torch._C._cuda_getDevice
except AttributeError:   # pragma: no cover - older torch
    _raw_stream = None


def stream():
    """hipStream_t (as int) of the current stream of the current device."""
    if _raw_stream is not None:
        return _raw_stream(_cur_dev())
    return torch.cuda.current_stream().cuda_stream


_fns = {}


def call(name, *args):
    fn = _fns.get(name)
    if fn is None:
        fn = _fns[name] = getattr(load(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError("%s failed with status %d (%s)" % (name, rc, "bad argument" if rc == 1 else "hip error %d" % -rc))
    if _debug.ON:
        _debug.sync(name)

"""Tensor-level wrappers over the C ABI (k3m_amd/_lib.py).  Every function launches libk3m_hip
kernels on torch's current stream; torch is used only to allocate outputs/workspaces."""
import ctypes as C
import os

import torch

from . import _lib as L
from . import debug as _debug
from ._lib import call, ptr, stream

_DT = {torch.float32: L.F32, torch.bfloat16: L.BF16}


def dt(t):
    return _DT[t.dtype]


def _ld(t):
    assert t.dim() == 2 and t.stride(1) == 1, "row-major 2-D view expected"
    return t.stride(0)


def empty(shape, like=None, dtype=torch.float32, device=None):
    return torch.empty(shape, dtype=dtype, device=device if device is not None else like.device)


# ------------------------------------------------------------------ GEMM
# fp32-operand GEMM algorithm (include/k3m_hip.h K3mF32Algo): the bf16x6 split on the bf16 matrix
# cores by default; K3M_F32_ALGO=mfma selects the exact-f32 v_mfma_f32_32x32x2_f32 kernels.
F32_ALGO = {"x6": L.F32_SPLIT_BF16X6, "mfma": L.F32_MFMA_F32}[os.environ.get("K3M_F32_ALGO", "x6")]


class _Grouper(object):
    """Collects the GEMMs issued inside ``with grouped():`` and launches them on exit, one
    k3m_gemm_grouped per kernel template (layout, epilogue, dtypes).  The GEMMs of one group must
    be independent: nothing issued inside the block may read a GEMM output of the same block."""

    def __init__(self):
        self.pending = []
        self.after = []   # non-GEMM work that must wait for the block's side-stream branches
        self.post = []    # work that reads a GEMM output of the block: runs after the launches

    def flush(self):
        after, self.after = self.after, []
        for fn in after:
            fn()
        groups = {}
        for g, keep in self.pending:
            key = (g.a_trans, g.b_trans, g.epilogue, g.dtype, g.c_dtype, g.f32_algo)
            groups.setdefault(key, []).append((g, keep))
        self.pending = []
        for key, items in groups.items():
            if key[0] == 1 and not GROUP_WGRAD:   # weight gradients: each keeps its own split-K sizing
                for g, _ in items:
                    call("k3m_gemm", L.C.byref(g), stream())
                continue
            for i in range(0, len(items), GROUP_MAX):
                chunk = items[i:i + GROUP_MAX]
                arr = (L.K3mGemm * len(chunk))(*[g for g, _ in chunk])
                call("k3m_gemm_grouped", L.C.cast(arr, L.C.c_void_p), len(chunk), stream())
        post, self.post = self.post, []
        for fn in post:
            fn()


GROUP_MAX = 8
GROUP_WGRAD = os.environ.get("K3M_GROUP_WGRAD", "1") != "0"
_grouper = None


class grouped(object):
    """Context manager: defer and group the GEMMs issued inside (see _Grouper)."""

    def __enter__(self):
        global _grouper
        assert _grouper is None, "grouped() does not nest"
        _grouper = _Grouper()
        return _grouper

    def __exit__(self, *exc):
        global _grouper
        g, _grouper = _grouper, None
        if exc[0] is None:
            g.flush()
        return False


class branches(object):
    """Context manager for independent launches on side streams: ``branch(fn, ...)`` inside runs fn
    with a pool stream current (waiting first on everything the main stream issued before the
    region); on exit the main stream waits for every branch.  Small launches that each leave most
    CUs idle (one workgroup per (sequence, head) of a short attention) then overlap."""

    _pool = {}

    def __enter__(self):
        global _branches
        self.main = torch.cuda.current_stream()
        dev = self.main.device
        if dev not in branches._pool:
            branches._pool[dev] = [torch.cuda.Stream(device=dev) for _ in range(max(1, BRANCH_STREAMS))]
        self.streams = branches._pool[dev]
        self.ev = torch.cuda.Event()
        self.ev.record(self.main)
        self.n = 0
        self.waited = []
        self.prev, _branches = _branches, self
        return self

    def __exit__(self, *exc):
        global _branches
        _branches = self.prev
        for s in self.waited:
            self.main.wait_stream(s)
        return False

    def run(self, fn, *args, **kw):
        s = self.streams[self.n % len(self.streams)]
        self.n += 1
        if s not in self.waited:
            s.wait_event(self.ev)
            self.waited.append(s)
        with torch.cuda.stream(s):
            return fn(*args, **kw)


# off by default: overlapping the short attention launches on side streams measured 3.7 % SLOWER
# (423 vs 439 samples/s, same box) — kept selectable for other shapes (K3M_BRANCH_STREAMS=4)
BRANCH_STREAMS = int(os.environ.get("K3M_BRANCH_STREAMS", "1"))
_branches = None


def branch(fn, *args, **kw):
    """fn(*args) on a side stream inside ``with branches()``, inline otherwise."""
    if _branches is None or BRANCH_STREAMS <= 1:
        return fn(*args, **kw)
    return _branches.run(fn, *args, **kw)


def gemm(a, a_trans, b, b_trans, c, m, n, k, epi=L.EPI_NONE, bias=None, aux=None, alpha=1.0, beta=0.0, splitk=1,
         ws=None, f32_algo=None):
    g = L.K3mGemm()
    g.f32_algo = F32_ALGO if f32_algo is None else f32_algo
    g.m, g.n, g.k = m, n, k
    g.a_trans, g.b_trans = a_trans, b_trans
    assert a.dtype == b.dtype, "A and B must share a dtype"
    assert aux is None or aux.dtype == c.dtype, "aux has the dtype of C"
    g.epilogue, g.dtype, g.splitk, g.c_dtype = epi, dt(a), splitk, dt(c)
    g.lda, g.ldb, g.ldc = _ld(a), _ld(b), _ld(c)
    g.ldaux = _ld(aux) if aux is not None else 0
    g.a, g.b, g.c = ptr(a), ptr(b), ptr(c)
    g.bias, g.aux, g.ws = ptr(bias), ptr(aux), ptr(ws)
    if (splitk <= 1 and ws is None and _grouper is None and a.dtype == torch.float32 and c.dtype == torch.float32
            and g.f32_algo == L.F32_SPLIT_BF16X6):
        s = small_splitk(m, n, k)
        if s > 1:   # a small fp32 product split over k; the epilogue runs in the split-K reduction
            splitk, ws = s, torch.empty((s * m * n,), dtype=torch.float32, device=c.device)
            g.splitk, g.ws = s, ptr(ws)
    g.alpha, g.beta = alpha, beta
    if _grouper is not None:
        _grouper.pending.append((g, (a, b, c, bias, aux, ws)))   # keep the tensors alive until the flush
        return c
    call("k3m_gemm", L.C.byref(g), stream())
    return c


def linear(x, W, b=None, out=None, epi=None, aux=None, alpha=1.0, beta=0.0, out_dtype=None):
    """out = x . W^T (+ b) with epilogue; x [M,K] (row view), W [N,K]."""
    M, K = x.shape
    N = W.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype or x.dtype, device=x.device)
    if epi is None:
        epi = L.EPI_BIAS if b is not None else L.EPI_NONE
    return gemm(x, 0, W, 1, out, M, N, K, epi, b, aux, alpha, beta)


def dgrad_colsum_ok(dy, beta=0.0):
    """Whether an input gradient with the dGELU epilogue can leave its bias-gradient column sums as deferred
    slabs (K3M_GEMM_COLSUM_SLABS) instead of a separate k3m_colsum pass over its output."""
    return DGRAD_COLSUM and DEFER and _deferred is not None and beta == 0.0 and _deferred.active_here()


DGRAD_COLSUM = os.environ.get("K3M_DGRAD_COLSUM", "1") != "0"   # A/B knob


def linear_dgrad(dy, W, dx=None, beta=0.0, dgelu_aux=None, alpha=1.0, colsum_out=None):
    """dx (+)= dy . W (optionally * gelu'(aux)); dy [M,N], W [N,K].  A plain input gradient whose output
    fills few tiles but whose reduction is long (the tied MLM decoder: 1,536 labelled rows x 768 over the
    21,128-word vocabulary) is split over K like a weight gradient (fp32 slabs reduced with alpha/beta)."""
    M, N = dy.shape
    K = W.shape[1]
    if dx is None:
        dx = torch.empty((M, K), dtype=dy.dtype, device=dy.device)
    epi = L.EPI_DGELU if dgelu_aux is not None else L.EPI_NONE
    # (no K split when the column sums of dx are wanted: the split-K path leaves no place for them)
    s = _splitk(M, K, N, dy.dtype) if (epi == L.EPI_NONE and dx.dtype == torch.float32 and N >= 8192
                                       and colsum_out is None) else 1
    if s > 1:
        ws = torch.empty((s * M * K,), dtype=torch.float32, device=dy.device)
        return gemm(dy, 0, W, 0, dx, M, K, N, epi, None, None, alpha, beta, s, ws)
    if colsum_out is not None:
        # colsum_out += column sums of dx (the bias gradient of the Linear dx feeds): from the epilogue as
        # 32-row slabs joining the deferred reduction, or by a separate pass when that is not possible
        if epi == L.EPI_DGELU and dgrad_colsum_ok(dy, beta):
            ns = (M + 31) // 32
            ws = torch.empty((ns * K,), dtype=torch.float32, device=dy.device)
            _deferred.keep.append(ws)
            _deferred.add(ptr(ws), colsum_out, ns, K)
            return gemm(dy, 0, W, 0, dx, M, K, N, epi | L.GEMM_COLSUM_SLABS, None, dgelu_aux, alpha, beta, 1, ws)
        gemm(dy, 0, W, 0, dx, M, K, N, epi, None, dgelu_aux, alpha, beta)
        if _grouper is not None:   # the GEMM is still pending: sum its output after the group's launches
            _grouper.post.append(lambda: colsum(dx, colsum_out, accumulate=True))
        else:
            colsum(dx, colsum_out, accumulate=True)
        return dx
    return gemm(dy, 0, W, 0, dx, M, K, N, epi, None, dgelu_aux, alpha, beta)


# relative cost per extra split-K slice (its slab write + read), fp32 / bf16 weight gradients (A/B knobs)
SPLITK_COST_F32 = float(os.environ.get("K3M_SPLITK_COST_F32", "0.01"))
SPLITK_COST_BF16 = float(os.environ.get("K3M_SPLITK_COST_BF16", "0.02"))
# fewest k rows per split-K slice of an fp32 weight gradient (A/B knob)
SPLITK_MINK_F32 = int(os.environ.get("K3M_SPLITK_MINK_F32", "1024"))


# Under-filled fp32 weight gradients (K3M_SPLITK_FILL, A/B knob): an ungrouped split-K GEMM whose split under
# the default minimum k per slice leaves half of the 256 CUs idle or more (the image-stream 1,024 x 1,024 x 4,736
# projections: 128 work units) may use slices of half that depth, none of them empty.  Grouped GEMMs share one
# grid with the group's others and keep the default (a global minimum of 512 cost 0.6 % of the fp32 step,
# profiles/r4b_ab_mink.txt).  bf16 (a slice's MFMA time ~1/6 of the x6 one, so the extra slabs' traffic
# weighs more): _bf16_fill_split's time model, for splits leaving half of the CUs idle or more.
SPLITK_FILL = os.environ.get("K3M_SPLITK_FILL", "1") != "0"


def _split_cost_min(tiles, k, kmin, cost_per, bk, smax=32, nonempty=False):
    best, best_cost = 1, float("inf")
    for s in range(1, min(smax, k // kmin) + 1):
        if nonempty and s > 1:
            kt = (k + bk - 1) // bk
            per = (kt + s - 1) // s
            if per * (s - 1) >= kt:   # the last slice would be empty
                continue
        cost = ((tiles * s + 255) // 256) / s * (1.0 + cost_per * s)
        if cost < best_cost - 1e-9:
            best, best_cost = s, cost
    return best, best_cost


B16_MIN256 = int(os.environ.get("K3M_B16_256", "128"))   # gemm_bf16.hip big_prefers_256 (same env knob)


def _bf16_fill_split(m, n, k, s0):
    """An ungrouped bf16 weight gradient whose default split leaves half of the CUs idle or more (the image-stream
    1,024 x 1,024 x 4,736 projections: 128 units of 256 x 128): the split minimising a time model of waves x
    tile MFMA time (at 20 % of the per-CU peak: the split-4 launch measured 61 us, profiles/r4b_gemm_calls_cfg3.txt,
    for 52 in this model) + the slabs' HBM write and read (5 TB/s), with the tile the
    library will pick (256 x 128 below B16_MIN256 units of 256 x 256), no empty slice, >= 4 k-tiles per slice.
    Kept only if the model gains 20 %."""
    kt = (k + 63) // 64

    def model(s):
        t256 = ((m + 255) // 256) * ((n + 255) // 256)
        nb256 = t256 * s
        tbn = 256 if nb256 >= B16_MIN256 else 128
        units = ((m + 255) // 256) * ((n + tbn - 1) // tbn) * s
        per = (kt + s - 1) // s * 64
        mfma = 256.0 * tbn * per * 2 / (2.5e15 / 256 * 0.2)
        slab = (s * m * n * 8.0) / 5e12 if s > 1 else 0.0
        return (units + 255) // 256 * mfma + slab

    best, best_t = s0, model(s0)
    for s in range(2, min(32, kt // 4) + 1):
        per = (kt + s - 1) // s
        if per * (s - 1) >= kt:
            continue
        t = model(s)
        if t < best_t:
            best, best_t = s, t
    return best if best_t < 0.8 * model(s0) else s0


SMALL_SPLITK = os.environ.get("K3M_SMALL_SPLITK", "1") != "0"   # A/B knob


def small_splitk(m, n, k):
    """k-split of a small fp32 product (few 64 x 64 tiles, long k: the m = 64 pooled / gate projections, the
    389-row region-head GEMMs): one workgroup per (tile, k-slice) instead of one per tile walking all of k, the
    requested epilogue applied by the split-K reduction.  1 = no split."""
    if not SMALL_SPLITK or m <= 0 or n <= 0 or k <= 0:   # empty products (e.g. a batch with no labelled rows)
        return 1
    if n <= 8:
        # the skinny kernel (gemm.hip gemm_skinny_kernel, 64 rows per workgroup): k-slices of >= 128 until the
        # row blocks x slices fill 256 workgroups (loc wgrad 1,024 x 5 x 2,368: 16 x 16)
        if k < 256:
            return 1
        return max(1, min(k // 128, max(1, 256 // ((m + 63) // 64)), 64))
    tiles = ((m + 63) // 64) * ((n + 63) // 64)
    # >= 64 tiles at k = 1,024 (the 389-row region heads) measured slower split (0.030 -> 0.040 ms)
    if tiles >= 128 or k < 512 or (tiles >= 64 and k < 1536):
        return 1
    # few tiles: slices of >= 64 k (4 k-steps of the 64 x 64 tile: a tiny product is a chain of dependent loads, so
    # fewer steps per workgroup is what makes it faster); more tiles: >= 256 k per slice
    s = min(k // 256 if tiles >= 64 else k // 64, max(2, 384 // tiles), 32)
    if ((m + 255) // 256) * ((n + 127) // 128) * s >= 256:
        return 1
    return max(1, s)


def _splitk(m, n, k, dtype=torch.float32, grouped=False):
    """K-split of a weight-gradient GEMM (C[m,n] summed over k ~ 20k rows): enough blocks to fill
    the 256 CUs in whole waves.  fp32 (bf16x6 kernel) tiles are 256x128 at one block per CU;
    bf16 tiles are 256x256 at one block per CU."""
    if dtype == torch.float32 and (n <= 8 or m <= 8):
        # n <= 8: the skinny kernel; m <= 8 (a one-output Linear such as struc_w2): the 64 x 64 tiles.  Both are
        # split over k by small_splitk inside gemm(), not here (a 256-row x6 tile would be >= 97 % padding)
        return 1
    if dtype == torch.float32 and F32_ALGO == L.F32_SPLIT_BF16X6:
        tiles = ((m + 255) // 256) * ((n + 127) // 128)
        if tiles >= 200 or k < 2048:
            return 1
        # minimise (waves of 256 blocks) x (k per split), plus ~1% per split for the slab reduction
        best, cost = _split_cost_min(tiles, k, SPLITK_MINK_F32, SPLITK_COST_F32, 32)
        if SPLITK_FILL and not grouped and tiles * best <= 128:
            s2, c2 = _split_cost_min(tiles, k, SPLITK_MINK_F32 // 2, SPLITK_COST_F32, 32, nonempty=True)
            if c2 < cost - 1e-9:
                best = s2
        return best
    if dtype == torch.bfloat16 and k % 64 == 0 and m % 8 == 0 and n % 8 == 0:
        # the large-tile bf16 kernel (gemm_b16_tile.h): 256x256 blocks, one per CU; >= 16 k-tiles per split
        tiles = ((m + 255) // 256) * ((n + 255) // 256)
        if tiles >= 192 or k < 2048:
            return 1
        best = _split_cost_min(tiles, k, 1024, SPLITK_COST_BF16, 64)[0]
        if SPLITK_FILL and not grouped and tiles * best <= 64:   # 256 x 256 tiles; <= 128 units of 256 x 128
            best = _bf16_fill_split(m, n, k, best)
        return best
    tiles = ((m + 127) // 128) * ((n + 127) // 128)
    if tiles >= 384 or k < 1024:
        return 1
    s = min(max(1, 768 // tiles), k // 512, 32)
    return max(1, s)


def linear_wgrad(dy, x, gW, gb=None, alpha=1.0):
    """gW += alpha * dy^T . x ; gb += alpha * colsum(dy) (gb None: the bias gradient was fused into
    dy's producer).  dy [M,N], x [M,K], gW [N,K] fp32."""
    M, N = dy.shape
    K = x.shape[1]
    s = _splitk(N, K, M, dy.dtype, grouped=_grouper is not None)
    ws = torch.empty((s * N * K,), dtype=torch.float32, device=dy.device) if s > 1 else None
    epi = L.EPI_NONE
    if s > 1 and DEFER and _deferred is not None and alpha == 1.0 and gW.is_contiguous() and _deferred.active_here():
        # split-K slabs reduced with the block's other slab jobs (K3M_GEMM_SLABS_ONLY): gW += sum of slabs
        epi |= L.GEMM_SLABS_ONLY
        _deferred.keep.append(ws)
        _deferred.add(ptr(ws), gW, s, N * K)
    gemm(dy, 1, x, 0, gW, N, K, M, epi, None, None, alpha, 1.0, s, ws)
    if gb is not None:
        if _grouper is not None:   # dy may come from a side-stream branch of the same grouped block
            _grouper.after.append(lambda: colsum(dy, gb, accumulate=True, alpha=alpha))
        else:
            colsum(dy, gb, accumulate=True, alpha=alpha)


# ------------------------------------------------------------------ deferred slab reductions
# The LayerNorm backward and the bias-gradient column sums leave fp32 slabs of column partials; inside
# deferred_reductions() those slabs are summed by ONE k3m_slab_reduce_batch launch per flush (the engine
# flushes each encoder block before handing it to the all-reduce) instead of one small reduction launch
# after every producer (~230 per step).  Workspaces stay referenced until their flush.
_deferred = None


class _Deferred(object):
    def __init__(self):
        self.jobs = []      # (ws pointer, out pointer, nslab, cols, accumulate)
        self.keep = []      # workspaces referenced until the flush
        self.stream = stream() if torch.cuda.is_available() else None

    def active_here(self):
        return self.stream is not None and stream() == self.stream

    def add(self, ws_ptr, out, nslab, cols, accumulate=1):
        self.jobs.append((ws_ptr, ptr(out), nslab, cols, accumulate))

    def flush(self):
        if not self.jobs:
            return
        import ctypes as C
        n = len(self.jobs)
        ws = (C.c_void_p * n)(*[j[0] for j in self.jobs])
        out = (C.c_void_p * n)(*[j[1] for j in self.jobs])
        ns = (C.c_int * n)(*[j[2] for j in self.jobs])
        cs = (C.c_int * n)(*[j[3] for j in self.jobs])
        acc = (C.c_int * n)(*[j[4] for j in self.jobs])
        call("k3m_slab_reduce_batch", C.cast(ws, C.c_void_p), C.cast(out, C.c_void_p), C.cast(ns, C.c_void_p),
             C.cast(cs, C.c_void_p), C.cast(acc, C.c_void_p), n, stream())
        self.jobs = []
        self.keep = []


class deferred_reductions(object):
    """Context: slab reductions of ln_bwd / colsum on the current stream are batched until flush()."""

    def __enter__(self):
        global _deferred
        self.prev = _deferred
        _deferred = self.d = _Deferred()
        return self.d

    def __exit__(self, *exc):
        global _deferred
        try:
            if exc[0] is None:
                self.d.flush()
        finally:
            _deferred = self.prev
        return False


def _nslab(fn, rows):
    import ctypes as C
    v = C.c_int(0)
    call(fn, rows, C.byref(v))
    return v.value


DEFER = os.environ.get("K3M_DEFER_REDUCE", "1") != "0"   # A/B knob


def colsum(x, out, accumulate=True, alpha=1.0):
    rows, cols = x.shape
    if DEFER and _deferred is not None and alpha == 1.0 and accumulate and rows > 0 and cols > 0 and \
            _deferred.active_here():
        ns = _nslab("k3m_colsum_nslab", rows)
        ws = torch.empty((ns * cols,), dtype=torch.float32, device=x.device)
        call("k3m_colsum_slabs", ptr(x), _ld(x), rows, cols, ptr(ws), dt(x), stream())
        _deferred.keep.append(ws)
        _deferred.add(ptr(ws), out, ns, cols)
        return
    ws = torch.empty(((256 + 16) * cols,), dtype=torch.float32, device=x.device)
    if alpha == 1.0:
        call("k3m_colsum", ptr(x), _ld(x), rows, cols, ptr(out), int(accumulate), ptr(ws), dt(x), stream())
    else:
        tmp = torch.empty((cols,), dtype=torch.float32, device=x.device)
        call("k3m_colsum", ptr(x), _ld(x), rows, cols, ptr(tmp), 0, ptr(ws), dt(x), stream())
        if accumulate:
            add_(out, tmp, alpha)
        else:
            out.zero_()
            add_(out, tmp, alpha)


# ------------------------------------------------------------------ LayerNorm / embeddings
def ln_fwd(x, res, gamma, beta, y, xhat, rstd, p_in=0.0, p_out=0.0, seed=0, off_in=0, off_out=0, eps=1e-12):
    rows, cols = x.shape
    for t in (x, res, y, xhat):
        assert t is None or (t.is_contiguous() or t.stride(0) == cols)
    call("k3m_ln_fwd", ptr(x), ptr(res), ptr(gamma), ptr(beta), ptr(y), ptr(xhat), ptr(rstd), rows, cols, eps, p_in,
         p_out, seed, off_in, off_out, dt(x), stream())


LN_BWD_SLABS = 512   # K3M_LN_BWD_SLABS (include/k3m_hip.h)


def ln_bwd(dy, xhat, rstd, gamma, dres, dx, dgamma, dbeta, p_in=0.0, p_out=0.0, seed=0, off_in=0, off_out=0,
           acc_res=False, dxsum=None):
    """dxsum: optional fp32 [cols] that the column sums of dx are accumulated into (the bias
    gradient of the Linear whose output fed this LayerNorm)."""
    rows, cols = dy.shape
    if DEFER and _deferred is not None and rows > 0 and _deferred.active_here():
        ns = _nslab("k3m_ln_bwd_nslab", rows)
        ws = torch.empty((3 * ns * cols,), dtype=torch.float32, device=dy.device)
        call("k3m_ln_bwd_slabs", ptr(dy), ptr(xhat), ptr(rstd), ptr(gamma), ptr(dres), ptr(dx), rows, cols, p_in,
             p_out, seed, off_in, off_out, int(acc_res), int(dxsum is not None), ptr(ws), dt(dy), stream())
        _deferred.keep.append(ws)
        base, step = ptr(ws), ns * cols * 4
        _deferred.add(base, dgamma, ns, cols)
        _deferred.add(base + step, dbeta, ns, cols)
        if dxsum is not None:
            _deferred.add(base + 2 * step, dxsum, ns, cols)
        return
    ws = torch.empty((3 * (LN_BWD_SLABS + 16) * cols,), dtype=torch.float32, device=dy.device)
    call("k3m_ln_bwd", ptr(dy), ptr(xhat), ptr(rstd), ptr(gamma), ptr(dres), ptr(dx), ptr(dgamma), ptr(dbeta),
         ptr(dxsum), rows, cols, p_in, p_out, seed, off_in, off_out, int(acc_res), ptr(ws), dt(dy), stream())


def embed_fwd(ids, tt, word, pos, typ, gamma, beta, y0, y1, y2, xhat, rstd, p_out, seed, off, eps=1e-12):
    nseq, ln = ids.shape
    if _debug.ON:
        _debug.check_range(ids, 0, word.shape[0], "embedding ids")
        _debug.check_range(tt, 0, typ.shape[0], "token type ids")
        _debug.check_len(ln, pos.shape[0], "sequence length")
    call("k3m_embed_fwd", ptr(ids), ptr(tt), ptr(word), ptr(pos), ptr(typ), ptr(gamma), ptr(beta), ptr(y0), ptr(y1),
         ptr(y2), ptr(xhat), ptr(rstd), nseq, ln, word.shape[1], eps, p_out, seed, off, dt(y0), stream())


# Deterministic mode (SURVEY §5 "deterministic-mode flag"): the backward kernels that summed through float atomics
# (embedding rows, structure aggregator, LPM) run their fixed-order forms (k3m_*_det), so a step is bit-reproducible
# run to run.  K3M_DETERMINISTIC=1 at import, or set_deterministic() at run time.
DETERMINISTIC = os.environ.get("K3M_DETERMINISTIC", "0") not in ("", "0")


def set_deterministic(on=True):
    global DETERMINISTIC
    DETERMINISTIC = bool(on)


def embed_bwd(ids, tt, ds, dword, dpos, dtyp):
    nseq, ln = ids.shape
    if DETERMINISTIC:
        # the fixed-order kernel sums the token-type rows for ids {0, 1} only (type_vocab_size 2, every config of
        # the reference); refuse another table size instead of folding ids >= 2 into row 1 (an explicit error, not
        # an assert that `python -O` would strip)
        if dtyp.shape[0] != 2:
            raise ValueError("deterministic embedding backward supports type_vocab_size 2, got %d" % dtyp.shape[0])
        ws = torch.empty((ln * 2 * dword.shape[1],), dtype=torch.float32, device=ds.device)
        call("k3m_embed_bwd_det", ptr(ids), ptr(tt), ptr(ds), ptr(dword), ptr(dpos), ptr(dtyp), nseq, ln,
             dword.shape[1], ptr(ws), dt(ds), stream())
        return
    call("k3m_embed_bwd", ptr(ids), ptr(tt), ptr(ds), ptr(dword), ptr(dpos), ptr(dtyp), nseq, ln, dword.shape[1],
         dt(ds), stream())


# ------------------------------------------------------------------ attention
SHORT_MAXL = 128   # attention.hip keeps a whole head in LDS up to this length; attention_long.hip beyond
LDS_MAX = 160 * 1024


def _r32(n):
    return (n + 31) & ~31


def _short_fits(lq, lk, hd, bwd):
    """attention.hip's whole-head LDS images (fwd_lds / bwd_lds there) fit one CU's 160 KB; the
    largest shapes (e.g. 128 x 128 keys at head dim 128: seq_len 128 text <-> 128 PV co-attention,
    BASELINE configs[3]) go to the chunked attention_long.hip kernels instead."""
    if max(lq, lk) > SHORT_MAXL:
        return False
    LQ, LK = _r32(lq), _r32(lk)
    if not bwd:
        return 4 * (LQ * hd + LK * hd + LQ * LK) <= LDS_MAX
    r2n = max(LK * hd, LQ * LK)
    return 4 * (LQ * hd + r2n + LQ * LK + (0 if LK * hd + LQ <= r2n else LQ)) <= LDS_MAX


# attention_bf16.hip: the key-major backward (flash_bwd_km_kernel, default) or the P / dS image kernel
FLASH_BWD_KM = os.environ.get("K3M_FLASH_BWD_KM", "1") != "0"


def flash_fits(lq, lk, hd):
    """attention_bf16.hip's LDS images (fwd_lds and bwd_km_lds / bwd_lds there) fit 160 KB."""
    if max(lq, lk) > SHORT_MAXL or hd not in (64, 96, 128):
        return False
    LQ, LK, h = _r32(lq), _r32(lk), 128 if hd == 96 else hd
    fwd = 2 * (LQ * h + 2 * LK * h) + 4 * LK
    if FLASH_BWD_KM:
        QW = 128 if LQ == 96 else LQ
        bwd = 2 * (max(2 * LQ * h, LK * QW) + LK * h) + 4 * (LK + 2 * LQ) + 4 * LQ * (h // 8)
    else:
        PW = 128 if LK == 96 else LK
        bwd = 2 * (2 * LQ * h + 2 * LK * h + 2 * LQ * PW) + 4 * (LK + 2 * LQ)
    return max(fwd, bwd) <= LDS_MAX


FLASH_LONG = os.environ.get("K3M_FLASH_LONG", "1") != "0"
LONG_MAXL = 512   # max_position_embeddings (config/bert_base_6layer_6conect.json:8)


def flash_long_fits(lq, lk, hd):
    """attention_flash_long.hip: bf16 flash attention for any lq, lk <= 512 (the shapes flash_fits rejects)."""
    return FLASH_LONG and 0 < lq <= LONG_MAXL and 0 < lk <= LONG_MAXL and hd in (64, 96, 128)


def attn_fwd(q, k, v, kmask, ctx, probs, nseq, lq, lk, nh, hd, scale, p_drop, seed, off):
    name = "k3m_attn_fwd" if _short_fits(lq, lk, hd, False) else "k3m_attn_long_fwd"
    call(name, ptr(q), _ld(q), ptr(k), _ld(k), ptr(v), _ld(v), ptr(kmask), ptr(ctx), _ld(ctx), ptr(probs),
         nseq, lq, lk, nh, hd, scale, p_drop, seed, off, dt(ctx), stream())


def attn_bwd(dctx, o, q, k, v, probs, dq, dk, dv, nseq, lq, lk, nh, hd, scale, p_drop, seed, off):
    if _short_fits(lq, lk, hd, True):
        call("k3m_attn_bwd", ptr(dctx), _ld(dctx), ptr(o), _ld(o), ptr(q), _ld(q), ptr(k), _ld(k), ptr(v), _ld(v),
             ptr(probs), ptr(dq), ptr(dk), ptr(dv), _ld(dq), _ld(dk), _ld(dv), nseq, lq, lk, nh, hd, scale, p_drop,
             seed, off, dt(dctx), stream())
        return
    ws = torch.empty_like(probs)
    call("k3m_attn_long_bwd", ptr(dctx), _ld(dctx), ptr(o), _ld(o), ptr(q), _ld(q), ptr(k), _ld(k), ptr(v), _ld(v),
         ptr(probs), ptr(ws), ptr(dq), ptr(dk), ptr(dv), _ld(dq), _ld(dk), _ld(dv), nseq, lq, lk, nh, hd, scale,
         p_drop, seed, off, dt(dctx), stream())


def flash_attn_fwd(q, k, v, kmask, ctx, lse, nseq, lq, lk, nh, hd, scale, p_drop, seed, off):
    """bf16 attention forward saving the row log-sum-exp (lse: fp32 [nseq*nh*lq]): the whole-head kernels of
    attention_bf16.hip where they fit (L <= 128), else attention_flash_long.hip (L <= 512)."""
    name = "k3m_flash_attn_fwd" if flash_fits(lq, lk, hd) else "k3m_flash_attn_long_fwd"
    call(name, ptr(q), _ld(q), ptr(k), _ld(k), ptr(v), _ld(v), ptr(kmask), ptr(ctx), _ld(ctx),
         ptr(lse), nseq, lq, lk, nh, hd, scale, p_drop, seed, off, stream())


_ws_cache = {}


def flash_long_ws_bytes(nseq, lq, lk, nh, hd):
    key = (nseq, lq, lk, nh, hd)
    b = _ws_cache.get(key)
    if b is None:
        out = C.c_longlong(0)
        call("k3m_flash_attn_long_ws_bytes", nseq, lq, lk, nh, hd, C.addressof(out))
        b = _ws_cache[key] = int(out.value)
    return b


def flash_attn_bwd(dctx, o, q, k, v, kmask, lse, dq, dk, dv, nseq, lq, lk, nh, hd, scale, p_drop, seed, off):
    if flash_fits(lq, lk, hd):
        call("k3m_flash_attn_bwd", ptr(dctx), _ld(dctx), ptr(o), _ld(o), ptr(q), _ld(q), ptr(k), _ld(k), ptr(v),
             _ld(v), ptr(kmask), ptr(lse), ptr(dq), ptr(dk), ptr(dv), _ld(dq), _ld(dk), _ld(dv), nseq, lq, lk, nh, hd,
             scale, p_drop, seed, off, stream())
        return
    nb = flash_long_ws_bytes(nseq, lq, lk, nh, hd)
    ws = torch.empty((max(nb, 16),), dtype=torch.uint8, device=dq.device)
    call("k3m_flash_attn_long_bwd", ptr(dctx), _ld(dctx), ptr(o), _ld(o), ptr(q), _ld(q), ptr(k), _ld(k), ptr(v),
         _ld(v), ptr(kmask), ptr(lse), ptr(dq), ptr(dk), ptr(dv), _ld(dq), _ld(dk), _ld(dv), ptr(ws), nb, nseq, lq, lk,
         nh, hd, scale, p_drop, seed, off, stream())


# ------------------------------------------------------------------ elementwise / rows
def dgelu(g, pre, out):
    call("k3m_dgelu", ptr(g), ptr(pre), ptr(out), g.numel(), dt(g), stream())


def add_(y, x, alpha=1.0):
    assert y.is_contiguous() and x.is_contiguous() and y.numel() == x.numel()
    call("k3m_add_inplace", ptr(y), ptr(x), y.numel(), alpha, dt(y), stream())


def convert(x, y, accumulate=False, alpha=1.0):
    """y (+)= alpha * x across dtypes (fp32 <-> bf16); both contiguous with equal numel."""
    assert x.numel() == y.numel() and x.is_contiguous() and y.is_contiguous()
    call("k3m_convert", ptr(x), dt(x), ptr(y), dt(y), x.numel(), int(accumulate), alpha, stream())
    return y


def gather_rows(src, idx, n, out):
    if _debug.ON:
        _debug.check_range(idx[:n], 0, src.shape[0], "gather_rows index")
    call("k3m_gather_rows", ptr(src), _ld(src), ptr(idx), n, src.shape[1], ptr(out), _ld(out), dt(src), stream())


def scatter_add_rows(src, idx, n, dst):
    if _debug.ON:
        _debug.check_range(idx[:n], 0, dst.shape[0], "scatter_add_rows index")
    call("k3m_scatter_add_rows", ptr(src), _ld(src), ptr(idx), n, src.shape[1], ptr(dst), _ld(dst), dt(src),
         stream())

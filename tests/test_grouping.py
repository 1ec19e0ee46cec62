"""Host logic of the grouped GEMM launch (k3m_amd.ops.grouped) on the CPU: GEMMs issued inside the
block are deferred, grouped by kernel template (layout, epilogue, dtypes), chunked by GROUP_MAX and
launched through k3m_gemm_grouped at the exit; deferred non-GEMM work runs at the flush; outside a
block every GEMM launches at once.  The launches are recorded instead of executed (no GPU)."""
import torch

from k3m_amd import ops, _lib as L


def _record(monkeypatch):
    calls = []

    def fake_call(name, *args):
        if name == "k3m_gemm_grouped":
            arr = L.C.cast(args[0], L.C.POINTER(L.K3mGemm))
            calls.append((name, [(arr[i].m, arr[i].n, arr[i].k, arr[i].epilogue, arr[i].a_trans) for i in range(args[1])]))
        elif name == "k3m_gemm":
            g = args[0]._obj
            calls.append((name, [(g.m, g.n, g.k, g.epilogue, g.a_trans)]))
        else:
            calls.append((name, None))
    monkeypatch.setattr(ops, "call", fake_call)
    monkeypatch.setattr(ops, "stream", lambda: None)
    return calls


def test_outside_a_block_launches_immediately(monkeypatch):
    calls = _record(monkeypatch)
    x, w = torch.zeros(64, 32), torch.zeros(16, 32)
    ops.linear(x, w)
    assert calls == [("k3m_gemm", [(64, 16, 32, L.EPI_NONE, 0)])]


def test_block_groups_by_template_and_chunks(monkeypatch):
    calls = _record(monkeypatch)
    xs = [torch.zeros(64 + i, 32) for i in range(11)]
    w, b = torch.zeros(16, 32), torch.zeros(16)
    with ops.grouped():
        for x in xs:
            ops.linear(x, w, b)                 # BIAS epilogue, nt: one template
        ops.linear(xs[0], w)                    # no bias: another template
        assert calls == []                      # nothing launched inside the block
    names = [c[0] for c in calls]
    assert names == ["k3m_gemm_grouped"] * 3
    sizes = sorted(len(c[1]) for c in calls)
    assert sizes == [1, 3, ops.GROUP_MAX]       # 11 BIAS problems -> 8 + 3; 1 NONE problem
    assert all(len({p[3] for p in c[1]}) == 1 for c in calls)


def test_wgrad_bias_colsum_deferred_to_flush(monkeypatch):
    calls = _record(monkeypatch)
    dy, x = torch.zeros(4096, 16), torch.zeros(4096, 32)
    gW, gb = torch.zeros(16, 32), torch.zeros(16)
    with ops.grouped():
        ops.linear_wgrad(dy, x, gW, gb)
        assert calls == []                      # the bias colsum waits for the flush too
    assert [c[0] for c in calls] == ["k3m_colsum", "k3m_gemm_grouped"]
    assert calls[1][1][0][4] == 1               # a_trans: dY^T . X


def test_blocks_do_not_nest(monkeypatch):
    _record(monkeypatch)
    with ops.grouped():
        try:
            with ops.grouped():
                pass
            raise RuntimeError("nested block accepted")
        except AssertionError:
            pass

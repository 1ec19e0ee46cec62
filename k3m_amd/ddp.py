"""Data-parallel gradient exchange: one process per GPU, RCCL all-reduce over xGMI (torch
"nccl" backend on ROCm), overlapped with the backward pass.

Replaces apex.parallel.DistributedDataParallel (train_concap_struc.py:303-308).  Design for
MI355X:
* gradients live in ONE flat fp32 buffer (k3m_amd/params.py), so a bucket is a contiguous slice —
  no bucket copy in or out;
* buckets follow the real grad-ready order of the wide engine: heads / fusion / structure
  aggregator first, then each encoder block (text layer, image layer, co-attention block) as soon
  as its backward finishes, embeddings last (the word embedding also carries the tied MLM
  decoder gradient, so it is final only at the very end);
* the 86 never-grad tensors (frozen segment) are excluded — apex/torch DDP would wait on them;
* all-reduces run on a dedicated HIP stream that waits on an event recorded after the block's
  backward, so RCCL traffic overlaps the remaining backward kernels; averaging (1/world) is
  folded into the AdamW kernel's grad_scale;
* parameters are broadcast from rank 0 at start (DDP's initial sync).
"""
import torch
import torch.distributed as dist

from .params import param_spec, segment_of


def _block_of(name):
    parts = name.split(".")
    if parts[0] == "encoder":
        kind = {"layer": "t", "v_layer": "v"}.get(parts[1], "c")
        return (kind, int(parts[2]))
    if parts[0] in ("embeddings", "v_embeddings"):
        return ("emb", 0)
    return ("head", 0)


class GradAllReducer(object):
    def __init__(self, fp, group=None, max_bucket_elems=32 * 1024 * 1024):
        self.group = group
        self.world = dist.get_world_size(group)
        self.fp = fp
        # contiguous ranges per readiness block
        ranges = {}
        for name, shape in fp.spec:
            if segment_of(name) == "frozen":
                continue
            blk = _block_of(name)
            o = fp.offsets[name]
            n = 1
            for s in shape:
                n *= s
            ranges.setdefault(blk, []).append((o, o + n))
        self.blocks = {}
        for blk, rs in ranges.items():
            rs.sort()
            merged = []
            for a, b in rs:
                # tensors of a block are adjacent up to 16-byte alignment padding
                if merged and a - merged[-1][1] < 4:
                    merged[-1] = (merged[-1][0], b)
                else:
                    merged.append((a, b))
            # split into buckets of at most max_bucket_elems
            out = []
            for a, b in merged:
                while b - a > max_bucket_elems:
                    out.append((a, a + max_bucket_elems))
                    a += max_bucket_elems
                out.append((a, b))
            self.blocks[blk] = out
        self.stream = None
        self.pending = []
        self.done = set()

    def broadcast_params(self, fp):
        dist.broadcast(fp.data, src=0, group=self.group)
        fp.shadow_fresh = False

    def begin(self, engine):
        self.done = set()
        self.pending = []
        if self.fp.grad.is_cuda and self.stream is None:
            self.stream = torch.cuda.Stream(device=self.fp.grad.device)

    def _launch(self, blk):
        if blk in self.done or blk not in self.blocks:
            return
        self.done.add(blk)
        g = self.fp.grad
        if g.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(g.device))
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                for a, b in self.blocks[blk]:
                    self.pending.append(dist.all_reduce(g[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        else:
            for a, b in self.blocks[blk]:
                self.pending.append(dist.all_reduce(g[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def grad_ready(self, kind, index):
        if kind in ("t", "v", "c"):
            self._launch(("head", 0))   # heads/fusion/struct grads are final before the encoder
            self._launch((kind, index))
        elif kind == "emb":
            self._launch(("head", 0))
            self._launch(("emb", 0))

    def finish(self):
        for blk in list(self.blocks):
            self._launch(blk)
        for w in self.pending:
            w.wait()
        self.pending = []
        if self.fp.grad.is_cuda:
            torch.cuda.current_stream(self.fp.grad.device).wait_stream(self.stream)

"""World-size-2 gloo test of the gradient exchange (k3m_amd/ddp.py) on CPU: buckets cover every
trainable parameter exactly once, follow the grad-ready order, exclude the frozen tensors, and the
all-reduced flat buffer equals the sum over ranks."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class FakeFlat(object):
    def __init__(self, cfg):
        from k3m_amd.params import flat_layout
        self.spec, self.offsets, self.segments, self.total, self.shapes = flat_layout(cfg)
        self.grad = torch.zeros(self.total)
        self.data = torch.zeros(self.total)


def small_cfg():
    from k3m_amd.config import BertConfig
    c = BertConfig.from_json_file(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "configs", "bert_base_6layer_6conect.json"))
    c.hidden_size, c.intermediate_size, c.num_attention_heads = 64, 128, 4
    c.v_hidden_size, c.v_intermediate_size, c.bi_hidden_size = 64, 64, 64
    c.v_num_attention_heads, c.bi_num_attention_heads, c.vocab_size = 4, 4, 500
    c.v_feature_size, c.v_target_size = 32, 40
    c.with_coattention, c.if_pre_sampling = True, 1
    return c


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from k3m_amd.ddp import GradAllReducer
    from k3m_amd.params import segment_of
    fp = FakeFlat(small_cfg())
    g = torch.Generator().manual_seed(rank)
    r = torch.randn(fp.total, generator=g)
    for n, s in fp.spec:          # gaps between tensors and frozen tensors hold zero gradients
        if segment_of(n) != "frozen":
            o = fp.offsets[n]
            k = int(torch.tensor(s).prod())
            fp.grad[o:o + k] = r[o:o + k]
    want = fp.grad.clone()
    red = GradAllReducer(fp, max_bucket_elems=50000)
    red.begin(None)
    order = []
    orig = red._launch

    def spy(blk):
        if blk not in red.done:
            order.append(blk)
        orig(blk)
    red._launch = spy
    for kind, i in [("t", 11), ("v", 5), ("c", 5), ("t", 10), ("emb", 0)]:
        red.grad_ready(kind, i)
    red.finish()
    fp.data.copy_(torch.full((fp.total,), float(rank)))
    red.broadcast_params(fp)
    q.put((rank, want.numpy(), fp.grad.numpy().copy(), order, float(fp.data.max())))
    dist.destroy_process_group()


def test_allreduce_buckets_gloo():
    from k3m_amd.params import segment_of
    world = 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in ps:
        p.join(60)
    total = torch.from_numpy(res[0][1] + res[1][1])
    fp = FakeFlat(small_cfg())
    mask = torch.zeros(fp.total, dtype=torch.bool)
    for n, sh in fp.spec:
        if segment_of(n) != "frozen":
            o = fp.offsets[n]
            mask[o:o + int(torch.tensor(sh).prod())] = True
    for r in range(world):
        got = torch.from_numpy(res[r][2])
        assert torch.allclose(got[mask], total[mask], atol=1e-5)
        assert torch.all(got[~mask] == 0)
        assert res[r][4] == 0.0          # parameters broadcast from rank 0
    order = res[0][3]
    assert order[0] == ("head", 0) and order[1] == ("t", 11) and order[2] == ("v", 5)
    assert ("emb", 0) in order

"""Measure the data path at the driver's geometry (B=64, T=36, P=128,
36 regions x 2048 features, 1601 targets):

* collate kernel: k3m_collate_regions timed with HIP events on its own stream; algorithmic bytes
  per launch = B*R*F*4 read + B*(R+1)*F*4 written + 2*B*R flag bytes; roofline vs 8 TB/s;
* host prep: BertPreprocessBatch.prepare (native masking; tokenisation by the character tokenizer
  of the golden fixtures) in samples/s on one core;
* loader: records -> batch dict on the GPU (prep + staging + H2D + collation), samples/s;
* cpu_baseline: the numpy collation of the reference (oracle/data_oracle.py) on the same batch.

Prints one JSON line.  Usage: python scripts/bench_data.py [--reps 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

from k3m_amd import _lib, data as D  # noqa: E402
from make_golden import CharTokenizer  # noqa: E402
from oracle import data_oracle as DO  # noqa: E402

PEAK_HBM = 8.0e12


def synth_records(n, rng, F=2048, C=1601):
    recs = []
    for i in range(n):
        nb = int(rng.integers(10, 37))
        x1 = rng.uniform(0, 500, nb)
        y1 = rng.uniform(0, 400, nb)
        boxes = np.stack([x1, y1, x1 + rng.uniform(20, 300, nb), y1 + rng.uniform(20, 200, nb)], 1).astype(np.float32)
        title = "".join(chr(0x4e00 + int(c)) for c in rng.integers(0, 2000, int(rng.integers(10, 40))))
        pv = "#;#".join("%s#:#%s" % ("".join(chr(0x4e00 + int(c)) for c in rng.integers(0, 2000, 3)),
                                      "".join(chr(0x4e00 + int(c)) for c in rng.integers(0, 2000, 4)))
                        for _ in range(int(rng.integers(0, 15))))
        recs.append(("id%d" % i, title, pv, "", 600, 800, nb, boxes,
                     np.abs(rng.standard_normal((nb, F))).astype(np.float32),
                     rng.random((nb, C)).astype(np.float32)))
    return recs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    B, R, F = a.batch, 36, 2048
    rng = np.random.default_rng(0)
    recs = synth_records(4 * B, rng)
    tok = CharTokenizer()
    pre = D.BertPreprocessBatch(tok, max_seq_len=36, max_seq_len_pv=128, max_num_pv=20, max_region_len=R,
                                streams=D.RandomStreams(1))
    # host prep, one core
    t0 = time.perf_counter()
    samples = [pre.prepare(r) for r in recs]
    host_sps = len(recs) / (time.perf_counter() - t0)

    dev = torch.device("cuda", 0)
    col = D.RegionCollator(dev, R, F, 1601)
    batch, _ = col(samples[:B])
    torch.cuda.synchronize()
    # loader (prep + staging + H2D + collation), steady state
    n_it = 3
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(n_it):
        sb = [pre.prepare(r) for r in recs[it * B:(it + 1) * B]]
        batch, _ = col(sb)
    torch.cuda.synchronize()
    loader_sps = n_it * B / (time.perf_counter() - t0)

    # collate kernel alone on a side stream, HIP events
    feat = torch.from_numpy(np.stack([np.pad(s.feat, ((0, R - s.feat.shape[0]), (0, 0))) for s in samples[:B]])).to(dev)
    zero = torch.from_numpy(np.stack([s.zero_feat for s in samples[:B]])).to(dev)
    mlab = torch.from_numpy(np.stack([s.masked_label for s in samples[:B]])).to(dev)
    out = torch.empty((B, R + 1, F), device=dev)
    st = torch.cuda.Stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        for _ in range(10):
            _lib.call("k3m_collate_regions", feat.data_ptr(), R * F, zero.data_ptr(), mlab.data_ptr(), None, B, R, F,
                      out.data_ptr(), st.cuda_stream)
        e0.record(st)
        for _ in range(a.reps):
            _lib.call("k3m_collate_regions", feat.data_ptr(), R * F, zero.data_ptr(), mlab.data_ptr(), None, B, R, F,
                      out.data_ptr(), st.cuda_stream)
        e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.reps
    byts = B * R * F * 4 + B * (R + 1) * F * 4 + 2 * B * R
    want = DO.collate_regions(feat.cpu().numpy(), zero.cpu().numpy(), mlab.cpu().numpy())
    exact = bool(np.array_equal(out.cpu().numpy(), want))

    # CPU baseline: the reference's numpy collation of one batch
    f_np, z_np, m_np = feat.cpu().numpy(), zero.cpu().numpy(), mlab.cpu().numpy()
    t0 = time.perf_counter()
    n_cpu = 0
    while time.perf_counter() - t0 < 10.0:
        DO.collate_regions(f_np, z_np, m_np)
        n_cpu += 1
    cpu_sps = n_cpu * B / (time.perf_counter() - t0)

    line = {"metric": "data_path_samples_per_sec", "value": loader_sps, "unit": "samples/s",
            "config": {"workload": "records -> GPU batch (bert_base_6layer_6conect geometry)", "batch": B,
                       "regions": R, "v_feature_size": F, "seq_len": 36, "seq_len_pv": 128},
            "host_prep_samples_per_sec_1core": host_sps,
            "collate_kernel": {"us": us, "bytes": byts, "achieved_GBs": byts / us / 1e3, "peak_GBs": PEAK_HBM / 1e9,
                               "frac": byts / us / 1e3 / (PEAK_HBM / 1e9), "bit_exact_vs_oracle": exact},
            "cpu_baseline": {"value": cpu_sps, "unit": "samples/s", "cores": 1, "kind": "port",
                             "sample": "numpy collation (oracle/data_oracle.py) of one B=%d batch, repeated ~10 s" % B}}
    print(json.dumps(line))


if __name__ == "__main__":
    main()

"""Benchmark: K3M tri-modal pretraining step (bert_base_6layer_6conect) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config {2,3,4,5}] [--dtype fp32|bf16]
                    [--batch B] [--no-cpu-baseline]

One step = forward + backward + (RCCL gradient all-reduce when N > 1) + AdamW + LR schedule over
one synthetic batch resident in HBM (SURVEY.md §8(d) input spec: random token ids, region
features, PV triples).  Workloads (BASELINE.json configs):
  2 (default) bert_base_6layer_6conect fp32, bs=64/GPU, T=36, P=128, 36 boxes, 10 triples — the metric's config;
  3 the same in bf16 (mixed precision: bf16 encoder, fp32 master weights / heads / optimizer);
  4 T=128, 100 boxes, bs=256/GPU (bf16);   5 P=320, 50 triples (NPV 50), bs=128/GPU (bf16).
N > 1: one rank per GPU over RCCL.  Under torch.distributed.run (WORLD_SIZE set) this process is a
rank; with ``--gpus N`` and no WORLD_SIZE it launches ``torch.distributed.run --nproc-per-node N``
itself, before touching the GPU, and exits with its status.  Each rank runs its own bs=B batch
(weak scaling, global batch = B N); the timed region is bracketed by barrier + synchronize and the
max over ranks is taken.

Rank 0 prints ONE JSON line with the driver's contract plus
  roofline        — the dominant kernel by time (the 256x256 weight-gradient walk, ~21 % of the fp32 step) on its
                    largest launch shape, the text-layer FFN1 weight gradient (3072 x 768 x 2BT+2BP rows),
                    timed with HIP events on its stream over the timed steps, against the peak of the
                    arithmetic it runs on (fp32: bf16x6 split = bf16 dense peak / 6; bf16: bf16 peak);
                    ``class``: every text-layer weight gradient on that kernel;
  roofline_ffn1   — the text-layer FFN1 forward GEMM (2BT+2BP rows x 3072 x 768, bias+GELU), as rounds 1-5;
  parity          — the engine's five losses against the CPU oracle's on the CPU baseline's bs=64 batch;
  coattn          — the co-attention blocks (18 layers: both directions' attention, projections,
                    FFNs, LayerNorms; forward + backward) timed with HIP events: their algorithmic
                    FLOPs / time against the same peak (north-star target >= 0.40);
  cpu_baseline    — the CPU oracle (plain PyTorch fp32 restatement of the same step, oracle/) on the
                    host cores, bounded sample (rank 0, N = 1 only).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

# BASELINE.json "metric"; `value` is the whole-job aggregate over the n_gpus ranks (per_gpu_samples_s beside it)
BASELINE_METRIC = "pretrain samples/sec/GPU (bert_base_6layer_6conect, bs=64) at 1/2/4/8 MI355X"
PEAK_F32_MFMA = 157.3e12      # MI355X f32 MFMA dense peak (MI355X_MICROARCH.md)
PEAK_BF16_MFMA = 2.5e15
PROBE_STEPS = 2   # eager steps that carry the HIP-event probes when the timed steps are graph replays
PEAK_F32_X6 = PEAK_BF16_MFMA / 6   # fp32 GEMM as 6 bf16 MFMA partial products (gemm_x6_tile.h)

# BASELINE.json configs -> synthetic workload shapes
CONFIGS = {
    2: dict(B=64, T=36, P=128, nbox=36, n_triples=10, npv=20, dtype="fp32"),
    3: dict(B=64, T=36, P=128, nbox=36, n_triples=10, npv=20, dtype="bf16"),
    4: dict(B=256, T=128, P=128, nbox=100, n_triples=10, npv=20, dtype="bf16"),
    5: dict(B=128, T=36, P=320, nbox=36, n_triples=50, npv=50, dtype="bf16"),
}


def ref_fwd_flops(T, P, R, Nt, H=768, I=3072, V=21128, Hv=1024, Iv=1024, Hb=1024, Cv=1601):
    """Reference algorithmic forward FLOPs per sample (SURVEY.md §8(d) formula; 106.48 GF at config 2)."""
    def f_t(L): return 2 * L * (4 * H * H + 2 * H * I) + 4 * L * L * H
    def f_v(R_): return 2 * R_ * (4 * Hv * Hv + 2 * Hv * Iv) + 4 * R_ * R_ * Hv
    c = coattn_fwd_flops(T, P, R, H, I, Hv, Iv, Hb)
    return (24 * f_t(T) + 24 * f_t(P) + 12 * f_v(R) + c + 2 * R * (2048 + 5) * Hv
            + 2 * (T + P) * (H * H + H * V) + 2 * R * (Hv * Hv + Hv * Cv)
            + 3 * 2 * R * 3 * Hb * Hb + 3 * 2 * (T + P) * 3 * H * H + 2 * Nt * 3 * H * H)


def coattn_fwd_flops(T, P, R, H=768, I=3072, Hv=1024, Iv=1024, Hb=1024):
    """6 x c_layer(T,R) + 6 x c_layer_pv_v(P,R) + 6 x c_layer_pv_t(T,P) forward FLOPs per sample."""
    def c_tv(L, R_): return (2 * R_ * (3 * Hv * Hb + Hb * Hv + 2 * Hv * Iv) + 2 * L * (3 * H * Hb + Hb * H + 2 * H * I)
                             + 8 * L * R_ * Hb)
    def c_tt(T_, P_): return (T_ + P_) * (2 * (3 * H * H + H * H + 2 * H * I)) + 8 * T_ * P_ * H
    return 6 * c_tv(T, R) + 6 * c_tv(P, R) + 6 * c_tt(T, P)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--dtype", default=None, choices=["fp32", "bf16"], help="default: the config's")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=64, help="CPU baseline batch (the GPU workload's bs=64)")
    ap.add_argument("--cpu-steps", type=int, default=1, help="timed CPU steps at --cpu-batch (after a bs=8 "
                    "warm-up step and a bs=8 sample of 2 timed steps)")
    ap.add_argument("--backend", default="nccl", help="nccl (RCCL) for real runs; gloo only to rehearse the "
                    "multi-rank path with several ranks sharing one GPU")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("--graph", default=None, choices=["auto", "on", "off"],
                    help="hipGraph replay of the step (k3m_amd/graph.py); default: K3M_GRAPH (auto)")
    ap.add_argument("--ddp", action="store_true", help="run the data-parallel path (process group, bucketed "
                    "all-reduce on the comm stream) even at one rank: exercises RCCL at world size 1")
    return ap.parse_args()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """--gpus N without a torch.distributed.run parent: start N ranks as children (no GPU touched here)."""
    port = args.master_port or free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


class GemmProbe(object):
    """Times every launch of one GEMM shape (or of a set of shapes) with HIP events on the launching stream."""

    def __init__(self, m, n, k, more=()):
        self.key = (m, n, k)
        self.keys = {self.key} | set(more)
        self.events = []
        self.shapes = []
        self.active = False

    def install(self):
        import torch
        from k3m_amd import ops
        orig = ops.gemm
        probe = self

        def wrapped(a, a_trans, b, b_trans, c, m, n, k, *args, **kw):
            if probe.active and (m, n, k) in probe.keys and ops._grouper is None:   # a deferred GEMM is not timed here
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                r = orig(a, a_trans, b, b_trans, c, m, n, k, *args, **kw)
                e.record()
                probe.events.append((s, e))
                probe.shapes.append((m, n, k))
                return r
            return orig(a, a_trans, b, b_trans, c, m, n, k, *args, **kw)

        prev = ops.gemm
        ops.gemm = wrapped
        return prev

    def launches(self, key=None):
        return [se for se, sh in zip(self.events, self.shapes) if key is None or sh == key]

    def mean_ms(self, key=None):
        ev = self.launches(key if key is not None else self.key)
        if not ev:
            return None
        return sum(s.elapsed_time(e) for s, e in ev) / len(ev)

    def aggregate(self):
        """(launches, total ms, total FLOPs) over every probed launch of every probed shape."""
        if not self.events:
            return 0, 0.0, 0.0
        return (len(self.events), sum(s.elapsed_time(e) for s, e in self.events),
                sum(2.0 * m * n * k for m, n, k in self.shapes))


class CoattnProbe(object):
    """HIP events around every co-attention block (the engine's lock-step runs of the three
    co-attention layers of one schedule step, forward and backward)."""

    def __init__(self):
        self.events = []
        self.active = False

    def install(self):
        import torch
        from k3m_amd import engine
        orig = engine._lockstep
        probe = self

        def wrapped(gens):
            if not probe.active:
                return orig(gens)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = orig(gens)
            e.record()
            probe.events.append((s, e))
            return r

        engine._lockstep = wrapped

    def total_ms(self):
        return sum(s.elapsed_time(e) for s, e in self.events)


class GemmAllProbe(object):
    """HIP events around EVERY GEMM launch (single and grouped, as scripts/gemm_calls.py) of one eager step run after
    the timed region: the step's GEMM aggregate (algorithmic TFLOP / GEMM ms) and its largest call class."""

    def __init__(self):
        self.rec = []
        self.active = False

    def install(self):
        import torch
        from k3m_amd import ops, _lib as L
        orig = L.call
        probe = self

        def sig(g):
            return "%s%s m=%d n=%d k=%d epi=%d s=%d" % ("t" if g.a_trans else "n", "t" if g.b_trans else "n", g.m, g.n,
                                                        g.k, g.epilogue & 0xff, g.splitk)

        def wrapped(name, *a):
            if not probe.active or name not in ("k3m_gemm", "k3m_gemm_grouped"):
                return orig(name, *a)
            if name == "k3m_gemm":
                gs = [a[0]._obj]
            else:
                arr = L.C.cast(a[0], L.C.POINTER(L.K3mGemm))
                gs = [arr[i] for i in range(a[1])]
            key = ("group[%d] " % len(gs) if name == "k3m_gemm_grouped" else "") + " + ".join(sig(g) for g in gs)
            flops = sum(2.0 * g.m * g.n * g.k for g in gs)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            r = orig(name, *a)
            e.record()
            probe.rec.append((key, flops, s, e))
            return r
        L.call = wrapped
        ops.call = wrapped

    def summary(self, peak):
        import collections
        agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
        for key, flops, s, e in self.rec:
            a = agg[key]
            a[0] += 1
            a[1] += s.elapsed_time(e)
            a[2] += flops
        ms = sum(v[1] for v in agg.values())
        tf = sum(v[2] for v in agg.values()) / 1e12
        if ms <= 0:
            return None
        top_key, (n, tms, tfl) = max(agg.items(), key=lambda kv: kv[1][1])
        return {"ms_per_step": round(ms, 3), "tflop_per_step": round(tf, 4), "launches": len(self.rec),
                "achieved": round(tf / (ms * 1e-3), 2), "peak": peak / 1e12, "unit": "TFLOP/s",
                "frac": round(tf * 1e12 / (ms * 1e-3) / peak, 4),
                "largest_class": {"calls": top_key[:160], "launches": n, "ms_per_step": round(tms, 3),
                                  "share": round(tms / ms, 4), "achieved": round(tfl / (tms * 1e-3) / 1e12, 2)},
                "probe": "HIP events around every GEMM launch of one eager step after the timed region "
                         "(scripts/gemm_calls.py's method)"}


def head_kernel(bf):
    """Full-name fragment of the kernel the probed GEMM runs at HEAD with the default knobs (gemm.hip /
    gemm_bf16.hip dispatch of a 256x256-tile problem of >= K3M_*_PERSIST_MIN blocks)."""
    if bf:   # FFN1 has the GELU epilogue: K3M_B16_DUAL (default 2) runs it on the two-workgroups-per-CU kernel
        if os.environ.get("K3M_B16_DUAL", "2") != "0":
            return "k3m_b16::gemm_dual_kernel<256, 128"
        return "k3m_b16::gemm_persist_kernel<256, 256" if os.environ.get("K3M_B16_PERSIST", "1") != "0" \
            else "k3m_b16::gemm_kernel<256, 256"
    if os.environ.get("K3M_X6_PERSIST", "1") == "0":
        return "k3m_x6::gemm_x6_kernel<256, 256"
    # the FFN1 forward (both operands K-contiguous, bias+GELU epilogue = 2); last argument: the main loop
    # (0 compiler-scheduled, 1 ping-pong: K3M_X6_PP bit 0, on by default)
    pp = (int(os.environ.get("K3M_X6_PP", "63")) & 1) != 0
    return "k3m_x6::gemm_x6_persist_kernel<256, 256, 4, 2, 16, true, true, 2, true, %d>" % (1 if pp else 0)


def head_wgrad_kernel(bf):
    """Full-name fragment of the kernel the text-layer weight gradients (tn, k = 20,992 split over k) run on at HEAD:
    the 256x256 walk with both operands MN-contiguous and no epilogue; fp32: the last argument is the main loop
    (2 = PPDLoop, LDS-DMA staged raw tiles, K3M_X6_PP bits 1|2 on by default)."""
    if bf:
        return "k3m_b16::gemm_persist_kernel<256, 256, 2, 4, false, false, 0, float, 32, false>"
    if os.environ.get("K3M_X6_PERSIST", "1") == "0":
        return "k3m_x6::gemm_x6_kernel<256, 256"
    pp = int(os.environ.get("K3M_X6_PP", "63"))
    loop = 2 if (pp & 4 and pp & 32) else (1 if pp & 4 else 0)   # gemm_x6p.hip kPP: 4 weight gradients, 32 on PPDLoop
    return "k3m_x6::gemm_x6_persist_kernel<256, 256, 2, 4, 16, false, false, 0, false, %d>" % loop


def pmc_traffic(key, kernel):
    """HBM-side bytes per launch of the probed GEMM from the newest committed rocprofv3 PMC record of THIS
    kernel and shape (profiles/r*_pmc_*.json from scripts/pmc_gemm.sh + scripts/pmc_table.py: FETCH_SIZE x2
    gfx950 correction + WRITE_SIZE), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(HERE, "profiles", "r*pmc*.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        # rocprofv3 names keep the "(anonymous namespace)::" of the kernels' translation units
        names = [n.replace("(anonymous namespace)::", "") for n in (d.get("kernel_names") or [d.get("kernel", "")])]
        if tuple(d.get("shape") or ()) == tuple(key) and d.get("traffic_bytes") and any(kernel in n for n in names):
            return int(d["traffic_bytes"]), os.path.relpath(path, HERE)
    return None, None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """Threads for the CPU baseline = this process's CPU share: the affinity mask (os.sched_getaffinity),
    capped by the cgroup's CPU quota (cpu.max) when one is set — on the GPU box nproc / os.cpu_count()
    report the whole machine.  Returns (threads, how it was determined)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    n = min(aff, quota) if quota else aff
    return n, "sched_getaffinity=%d, cgroup cpu.max=%s, nproc=%d" % (aff, quota if quota else "max",
                                                                      os.cpu_count() or 0)


PARITY_LOSSES = ("masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv", "loss_lpm", "next_sentence_loss", "loss")


def parity_inputs(cfg, shape, b, device):
    """The CPU baseline's batch, gumbel noise and LPM negative tables (seeded, identical on every device)."""
    import torch
    from k3m_amd.synthetic import synthetic_batch, synthetic_noise
    T, Pl, nbox = shape["T"], shape["P"], shape["nbox"]
    batch = synthetic_batch(cfg, b, "cpu", seed=99, T=T, P=Pl, n_boxes=nbox, n_triples=shape["n_triples"],
                            npv=shape["npv"])
    noise = synthetic_noise(cfg, b, seed=1, T=T, P=Pl, R=nbox + 1)
    NPV = batch["index_p"].shape[1]
    nt = shape["n_triples"]
    ent = torch.full((b, NPV, 2), -1, dtype=torch.int64)
    val = torch.full((b, NPV, 2), -1, dtype=torch.int64)
    for i in range(b):
        for j in range(nt):
            ent[i, j, 0] = (i + 1) % b if b > 1 else -1
            ent[i, j, 1] = (i + 2) % b if b > 2 else -1
            val[i, j, 0] = (j + 1) % nt
            val[i, j, 1] = (j + 2) % nt
    if device != "cpu":
        batch = {k: v.to(device) for k, v in batch.items()}
        noise = {k: v.to(device) for k, v in noise.items()}
    return batch, noise, ent, val


def gpu_parity_losses(tr, cfg, shape, bsz):
    """The HIP engine's eval-mode losses on the CPU baseline's first timed batch, from the oracle's starting weights
    (init_values(cfg, 0), the reference initialisation): the GPU half of the full-size parity field (VERDICT r5
    item 3; north_star "loss parity <= 1e-3 vs CPU reference").  Runs after the timed region on the bench's own
    engine (its trained weights are overwritten: the bench is done with them)."""
    import torch
    from k3m_amd.weights import init_values
    eng = tr.engine
    eng.fp.load(init_values(cfg, 0))
    batch, noise, ent, val = parity_inputs(cfg, shape, bsz, eng.fp.device)
    with torch.no_grad():
        out, _ = eng.forward(batch, train=False, noise=noise, ent_neg=ent, val_neg=val)
    torch.cuda.synchronize()
    return {k: float(out[k]) for k in PARITY_LOSSES}


def cpu_baseline(cfg, shape, bsz, steps, gpu_losses=None, bar=1e-3):
    """Oracle (torch CPU fp32) fwd+bwd+AdamW on a bounded sample of the same workload; baseline only.
    Threads: this process's CPU share on the GPU box (os.sched_getaffinity), not the machine's nproc
    (reported beside it).  One bs=8 warm-up step, a bs=8 sample (2 timed steps), then
    ``steps`` timed steps at ``bsz`` (the GPU workload's batch).  The bs=``bsz`` steps start from the initial weights
    (restored after the bs=8 steps), so the first one's forward is also the oracle half of the parity field: its five
    losses against ``gpu_losses`` (the engine on the same batch, weights, noise and negatives)."""
    import torch
    from oracle import k3m_oracle as O
    from k3m_amd.weights import init_values
    ncores, share = cpu_share()
    torch.set_num_threads(ncores)
    P = {k: torch.from_numpy(v).requires_grad_(True) for k, v in init_values(cfg, 0).items()}
    P0 = {k: v.detach().clone() for k, v in P.items()}
    state = {k: (torch.zeros_like(v), torch.zeros_like(v)) for k, v in P.items()}

    tstep = [0]
    first = {}

    def step(inp):
        tstep[0] += 1
        out = O.forward(P, cfg, *inp)
        if not first and inp[0]["input_ids"].shape[0] == bsz and tstep[0] == 1:
            first.update({k: float(out[k]) for k in PARITY_LOSSES})
        out["loss"].backward()
        with torch.no_grad():
            for k, p in P.items():
                if p.grad is None:
                    continue
                m, v = state[k]
                O.adamw_step(p.data, p.grad, m, v, tstep[0], 1e-4, 0.0 if ("bias" in k or "LayerNorm" in k) else 0.01)
                p.grad = None

    small = parity_inputs(cfg, shape, 8, "cpu")
    step(small)
    t0 = time.perf_counter()
    for _ in range(2):
        step(small)
    dt8 = time.perf_counter() - t0
    # back to the initial weights and a fresh optimizer for the timed bs=bsz steps (same work per step)
    with torch.no_grad():
        for k, p in P.items():
            p.copy_(P0[k])
            state[k][0].zero_()
            state[k][1].zero_()
    tstep[0] = 0
    big = parity_inputs(cfg, shape, bsz, "cpu") if bsz != 8 else small
    t0 = time.perf_counter()
    for _ in range(steps):
        step(big)
    dt = time.perf_counter() - t0
    res = {"value": round(bsz * steps / dt, 4), "unit": "samples/s", "cores": ncores, "kind": "port",
           "nproc": os.cpu_count(), "cpu_share": share, "cpu_model": cpu_model(),
           "bs8_samples_s": round(8 * 2 / dt8, 4),
           "sample": "oracle/k3m_oracle.py fwd+bwd+AdamW, fp32, bs=%d, %d timed step(s) (%.1f s) after a bs=8 warm-up; "
                     "bs=8: 2 timed steps %.1f s (same shapes as the GPU workload; torch CPU, %d threads = this "
                     "process's CPU share; the machine has %d).  Bounded sample: the bench contract asks for ~10-30 s "
                     "of CPU work so the default run ends in minutes, so bs=64 runs %d step(s), not SURVEY §8(d)'s 3 "
                     "after 1 warm-up (--cpu-steps 3 runs those)" % (bsz, steps, dt, dt8, ncores, os.cpu_count() or 0,
                                                                      steps)}
    parity = None
    if gpu_losses is not None and first:
        rel = {k: abs(gpu_losses[k] - first[k]) / max(abs(first[k]), 1e-3) for k in PARITY_LOSSES}
        parity = {"loss_gpu": {k: round(v, 7) for k, v in gpu_losses.items()},
                  "loss_oracle": {k: round(v, 7) for k, v in first.items()},
                  "rel": {k: float("%.3e" % v) for k, v in rel.items()},
                  "max_rel": float("%.3e" % max(rel.values())), "bar": bar, "pass": bool(max(rel.values()) <= bar),
                  "what": "eval-mode losses of the HIP engine vs the CPU oracle on the same bs=%d batch (seed 99), "
                          "initial weights init_values(cfg, 0), gumbel noise and LPM negatives; relative error per "
                          "loss (denominator max(|oracle|, 1e-3))" % bsz}
    return res, parity


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    shape = dict(CONFIGS[args.config])
    dtype = args.dtype or shape["dtype"]
    B = args.batch or shape["B"]
    dist = None
    use_dist = world > 1 or args.ddp
    if use_dist:
        import torch.distributed as dist
        if "WORLD_SIZE" not in os.environ:   # --ddp at one rank without a launcher
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(args.master_port or free_port()))
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
        from k3m_amd.ddp import GradAllReducer
    from k3m_amd.config import pretrain_config
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    from k3m_amd.engine import label_counts
    cfg = pretrain_config(os.path.join(HERE, "configs", "bert_base_6layer_6conect.json"))
    tr = Trainer(cfg, dev, lr=1e-4, warmup_steps=max(1, (args.steps + args.warmup) // 10),
                 total_steps=10 * (args.steps + args.warmup), seed=1234, init=True, dtype=dtype)
    if args.graph is not None:
        tr.graph = {"auto": "auto", "on": True, "off": False}[args.graph]
    if use_dist:
        ddp = GradAllReducer(tr.engine.fp, comm_dtype=torch.bfloat16 if dtype == "bf16" else None)
        ddp.broadcast_params(tr.engine.fp)
        tr.ddp = ddp
    batch = synthetic_batch(cfg, B, dev, seed=1234 + rank, T=shape["T"], P=shape["P"], n_boxes=shape["nbox"],
                            n_triples=shape["n_triples"], npv=shape["npv"])
    batch["_label_counts"] = label_counts(batch)   # known on the host when a loader builds the batch
    T, P, R = shape["T"], shape["P"], shape["nbox"] + 1
    rows = 2 * B * T + 2 * B * P   # the wide text buffer
    H, I = cfg.hidden_size, cfg.intermediate_size
    probe = GemmProbe(rows, I, H)   # FFN1 forward
    probe.install()
    # the dominant kernel by time: the weight-gradient walk; its launches of the text-layer weight gradients
    # (gW[n_out, n_in] += dY^T X over the 20,992 wide rows; FFN1's 3072 x 768 x 20,992 is the largest shape)
    wprobe = GemmProbe(I, H, rows, more=[(H, I, rows), (3 * H, H, rows), (H, H, rows)])
    wprobe.install()
    cprobe = CoattnProbe()
    cprobe.install()
    gall = GemmAllProbe()
    gall.install()

    def barrier():
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()

    # a repeated step may be replayed as one hipGraph (k3m_amd/graph.py): its first sighting runs eagerly, the
    # second is timed and the third decides (and captures): three untimed steps keep that out of the timed region
    warm = max(args.warmup, 3) if (tr.graph and not use_dist) else args.warmup
    for _ in range(warm):
        tr.step(batch)
    barrier()
    # host issue cost from an idle GPU (the timed loop's host time includes blocking on a full launch queue): two
    # more untimed steps before the timed region (so a profile's last steps are the timed ones)
    issue = []
    for _ in range(2):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        tr.step(batch)
        issue.append(time.perf_counter() - h0)
    barrier()
    # the GEMM / co-attention HIP-event probes bracket Python-issued launches: live in the timed region when the
    # step is issued eagerly; with graph replay (a captured launch cannot be bracketed by timing events) they
    # run in PROBE_STEPS eager steps right after it (same kernels, same shapes)
    graphed = tr.graph and tr._graphs is not None and tr._graphs.graph is not None
    probe.active = wprobe.active = cprobe.active = not graphed
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(args.steps):
        h0 = time.perf_counter()
        out = tr.step(batch)
        host += time.perf_counter() - h0
    barrier()
    dt = time.perf_counter() - t0
    loss = float(out["loss"])   # the last timed step's (a replay's outputs are overwritten by the next)
    probe.active = wprobe.active = cprobe.active = False
    per_rank = [dt]
    if use_dist:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        gl = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(gl, t)
        per_rank = [float(x) for x in gl]
        dt = max(per_rank)
    probe_steps = args.steps
    if graphed:
        probe_steps = PROBE_STEPS
        mode, tr.graph = tr.graph, False
        probe.active = wprobe.active = cprobe.active = True
        for _ in range(probe_steps):
            tr.step(batch)
        barrier()
        probe.active = wprobe.active = cprobe.active = False
        tr.graph = mode
    # every GEMM of one eager step, after the timed region (the per-launch events would perturb the timed steps)
    mode, tr.graph = tr.graph, False
    gall.active = True
    tr.step(batch)
    barrier()
    gall.active = False
    tr.graph = mode
    tr.finish()
    ms_step = 1000.0 * dt / args.steps
    value = world * B * args.steps / dt
    gemm_ms = probe.mean_ms()
    Mg, Ng, Kg = probe.key
    gemm_flops = 2.0 * Mg * Ng * Kg
    achieved = gemm_flops / (gemm_ms * 1e-3) if gemm_ms else None
    bf = dtype == "bf16"
    from k3m_amd import ops as _ops, _lib as _L
    x6 = not bf and _ops.F32_ALGO == _L.F32_SPLIT_BF16X6
    peak = PEAK_BF16_MFMA if bf else (PEAK_F32_X6 if x6 else PEAK_F32_MFMA)
    kname = head_kernel(bf) if (bf or x6) else "gemm_f32_kernel"
    traffic, traffic_src = pmc_traffic(probe.key, kname)
    wkname = head_wgrad_kernel(bf) if (bf or x6) else "gemm_f32_kernel"
    w_ms = wprobe.mean_ms()
    Mw, Nw, Kw = wprobe.key
    w_flops = 2.0 * Mw * Nw * Kw
    w_ach = w_flops / (w_ms * 1e-3) if w_ms else None
    w_traffic, w_traffic_src = pmc_traffic(wprobe.key, wkname)
    nw, w_tot_ms, w_tot_flops = wprobe.aggregate()
    ref_sample = 3.0 * ref_fwd_flops(T, P, R, shape["n_triples"])
    co_flops = 3.0 * coattn_fwd_flops(T, P, R) * B
    co_ms = cprobe.total_ms() / probe_steps if cprobe.events else None
    res = {
        "metric": BASELINE_METRIC,
        "value": round(value, 3), "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": warm,
        "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": dtype, "data": "synthetic (SURVEY §8(d): random token ids, %dx2048 region feats, %d PV triples)" % (
            shape["nbox"], shape["n_triples"]),
        "config": {"workload": "config %d: bert_base_6layer_6conect %s bs=%d/GPU T=%d P=%d R=%d %d triples" % (
                       args.config, "bf16 encoder (fp32 master weights, heads, AdamW)" if bf else "fp32", B, T, P, R,
                       shape["n_triples"]),
                   "model": "bert_base_6layer_6conect", "global_batch": B * world, "seq_len": T,
                   "parallelism": "dp%d" % world},
        "per_gpu_samples_s": round(value / world, 3),
        # host time to issue one step (Python engine + launches; the GPU runs behind it): when this
        # approaches ms_per_step the step is launch-bound and the GPU idles between kernels
        "host_ms_per_step": round(1000.0 * host / args.steps, 3),
        # the same, each step issued from an idle GPU (two extra untimed steps): the Python engine's own cost
        "host_issue_ms": round(1000.0 * min(issue), 3),
        # the step's issue mode: K3M_GRAPH auto replays a hipGraph when the eager issue time is a large share of
        # the GPU time (decision: the measured eager step); captures / replays count graph launches
        "graph": ({"captures": tr._graphs.captures, "replays": tr._graphs.replays,
                   "decision": tr._graphs.last_decision} if tr._graphs is not None else None),
        "loss": round(loss, 4),
        "step_mfma_frac_vs_ref_flops": round(B * ref_sample / (ms_step * 1e-3) / peak, 4),
        # the dominant kernel by time (profiles/r5e/cfg2/step_split.txt: the 256x256 weight-gradient walk, 21 % of the
        # fp32 step; the bf16 step's largest class likewise), measured on its largest launch shape: the FFN1 weight
        # gradient, 12 launches per step
        "roofline": {"bound": "mfma", "kernel": "%s, FFN1 weight gradient %dx%dx%d (split-K, tn)" % (wkname, Mw, Nw, Kw),
                     "achieved": round(w_ach / 1e12, 2) if w_ach else None,
                     "peak": peak / 1e12, "unit": "TFLOP/s",
                     "frac": round(w_ach / peak, 4) if w_ach else None,
                     "traffic": w_traffic,
                     "avg_launch_ms": round(w_ms, 4) if w_ms else None,
                     "launches": len(wprobe.launches(wprobe.key)),
                     "probe": "HIP events, %s" % ("%d eager steps after the timed graph replays" % probe_steps if graphed
                                                  else "timed region"),
                     "algorithmic_flops_per_launch": w_flops,
                     "peak_basis": ("bf16 dense MFMA" if bf else "fp32 via 6 bf16 MFMA partial products = bf16 dense "
                                    "peak / 6" if x6 else "f32 MFMA"),
                     "traffic_unit": "HBM bytes/launch (rocprofv3 PMC, %s)" % w_traffic_src if w_traffic else None,
                     # every text-layer weight gradient on this kernel (QKV, attention output, FFN1, FFN2 x 12 layers)
                     "class": {"launches": nw, "ms_per_step": round(w_tot_ms / probe_steps, 3) if nw else None,
                               "achieved": round(w_tot_flops / (w_tot_ms * 1e-3) / 1e12, 2) if nw else None,
                               "frac": round(w_tot_flops / (w_tot_ms * 1e-3) / peak, 4) if nw else None}},
        # the FFN1 forward (bias + GELU epilogue), the roofline line of rounds 1-5
        "roofline_ffn1": {"bound": "mfma", "kernel": "%s text-layer FFN1 %dx%dx%d" % (kname, Mg, Ng, Kg),
                          "achieved": round(achieved / 1e12, 2) if achieved else None,
                          "peak": peak / 1e12, "unit": "TFLOP/s",
                          "frac": round(achieved / peak, 4) if achieved else None,
                          "traffic": traffic,
                          "avg_launch_ms": round(gemm_ms, 4) if gemm_ms else None,
                          "launches": len(probe.launches(probe.key)),
                          "algorithmic_flops_per_launch": gemm_flops,
                          "traffic_unit": "HBM bytes/launch (rocprofv3 PMC, %s)" % traffic_src if traffic else None},
        "gemm_all": gall.summary(peak),
        "coattn": {"ms_per_step": round(co_ms, 3) if co_ms else None,
                   "algorithmic_tflop_per_step": round(co_flops / 1e12, 3),
                   "achieved": round(co_flops / (co_ms * 1e-3) / 1e12, 2) if co_ms else None,
                   "frac": round(co_flops / (co_ms * 1e-3) / peak, 4) if co_ms else None,
                   "scope": "18 co-attention layers fwd+bwd (lock-step blocks incl. attention and LayerNorm)"},
    }
    if use_dist:
        res["per_rank_s"] = [round(x, 4) for x in per_rank]
        res["backend"] = args.backend
        res["world_size_seen"] = dist.get_world_size()
        tm = tr.ddp.timing(last=args.steps)
        if tm is not None:
            # rank 0's view: end of its last all-reduce minus end of its backward, averaged over the timed
            # steps (0 = fully hidden behind the backward); busy = time the comm stream spent in buckets
            res["allreduce_exposed_ms"] = round(tm["allreduce_exposed_ms"], 3)
            res["allreduce_busy_ms"] = round(tm["allreduce_busy_ms"], 3)
            res["allreduce_buckets_per_step"] = tm["buckets_per_step"]
            res["allreduce_dtype"] = tm["comm_dtype"]
            res["grad_bytes_per_rank"] = int(sum(b - a for blk in tr.ddp.blocks.values() for a, b in blk) *
                                             (2 if tm["comm_dtype"] == "bf16" else 4))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            gl = gpu_parity_losses(tr, cfg, shape, args.cpu_batch)
        except Exception as e:  # noqa: BLE001 - reported, never masks the GPU result
            gl = None
            res["parity"] = {"error": repr(e)}
        try:
            # fp32: the north-star bar 1e-3; the bf16 encoder: the bar of the bf16 goldens (tests/test_gpu_parity.py)
            res["cpu_baseline"], par = cpu_baseline(cfg, shape, args.cpu_batch, args.cpu_steps, gl,
                                                    bar=7e-3 if bf else 1e-3)
            if par is not None:
                res["parity"] = par
        except Exception as e:  # baseline only; never masks the GPU result
            res["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    elif world > 1:
        print("rank %d/%d: %.3f samples/s/GPU (%.1f ms/step)" % (rank, world, B * args.steps / per_rank[rank],
                                                                1000.0 * per_rank[rank] / args.steps),
              file=sys.stderr, flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

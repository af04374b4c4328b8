"""Benchmark: batched 10-NN QPS on MI355X (BASELINE.json metric).

Default workload (configs[1] of BASELINE.json): exact brute-force 10-NN over a
1M x 128-d L2Squared corpus with a 10k-query batch -- recall@10 = 1.0 by
construction and ids identical to the reference distancer path.  A "step" is
one batch of queries searched over the whole corpus.

N GPUs (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
the corpus is sharded by contiguous id range over the ranks (local top-k per
shard), the per-shard (dist, id) lists are all-gathered over RCCL/xGMI and
merged on every rank (index.go:967-1044 restated on device).  Total work is
fixed, so scaling is "strong"; value = queries/s over the whole corpus.

--workload hnsw (BASELINE configs[0]): beam search over a graph built by the
CPU restatement (oracle/, test infrastructure; --graph-build gpu builds it
with wv_index_build_graph instead) on SIFT-shaped data; reports QPS and
recall@10 next to the restatement's on the same graph.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "batched 10-NN QPS at recall@10≥0.95, 1M×128-d L2, on 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_MFMA_PEAK_TF = 157.3    # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_MFMA_PEAK_TF = 2500.0   # MI355X_MICROARCH.md: bf16 dense MFMA peak (no sparsity)
F16_MFMA_PEAK_TF = 2500.0    # MI355X_MICROARCH.md: f16 MFMA runs at the bf16 rate (same cycles per instruction)
# measured on the box: a bare f16 MFMA loop (operands in registers, 64x64 per
# wave, two waves per SIMD, random data) at the clock the chip holds under it
# (tools/mfma_shape_bench.cpp, profiles/r02_mfma_shape_bench.log)
F16_MFMA_BARE_LOOP_TF = {"32x32x16": 1670.0, "16x16x32": 1920.0}


def _par_rows(fn, seed: int, row0: int, nrows: int, dim: int, chunk: int = 1 << 16) -> np.ndarray:
    """fn(seed, row0, nrows, dim) over row chunks on a thread pool (numpy
    releases the GIL in its ufuncs); rows are independent, so the result is
    the same array as one call."""
    if nrows <= chunk:
        return fn(seed, row0, nrows, dim)
    from concurrent.futures import ThreadPoolExecutor
    out = np.empty((nrows, dim), np.float32)

    def one(r0):
        r1 = min(nrows, r0 + chunk)
        out[r0:r1] = fn(seed, row0 + r0, r1 - r0, dim)

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
        list(ex.map(one, range(0, nrows, chunk)))
    return out


def counter_uniform(seed: int, row0: int, nrows: int, dim: int) -> np.ndarray:
    """Counter-based U[0,1) float32: value(row, col) depends only on (seed, row,
    col), so every rank can generate exactly its own rows of the corpus."""
    if nrows > (1 << 16):
        return _par_rows(counter_uniform, seed, row0, nrows, dim)
    out = np.empty((nrows, dim), np.float32)
    chunk = max(1, (1 << 22) // dim)
    cols = np.arange(dim, dtype=np.uint64)
    for r0 in range(0, nrows, chunk):
        r1 = min(nrows, r0 + chunk)
        rows = np.arange(row0 + r0, row0 + r1, dtype=np.uint64)[:, None]
        x = rows * np.uint64(dim) + cols[None, :]
        x = x * np.uint64(0x9E3779B97F4A7C15) + np.uint64((seed * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF)
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
        out[r0:r1] = (x >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24))
    return out


def counter_gauss(seed: int, row0: int, nrows: int, dim: int) -> np.ndarray:
    """N(0,1)/sqrt(dim) float32 by Box-Muller over two counter-based streams
    (GloVe / Deep / C4-shaped data)."""
    if nrows > (1 << 16):
        return _par_rows(counter_gauss, seed, row0, nrows, dim)
    u1 = counter_uniform(seed, row0, nrows, dim).astype(np.float64)
    u2 = counter_uniform(seed + 1000, row0, nrows, dim).astype(np.float64)
    z = np.sqrt(-2.0 * np.log(u1 + 2.0 ** -25)) * np.cos(2.0 * np.pi * u2)
    return (z / np.sqrt(dim)).astype(np.float32)


def counter_sift(seed: int, row0: int, nrows: int, dim: int) -> np.ndarray:
    """SIFT-shaped data (BASELINE configs[0]): non-negative integer-valued
    features with low intrinsic dimension -- 1024 cluster centres plus a
    24-d latent spread and a little isotropic noise, rounded and clipped at 0
    (SIFT descriptors are small non-negative integers).  Corpus and queries
    share the centres and the latent basis; everything else is counter-based
    per row like counter_uniform.  Uniform 128-d data has intrinsic dimension
    128 and no HNSW operating point near recall 0.95 at ef=64; this does
    (about 0.99 at 100k rows)."""
    if nrows > (1 << 16):
        return _par_rows(counter_sift, seed, row0, nrows, dim)
    C, L = 1024, 24
    centres = counter_uniform(77, 0, C, dim) * np.float32(60.0)
    basis = counter_gauss(78, 0, dim, L) * np.float32(np.sqrt(L))
    cid = (counter_uniform(seed + 2000, row0, nrows, 1)[:, 0] * C).astype(np.int64)
    z = counter_gauss(seed + 3000, row0, nrows, L) * np.float32(np.sqrt(L))
    e = counter_gauss(seed + 4000, row0, nrows, dim) * np.float32(np.sqrt(dim))
    x = centres[cid] + (z @ basis.T) * np.float32(12.0) + e * np.float32(3.0)
    return np.maximum(np.rint(x), 0).astype(np.float32)


GLOVE_DESC = ("GloVe-100-shaped (4096 Zipf-weighted clusters in a 24-d latent family + full-rank noise, "
              "log-normal row norms before the cosine normalisation)")


def counter_glove(seed: int, row0: int, nrows: int, dim: int) -> np.ndarray:
    """GloVe-100-shaped data (BASELINE configs[2]): word vectors are
    clustered with heavily skewed cluster sizes (word frequency), live near a
    low-dimensional family of directions, keep a sizeable full-rank residual,
    and have heavy-tailed norms -- which the cosine distancer normalises away
    (insert.go:56-60), so only the directions matter for the search.  I.i.d.
    Gaussians (round 1's C3 data) have none of this structure and no HNSW
    operating point (recall@10 0.15-0.39 for ef 32-256); this data has one in
    the reference's range.  Counter-based per row like counter_uniform."""
    if nrows > (1 << 16):
        return _par_rows(counter_glove, seed, row0, nrows, dim)
    C, L = 4096, 24
    centres = counter_gauss(81, 0, C, L) * np.float32(np.sqrt(L))          # cluster centres in the latent space
    basis = counter_gauss(82, 0, dim, L) * np.float32(np.sqrt(L))          # latent -> ambient
    u = counter_uniform(seed + 2000, row0, nrows, 1)[:, 0].astype(np.float64)
    cid = np.minimum((C * u ** 3).astype(np.int64), C - 1)                 # Zipf-like cluster sizes
    z = centres[cid] + np.float32(0.55) * counter_gauss(seed + 3000, row0, nrows, L) * np.float32(np.sqrt(L))
    e = counter_gauss(seed + 4000, row0, nrows, dim) * np.float32(np.sqrt(dim))
    x = (z @ basis.T) / np.float32(np.sqrt(L)) + np.float32(GLOVE_NOISE) * e
    s = np.exp(np.float32(0.6) * counter_gauss(seed + 5000, row0, nrows, 1) * np.float32(1.0))
    return (x * s).astype(np.float32)


GLOVE_NOISE = 0.9   # measured: recall@10 0.87 / 0.94 / 0.97 / 0.99 at ef 32 / 64 / 128 / 256 (M=64, efC=128)


def parity_stats(gi, gd, oi, od):
    """ids position-equal / distances bitwise equal / identical up to the
    order among equal distances (the reference orders ties by heap layout,
    SURVEY 8c) -- fractions of queries."""
    id_eq = float((gi == oi).all(axis=1).mean())
    d_eq = float((gd.view(np.uint32) == od.view(np.uint32)).all(axis=1).mean())
    tie_ok = 0
    for a_i, a_d, b_i, b_d in zip(gi, gd, oi, od):
        ok = np.array_equal(a_d.view(np.uint32), b_d.view(np.uint32))
        if ok:
            for v in np.unique(a_d[:-1]):
                if v != a_d[-1] and set(a_i[a_d == v].tolist()) != set(b_i[b_d == v].tolist()):
                    ok = False
                    break
        tie_ok += ok
    return id_eq, d_eq, tie_ok / max(len(gi), 1)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N ranks (one process per GPU) as
    a child torch.distributed.run and return its exit code.  Runs before this
    process touches the GPU (nothing is exec'd)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


class Ctx:
    """One rank: its device, stream and the process group (if any)."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.ws, self.rank, self.local = dist_env()
        self.gpu = self.local % max(torch.cuda.device_count(), 1)
        self.gloo = self.ws > 1 and args.dist_backend == "gloo"
        if self.ws > 1:
            if self.gloo:
                dist.init_process_group(backend="gloo")
            else:
                dist.init_process_group(backend="nccl", device_id=torch.device("cuda", self.gpu))
        torch.cuda.set_device(self.gpu)
        self.dev = torch.device("cuda", self.gpu)
        # one real stream for everything this rank queues (torch ops and the
        # library's device batches): the default stream's handle is 0, which
        # the C ABI reads as "the index's own stream"
        self.stream_obj = torch.cuda.Stream(self.dev)
        torch.cuda.set_stream(self.stream_obj)
        self.stream = self.stream_obj.cuda_stream
        self.n_devices = self.ws
        if self.ws > 1:   # distinct devices behind the ranks (a gloo rehearsal may share one)
            t = torch.tensor([self.gpu], dtype=torch.int64)
            parts = [torch.zeros(1, dtype=torch.int64) for _ in range(self.ws)]
            if self.gloo:
                dist.all_gather(parts, t)
            else:
                tt = t.to(self.dev)
                pp = [p.to(self.dev) for p in parts]
                dist.all_gather(pp, tt)
                parts = [p.cpu() for p in pp]
            self.n_devices = len({int(p.item()) for p in parts})

    def barrier(self):
        if self.ws > 1:
            self.dist.barrier()

    def per_rank(self, x: int) -> list:
        """x from every rank, in rank order (a collective: every rank calls it)"""
        if self.ws == 1:
            return [int(x)]
        torch = self.torch
        t = torch.tensor([int(x)], dtype=torch.int64, device="cpu" if self.gloo else self.dev)
        parts = [torch.zeros_like(t) for _ in range(self.ws)]
        self.dist.all_gather(parts, t)
        return [int(p.item()) for p in parts]

    def info(self) -> dict:
        """what the first multi-GPU run must be checked against line by line:
        the backend (torch "nccl" = RCCL on ROCm), the world it saw, the
        devices behind the ranks"""
        d = {"world_size": self.ws, "distinct_devices": self.n_devices, "rank0_device": self.gpu}
        if self.ws > 1:
            d["backend"] = str(self.dist.get_backend())
            d["uses_rccl"] = d["backend"] == "nccl"
            d["process_group_size"] = self.dist.get_world_size()
            try:
                d["rccl_version"] = ".".join(str(v) for v in self.torch.cuda.nccl.version())
            except Exception as e:  # (informational)
                d["rccl_version"] = f"unavailable: {type(e).__name__}"
        else:
            d["uses_rccl"] = False
        return d

    def max_over_ranks(self, x: float) -> float:
        if self.ws == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device="cpu" if self.gloo else self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def time_steps(self, step, steps, warmup, before_timed=None):
        """W untimed steps, then exactly K steps bracketed by barrier +
        synchronize on both sides; the max over ranks (bench contract).
        before_timed runs after the warmup, outside the timed region."""
        torch = self.torch
        for _ in range(warmup):
            step(False)
        torch.cuda.synchronize(self.dev)
        if before_timed:
            before_timed()
        self.barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step(True)
        torch.cuda.synchronize(self.dev)
        self.barrier()
        torch.cuda.synchronize(self.dev)
        return self.max_over_ranks(time.perf_counter() - t0)

    def allgather(self, out, t):
        """[ws, ...] all-gather of a device tensor: RCCL over xGMI (product),
        or through host memory for a gloo rehearsal."""
        if self.gloo:
            parts = [self.torch.empty_like(t, device="cpu") for _ in range(self.ws)]
            self.dist.all_gather(parts, t.cpu())
            out.copy_(self.torch.stack(parts).to(self.dev))
        else:
            self.dist.all_gather_into_tensor(out, t)


def _query_tensor(ctx, queries, dpad):
    torch = ctx.torch
    qt = torch.zeros((queries.shape[0], dpad), dtype=torch.float32, device=ctx.dev)
    qt[:, : queries.shape[1]] = torch.from_numpy(queries).to(ctx.dev)
    return qt


def _out_tensors(ctx, nq, k):
    torch = ctx.torch
    return (torch.empty((nq, k), dtype=torch.int64, device=ctx.dev), torch.empty((nq, k), dtype=torch.float32,
            device=ctx.dev), torch.empty((nq,), dtype=torch.int32, device=ctx.dev))


def _allow_words(args, lo, n_local):
    keep = counter_uniform(3, lo, n_local, 1)[:, 0] < args.allow_frac
    words = np.zeros((n_local + 63) // 64, np.uint64)
    idx = np.nonzero(keep)[0].astype(np.uint64)
    np.bitwise_or.at(words, (idx >> np.uint64(6)).astype(np.int64), np.uint64(1) << (idx & np.uint64(63)))
    return words, int(keep.sum())


def device_rows(ctx, kind, seed, row0, n, dim):
    """rows [row0, row0 + n) of a counter-based corpus generated on the device
    (tools/wv_synth.hip; measurement infrastructure)"""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth
    t = ctx.torch.empty((n, dim), dtype=ctx.torch.float32, device=ctx.dev)
    synth.fill(kind, seed, row0, t, stream=ctx.stream)
    return t


def upload_device_rows(ctx, ix, kind, seed, row0, n, dim, chunk=1 << 23, host_copy=False):
    """the index's rows [0, n) = corpus rows [row0, row0 + n), generated on the
    device chunk by chunk and uploaded from device memory; host_copy: also
    returned as a host array (for the CPU restatement)"""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import synth
    torch = ctx.torch
    host = np.empty((n, dim), np.float32) if host_copy else None
    chunk = max(1, min(chunk, (1 << 31) // (4 * dim)))
    t = torch.empty((min(n, chunk), dim), dtype=torch.float32, device=ctx.dev)
    for r0 in range(0, n, chunk):
        m = min(chunk, n - r0)
        synth.fill(kind, seed, row0 + r0, t[:m], stream=ctx.stream)
        torch.cuda.synchronize(ctx.dev)
        ix.upload_vectors_device(t.data_ptr(), m, first_id=r0)
        if host is not None:
            host[r0:r0 + m] = t[:m].cpu().numpy()
    del t
    torch.cuda.empty_cache()
    return host


_PHASE = ["start", time.time()]


def phase(name: str):
    """the bench's current phase, echoed to stderr (and every 30 s by the
    heartbeat: long silent phases -- a 100M-row graph build -- stay visible)"""
    _PHASE[0], _PHASE[1] = name, time.time()
    print(f"[bench] {name}", file=sys.stderr, flush=True)


def _heartbeat():
    import threading

    def run():
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"[bench] ... {_PHASE[0]} ({time.time() - _PHASE[1]:.0f} s in phase, {time.time() - t0:.0f} s total)",
                  file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O  # the checker / CPU baseline (test infrastructure), never the measured path
    return O


def exact_roofline(args, ix, kern_ms, stats, D, n_allowed, n_local, NQ):
    mfma_ms = float(np.mean([k["bf_mfma_ms"] for k in kern_ms]))
    seed_ms = float(np.mean([k.get("seed_ms", 0.0) for k in kern_ms]))
    flops = 2.0 * D * n_allowed * NQ    # algorithmic: 2*D*N_eff per query
    achieved = flops / (mfma_ms * 1e-3) / 1e12
    # Which key pass ran (wv_api.hip run_exact): the f16 pass (default, D <= 1024;
    # wv_bf_h16w_kernel above D = 128,
    # one v_mfma_f32_32x32x16_f16 product per fp32 product: peak = the dense
    # f16 MFMA rate), the bf16x3 split pass (WV_BF_SPLIT=1: 3 bf16 products per
    # fp32 product, peak = bf16 dense / 3) or the fp32 MFMA pass (WV_BF_FP32=1,
    # D > 1024, or a shared allow list compacted into a row list).
    fp32 = bool(os.environ.get("WV_BF_FP32")) or D > 1024
    if os.environ.get("WV_BF_SPLIT") and not fp32:
        kind = "split" if 2 * n_allowed >= n_local else "fp32"
    elif not fp32:
        # round 3: a shared list under half the corpus runs the f16 pass over
        # its gathered rows
        kind = "h16"
    else:
        kind = "fp32"
    peak, kname, kp = {"h16": (F16_MFMA_PEAK_TF, "wv_bf_h16w_kernel" if D > 128 else "wv_bf_h16_kernel",
                               "f16 MFMA keys (32x32x16; peak = f16 dense)"),
                       "split": (BF16_MFMA_PEAK_TF / 3, "wv_bf_split_kernel", "bf16x3 (peak = bf16 dense / 3)"),
                       "fp32": (FP32_MFMA_PEAK_TF, "wv_bf_mfma_kernel", "fp32 MFMA")}[kind]
    roof = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 2), "peak": round(peak, 1),
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": None, "key_pass": kp,
            "frac_of_fp32_mfma_peak": round(achieved / FP32_MFMA_PEAK_TF, 4), "kernel_ms": round(mfma_ms, 3),
            "finalize_ms": round(float(np.mean([k["bf_finalize_ms"] for k in kern_ms])), 3),
            "fallback_queries": stats["fallbacks"]}
    if kind == "h16":
        roof["frac_of_bare_mfma_loop"] = round(achieved / F16_MFMA_BARE_LOOP_TF["32x32x16"], 4)
        roof["bare_mfma_loop_tf"] = F16_MFMA_BARE_LOOP_TF["32x32x16"]
        roof["seed_pass_ms"] = round(seed_ms, 3)
        roof["achieved_incl_seed_pass"] = round(flops / ((mfma_ms + seed_ms) * 1e-3) / 1e12, 2)
    return roof, kind


def attach_traffic(roof, n_local, NQ, D, data, allow_frac=None):
    """roofline.traffic from a committed PMC summary -- only one collected from
    this build of the key pass (tools/build_hash.py) on the same shape"""
    import glob
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from build_hash import build_hash
    want = build_hash(roof["kernel"])
    # profiles/pmc_<kernel>.json and pmc_<kernel>_<shape>.json: the one of this shape
    for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_%s*.json" % roof["kernel"]))):
        with open(pmc) as f:
            p = json.load(f)
        if p.get("kernel") != roof["kernel"]:
            continue
        same_shape = (p.get("N"), p.get("nq"), p.get("dim"), p.get("data", "uniform"), p.get("allow_frac")) == \
            (n_local, NQ, D, data, allow_frac)
        if same_shape and p.get("build") == want:
            roof["traffic"] = p.get("hbm_bytes_per_launch")
            roof["traffic_source"] = p.get("source", os.path.relpath(pmc, ROOT))
            for key in ("per_mfma", "effective_clock_ghz", "mfma_busy_frac", "wait_inst_frac"):
                if key in p:
                    roof["pmc_" + key] = p[key]
            roof.pop("traffic_note", None)
            return
        if same_shape:
            roof["traffic_note"] = "profiles/%s is from another build (%s); not attached" % (
                os.path.basename(pmc), p.get("build"))


def run_exact(args, ctx, W):
    """configs[1]: exact 10-NN (flatSearch semantics) over the whole corpus.
    query split (default at N > 1): every rank holds the corpus and answers its
    own nq-query batch -- queries are independent units, no collective (weak
    scaling).  corpus split: rank r owns ids [r N/W, (r+1) N/W), all ranks take
    the same batch, the per-shard top-k are all-gathered over RCCL and merged
    on the device (index.go:967-1044; strong scaling)."""
    torch = ctx.torch
    N, D, NQ, K = args.rows, args.dim, args.nq, args.k
    ws, rank = ctx.ws, ctx.rank
    split = args.split
    gen = {"uniform": counter_uniform, "gauss": counter_gauss, "sift": counter_sift, "glove": counter_glove}[args.data]
    lo, hi = (N * rank // ws, N * (rank + 1) // ws) if split == "corpus" else (0, N)
    n_local = hi - lo
    base = gen(1, lo, n_local, D)
    q_row0 = rank * NQ if split == "query" else 0
    queries = gen(2, q_row0, NQ, D)
    ix = W.GPUVectorIndex(D, args.metric, capacity=max(n_local, 1), device=ctx.gpu, id_base=lo)
    ix.upload_vectors(base)
    dpad = ix.query_ld()
    qt = _query_tensor(ctx, queries, dpad)
    out_ids, out_d, out_n = _out_tensors(ctx, NQ, K)
    if split == "corpus" and ws > 1:
        g_ids = torch.empty((ws, NQ, K), dtype=torch.int64, device=ctx.dev)
        g_d = torch.empty((ws, NQ, K), dtype=torch.float32, device=ctx.dev)
        g_n = torch.empty((ws, NQ), dtype=torch.int32, device=ctx.dev)
        m_ids, m_d, m_n = _out_tensors(ctx, NQ, K)
    allow_ptr, allow_bits, n_allowed, words = 0, 0, n_local, None
    if args.allow_frac > 0:
        words, n_allowed = _allow_words(args, lo, n_local)
        allow_t = torch.from_numpy(words.view(np.int64)).to(ctx.dev)
        allow_ptr, allow_bits = allow_t.data_ptr(), n_local
    kern_ms = []

    # no host round trip inside the timed region: the kernel times (HIP
    # events per batch) and the batch stats are read after it
    def step(timed):
        ix.search_batch_device(qt.data_ptr(), NQ, K, out_ids.data_ptr(), out_d.data_ptr(), out_n.data_ptr(), ef=0,
                               mode="exact", stream=ctx.stream, allow_ptr=allow_ptr, allow_nbits=allow_bits)
        if split == "corpus" and ws > 1:
            ctx.allgather(g_ids, out_ids)
            ctx.allgather(g_d, out_d)
            ctx.allgather(g_n, out_n)
            W.merge_shards_device(g_d.data_ptr(), g_ids.data_ptr(), g_n.data_ptr(), ws, NQ, K, m_d.data_ptr(),
                                  m_ids.data_ptr(), m_n.data_ptr(), stream=ctx.stream)

    ix.set_timing(True)
    elapsed = ctx.time_steps(step, args.steps, args.warmup, before_timed=ix.last_kernel_times)
    kern_ms.append(ix.last_kernel_times())   # per-batch averages over the timed steps
    stats = ix.last_batch_stats()
    fin_ids, fin_d = (m_ids, m_d) if (split == "corpus" and ws > 1) else (out_ids, out_d)
    final_ids = fin_ids.cpu().numpy().view(np.uint64)
    final_d = fin_d.cpu().numpy()
    units = NQ * (ws if split == "query" else 1)
    res = {
        "value": round(units * args.steps / elapsed, 1),
        "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "scaling": "weak" if split == "query" else "strong",
        "workload": ("exact brute-force %d-NN, %s x %d-d %s, %d-query batch%s"
                     % (K, f"{N:,}", D, args.metric, NQ,
                        (" (BASELINE configs[1])" if (N, D, args.metric) == (1_000_000, 128, "l2-squared") else "")
                        if args.allow_frac <= 0 else
                        f", shared allow list p={args.allow_frac} ({n_allowed:,} rows on rank 0)")),
        "parallelism": {"query": f"{ws} GPU(s), each holding the whole corpus and answering its own {NQ}-query "
                                 f"batch (no collective)",
                        "corpus": f"corpus sharded over {ws} GPU(s) by id range" + (
                            ", RCCL all-gather of per-shard top-k + device merge" if ws > 1 else "")}[split],
    }
    roof, kind = exact_roofline(args, ix, kern_ms, stats, D, n_allowed, n_local, NQ)
    attach_traffic(roof, n_local, NQ, D, args.data)
    res["roofline"] = roof
    res["dtype"] = {"h16": "f32 (f16 MFMA keys certified by an error bound, f32 reference-order re-rank)",
                    "split": "f32 (bf16x3 MFMA keys, f32 re-rank)", "fp32": "f32"}[kind]
    state = dict(ix=ix, base=base, queries=queries, final_ids=final_ids, final_d=final_d, words=words,
                 n_allowed=n_allowed, lo=lo, n_local=n_local)
    return res, state


def c4_line(args, ctx, W, with_cpu):
    """configs[3]: 10M x 768-d dot product, exact (flatSearch) 10-NN of a
    1000-query batch under a shared allow list kept at 100 / 50 / 10 / 1 %
    (Bernoulli over ids, seed 3) -- the corpus sharded over the N GPUs by id
    range, the per-shard top-k all-gathered over RCCL and merged on the device
    (index.go:967-1044, flat_search.go:19-74).  Rows generated on the device
    (N(0,1)/sqrt(768), tools/wv_synth.hip).  The reference would take the
    filtered HNSW path at 1 % of 10M (100k > flatSearchCutoff 40k,
    search.go:74-78); this line is the exact search (cutoff above |allow|)."""
    torch = ctx.torch
    N, D, NQ, K = args.c4_rows, 768, args.c4_nq, args.k
    ws, rank = ctx.ws, ctx.rank
    lo, hi = N * rank // ws, N * (rank + 1) // ws
    n_local = hi - lo
    t0 = time.time()
    ix = W.GPUVectorIndex(D, "dot", capacity=n_local, device=ctx.gpu, id_base=lo)
    base = upload_device_rows(ctx, ix, "gauss", 1, lo, n_local, D, host_copy=with_cpu)
    queries = device_rows(ctx, "gauss", 2, 0, NQ, D).cpu().numpy()
    qt = _query_tensor(ctx, queries, ix.query_ld())
    setup_s = time.time() - t0
    out_ids, out_d, out_n = _out_tensors(ctx, NQ, K)
    if ws > 1:
        g_ids = torch.empty((ws, NQ, K), dtype=torch.int64, device=ctx.dev)
        g_d = torch.empty((ws, NQ, K), dtype=torch.float32, device=ctx.dev)
        g_n = torch.empty((ws, NQ), dtype=torch.int32, device=ctx.dev)
        m_ids, m_d, m_n = _out_tensors(ctx, NQ, K)
    O = _oracle() if with_cpu else None
    legs = {}
    for frac in args.c4_fracs:
        a = argparse.Namespace(**vars(args))
        a.allow_frac = frac
        allow_ptr, allow_bits, n_allowed, words = 0, 0, n_local, None
        if frac < 1.0:
            words, n_allowed = _allow_words(a, lo, n_local)
            allow_t = torch.from_numpy(words.view(np.int64)).to(ctx.dev)
            allow_ptr, allow_bits = allow_t.data_ptr(), n_local

        def step(timed):
            ix.search_batch_device(qt.data_ptr(), NQ, K, out_ids.data_ptr(), out_d.data_ptr(), out_n.data_ptr(),
                                   ef=0, mode="exact", stream=ctx.stream, allow_ptr=allow_ptr,
                                   allow_nbits=allow_bits)
            if ws > 1:
                ctx.allgather(g_ids, out_ids)
                ctx.allgather(g_d, out_d)
                ctx.allgather(g_n, out_n)
                W.merge_shards_device(g_d.data_ptr(), g_ids.data_ptr(), g_n.data_ptr(), ws, NQ, K, m_d.data_ptr(),
                                      m_ids.data_ptr(), m_n.data_ptr(), stream=ctx.stream)

        ix.set_timing(True)
        el = ctx.time_steps(step, args.steps, args.warmup, before_timed=ix.last_kernel_times)
        km = ix.last_kernel_times()
        stats = ix.last_batch_stats()
        ix.set_timing(False)
        roof, kind = exact_roofline(a, ix, [km], stats, D, n_allowed, n_local, NQ)
        attach_traffic(roof, n_local, NQ, D, "gauss" if frac >= 1.0 else f"gauss_allow{frac}")
        ms = 1000 * el / args.steps
        leg = {"value": round(NQ * args.steps / el, 1), "unit": "queries/s", "ms_per_step": round(ms, 3),
               "allowed_rows_rank0": int(n_allowed), "roofline": roof,
               "outside_key_pass_frac": round(max(0.0, 1.0 - roof["kernel_ms"] / ms), 3)}
        fin_ids, fin_d = (m_ids, m_d) if ws > 1 else (out_ids, out_d)
        if with_cpu:
            # flatSearch restated in C on the same rows and list (parity + baseline)
            cpu = {}
            for threads, secs in ((args.cpu_threads, args.c4_cpu_seconds), (1, args.c4_cpu_seconds_t1)):
                probe = max(1, min(8, threads))
                tp = time.perf_counter()
                O.flat_scan(O.DOT, base, queries[:probe], K, allow_bits=words, threads=threads)
                per_q = (time.perf_counter() - tp) / probe
                ns = int(min(NQ, max(probe, secs / max(per_q, 1e-9))))
                tp = time.perf_counter()
                oi, od, on = O.flat_scan(O.DOT, base, queries[:ns], K, allow_bits=words, threads=threads)
                cpu[threads] = (ns, time.perf_counter() - tp, oi, od)
            ns, ct, oi, od = cpu[args.cpu_threads]
            gi = fin_ids.cpu().numpy().view(np.uint64)[:ns]
            gd = fin_d.cpu().numpy()[:ns]
            id_eq, d_eq, tie_ok = parity_stats(gi, gd, oi, od)
            leg["parity_sample"] = {"queries": ns, "ids_and_dists_bit_identical": id_eq == 1.0 and d_eq == 1.0,
                                    "dists_bitwise_equal_frac": d_eq, "tie_aware_identical_frac": tie_ok}
            n1, t1 = cpu[1][0], cpu[1][1]
            leg["cpu_baseline"] = {"value": round(ns / ct, 2), "unit": "queries/s", "cores": args.cpu_threads,
                                   "kind": "port", "value_t1": round(n1 / t1, 2), "cores_t1": 1,
                                   "sample": f"{ns} (T={args.cpu_threads}) / {n1} (T=1) of the {NQ} queries over "
                                             f"the full {N:,}-row corpus and list; flatSearch restated in C (AVX2 "
                                             f"asm-order dot, oracle/)"}
        legs["allow_%g%%" % (100 * frac)] = leg
    ix.close()
    del base
    rows_per_rank = ctx.per_rank(n_local)
    return {"workload": f"exact {K}-NN, {N:,} x {D}-d dot, {NQ}-query batch, shared allow list (BASELINE configs[3])",
            "rows_per_rank": rows_per_rank,
            "parallelism": (f"corpus sharded over {ws} GPU(s) by id range ({n_local:,} rows per GPU), RCCL all-gather "
                            f"of per-shard top-k + device merge" if ws > 1 else "one GPU holding the whole corpus"),
            "scaling": "strong (fixed corpus and batch)", "setup_s": round(setup_s, 1),
            "data": "N(0,1)/sqrt(768) rows and queries generated on the device (counter-based, seeds 1 / 2)",
            "legs": legs}


def wide_k_line(args, ctx, st, W):
    """Secondary exact lines on the same index (N=1): k=100 through the batched
    wide path (search.go:90-158 asks limit 100 first), and SearchByVectorDistance
    (deepening from limit 100) on single queries over a flat allow list."""
    torch = ctx.torch
    ix, NQ = st["ix"], args.nq
    qt = _query_tensor(ctx, st["queries"], ix.query_ld())
    out = {}
    for k in (100,):
        oi, od, on = _out_tensors(ctx, NQ, k)
        ix.search_batch_device(qt.data_ptr(), NQ, k, oi.data_ptr(), od.data_ptr(), on.data_ptr(), mode="exact",
                               stream=ctx.stream)
        torch.cuda.synchronize(ctx.dev)
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            ix.search_batch_device(qt.data_ptr(), NQ, k, oi.data_ptr(), od.data_ptr(), on.data_ptr(), mode="exact",
                                   stream=ctx.stream)
        torch.cuda.synchronize(ctx.dev)
        dt = (time.perf_counter() - t0) / reps
        fb = ix.last_batch_stats()["fallbacks"] * reps   # the last batch's (all batches are the same)
        out[f"exact_k{k}"] = {"value": round(NQ / dt, 1), "unit": "queries/s", "ms_per_batch": round(1e3 * dt, 3),
                              "fallback_queries_per_batch": fb / reps, "nq": NQ}
        if k == 100:
            d100 = od.cpu().numpy()
    # SearchByVectorDistance: target = each query's 150th-nearest distance, so
    # the deepening runs two rounds (limit 100, then 1100).  The per-query
    # host loop (wv_search_by_vector_distance), the device batch
    # (wv_search_by_vector_distance_batch: every exact round one threshold
    # pass + sort) for one query and for 64, and T concurrent callers through
    # the micro-batcher (unfiltered on this graph-less index: flatSearch)
    n_local = st["n_local"]
    allow = W.AllowList.from_ids(np.arange(n_local, dtype=np.uint64), n_local)
    ix.update_user_config(flat_search_cutoff=n_local + 1)
    nt = 64
    o256 = _out_tensors(ctx, nt, 256)
    qsn = _query_tensor(ctx, st["queries"][:nt], ix.query_ld())
    ix.search_batch_device(qsn.data_ptr(), nt, 256, o256[0].data_ptr(), o256[1].data_ptr(), o256[2].data_ptr(),
                           mode="exact", stream=ctx.stream)
    targets = np.ascontiguousarray(o256[1].cpu().numpy()[:, 149])
    times, counts = [], []
    for i in range(4):
        t0 = time.perf_counter()
        ids, ds = ix.search_by_vector_distance(st["queries"][i], float(targets[i]), -1, allow=allow)
        times.append(time.perf_counter() - t0)
        counts.append(int(len(ids)))
    one = []
    for i in range(8):
        t0 = time.perf_counter()
        got1, _ = ix.search_by_vector_distance_batch(st["queries"][i:i + 1], targets[i:i + 1], -1, allow=allow,
                                                     cap=1024)
        one.append(time.perf_counter() - t0)
    same1 = all(ix.search_by_vector_distance(st["queries"][i], float(targets[i]), -1, allow=allow)[0].tolist() ==
                ix.search_by_vector_distance_batch(st["queries"][i:i + 1], targets[i:i + 1], -1, allow=allow,
                                                   cap=1024)[0][0][0].tolist() for i in range(4))
    ix.search_by_vector_distance_batch(st["queries"][:nt], targets, -1, allow=allow, cap=1024)
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        got, cnt = ix.search_by_vector_distance_batch(st["queries"][:nt], targets, -1, allow=allow, cap=1024)
    batch_s = (time.perf_counter() - t0) / reps
    ix.update_user_config(flat_search_cutoff=40000)
    out["search_by_vector_distance"] = {
        "ms_per_query": round(1e3 * float(np.median(one[1:])), 3),
        "ms_per_query_host_loop": round(1e3 * float(np.median(times[1:])), 3),
        "results_per_query": counts, "batch_equals_host_loop": bool(same1),
        "batch_64": {"ms_per_batch": round(1e3 * batch_s, 3), "queries_per_s": round(nt / batch_s, 1),
                     "mean_results": round(float(np.mean(cnt)), 1)},
        "note": "target = each query's 150th-nearest distance (rounds at limit 100 and 1100); flat allow list of "
                "every id; ms_per_query: one query per wv_search_by_vector_distance_batch call (device threshold "
                "pass + sort), ms_per_query_host_loop: the round-5 per-round host loop"}
    path = os.path.join(ROOT, "tests", "native", "libwvload.so")
    if args.concurrency and os.path.exists(path):
        import ctypes as C
        lib = C.CDLL(path)
        if hasattr(lib, "wvl_concurrent_distance"):
            lib.wvl_concurrent_distance.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                                    C.c_double, C.c_int, C.c_void_p]
            q = np.ascontiguousarray(st["queries"][:nt], dtype=np.float32)
            cc = {}
            for t in (1, 16, 64):
                r = np.zeros(7, np.float64)
                rc = lib.wvl_concurrent_distance(C.c_void_p(ix._h.value if hasattr(ix._h, "value") else ix._h),
                                                 q.ctypes.data, targets.ctypes.data, nt, q.shape[1], t, 1.5,
                                                 args.max_batch, r.ctypes.data)
                cc[str(t)] = {"error": f"status {rc}"} if rc else {
                    "value": round(r[0], 1), "unit": "queries/s", "p50_us": round(r[1], 1), "p99_us": round(r[2], 1),
                    "mean_batch": round(r[3], 1), "mean_results": round(r[6], 1)}
            out["search_by_vector_distance"]["concurrent_callers"] = cc
    return out


def exact_cpu_baseline(args, st, O):
    """flatSearch restated in C (AVX2 asm-order distancer), on a bounded
    sample of the same queries; T = --cpu-threads (GOMAXPROCS-equivalent) and
    T = 1.  The same pass is the parity sample."""
    K = args.k
    base, queries = st["base"], st["queries"]
    metric_id = O.METRICS[args.metric]
    if args.metric == "cosine-dot":   # stored vectors normalized on insert (insert.go:56-60), queries per search
        base = O.normalize_rows(base)
        queries = O.normalize_rows(queries)
    cpu_allow = st["words"]
    out = {}
    for threads, secs in ((args.cpu_threads, args.cpu_seconds), (1, args.cpu_seconds_t1)):
        probe = max(2, min(32, 2 * threads))
        t0 = time.perf_counter()
        O.flat_scan(metric_id, base, queries[:probe], K, allow_bits=cpu_allow, threads=threads)
        per_q = (time.perf_counter() - t0) / probe
        ns = int(min(args.nq, max(probe, secs / max(per_q, 1e-9))))
        t0 = time.perf_counter()
        oi, od, on = O.flat_scan(metric_id, base, queries[:ns], K, allow_bits=cpu_allow, threads=threads)
        out[threads] = (ns, time.perf_counter() - t0, oi, od)
    ns, cpu_t, oi, od = out[args.cpu_threads]
    id_eq, d_eq, tie_ok = parity_stats(st["final_ids"][:ns], st["final_d"][:ns], oi, od)
    parity = {"queries": ns, "ids_and_dists_bit_identical": id_eq == 1.0 and d_eq == 1.0,
              "dists_bitwise_equal_frac": d_eq, "tie_aware_identical_frac": tie_ok, "id_match_frac": id_eq}
    n1, t1 = out[1][0], out[1][1]
    base_line = {"value": round(ns / cpu_t, 1), "unit": "queries/s", "cores": args.cpu_threads, "kind": "port",
                 "host_cores": args.host_cores,
                 "value_t1": round(n1 / t1, 2), "cores_t1": 1,
                 "sample": f"{ns} (T={args.cpu_threads}) / {n1} (T=1) of the {args.nq} queries over the full "
                           f"{args.rows:,}-row corpus ({cpu_t:.2f} s / {t1:.2f} s); flatSearch restated in C "
                           f"(AVX2 asm-order distancer, oracle/), query-parallel like ssdhelpers.Concurrently, "
                           f"GOMAXPROCS-equivalent T={args.cpu_threads} and T=1"}
    return base_line, parity


def build_hnsw_graph(args, ctx, ix, base, n_local, O):
    """The configs[0] graph (M, efConstruction): on the GPU
    (wv_index_build_graph, insert.go in batches) or by the CPU restatement's
    sequential build (oracle/, test infrastructure)."""
    torch = ctx.torch
    cache = args.graph_cache % {"rank": ctx.rank} if args.graph_cache else ""
    t0 = time.time()
    if args.graph_build == "gpu":
        torch.cuda.synchronize(ctx.dev)
        ix.build_graph(ef_construction=args.efc, seed=1, batch_div=args.batch_div)
        torch.cuda.synchronize(ctx.dev)
        g = None
        src = f"built on the GPU (wv_index_build_graph, batch = inserted/{args.batch_div})"
    elif cache and os.path.exists(cache):
        z = np.load(cache)
        g = {k: (z[k] if z[k].ndim else int(z[k])) for k in z.files}
        ix.upload_graph(g)
        src = "loaded (cache) -- built earlier by the CPU restatement (oracle/)"
    else:
        import threading
        done = threading.Event()

        def progress():   # long CPU builds: keep the log moving
            while not done.wait(30):
                print(f"[bench] building hnsw graph over {n_local:,} rows: {time.time() - t0:.0f} s",
                      file=sys.stderr, flush=True)
        threading.Thread(target=progress, daemon=True).start()
        ref = O.Index(args.dim, args.metric, args.M, args.efc, capacity=n_local, seed=1)
        ref.add_batch(base, threads=args.hnsw_build_threads)
        done.set()
        g = ref.export_graph()
        if cache:
            np.savez(cache, **{k: np.asarray(v) for k, v in g.items()})
        ix.upload_graph(g)
        src = "built by the CPU restatement (oracle/)"
    return {"build_s": round(time.time() - t0, 2), "M": args.M, "efConstruction": args.efc, "source": src}


def run_hnsw(args, ctx, W, with_cpu):
    """configs[0] / configs[4]: hnsw beam search (knnSearchByVector) at ef.
    query split (default at N > 1 for 1M rows): every rank holds the whole
    graph and answers its own batch (weak scaling).  corpus split (the
    north-star layout, default for configs[4]-shaped runs): rank r owns ids
    [r N/W, (r+1) N/W) and the graph of those rows (built on its GPU), every
    rank searches the same batch over its shard graph, the per-shard top-k are
    all-gathered over RCCL and merged on the device (index.go:967-1044).
    Recall@10 against exact truths from the exact path (bit-identical to the
    restatement's flatSearch; sharded the same way); on rank 0 at N = 1 also
    the restatement's recall on the same graph and its CPU throughput."""
    torch = ctx.torch
    N, D, NQ, K = args.rows, args.dim, args.nq, args.k
    ws, rank = ctx.ws, ctx.rank
    corpus = args.split == "corpus" and ws > 1
    data = args.hnsw_data
    gen = {"uniform": counter_uniform, "gauss": counter_gauss, "sift": counter_sift, "glove": counter_glove}[data]
    lo, hi = (N * rank // ws, N * (rank + 1) // ws) if corpus else (0, N)
    n_local = hi - lo
    ix = W.GPUVectorIndex(D, args.metric, capacity=n_local, device=ctx.gpu, max_connections=args.M, id_base=lo)
    if getattr(args, "device_data", False):
        # configs[4]-sized shards: rows generated in HBM (tools/wv_synth.hip,
        # the same construction as the numpy generator) and uploaded from
        # there; the host never holds the corpus
        base = None
        queries = device_rows(ctx, data, 2, 0 if corpus else rank * NQ, NQ, D).cpu().numpy()
        upload_device_rows(ctx, ix, data, 1, lo, n_local, D)
    else:
        base = gen(1, lo, n_local, D)
        queries = gen(2, 0 if corpus else rank * NQ, NQ, D)
        ix.upload_vectors(base)
    O = _oracle() if (with_cpu or args.graph_build != "gpu") else None
    graph = build_hnsw_graph(args, ctx, ix, base, n_local, O)
    graph["max_level"] = int(ix.graph_info()["max_level"])
    dpad = ix.query_ld()
    qt = _query_tensor(ctx, queries, dpad)
    out_ids, out_d, out_n = _out_tensors(ctx, NQ, K)
    if corpus:
        g_ids = torch.empty((ws, NQ, K), dtype=torch.int64, device=ctx.dev)
        g_d = torch.empty((ws, NQ, K), dtype=torch.float32, device=ctx.dev)
        g_n = torch.empty((ws, NQ), dtype=torch.int32, device=ctx.dev)
        m_ids, m_d, m_n = _out_tensors(ctx, NQ, K)

    def merge():
        ctx.allgather(g_ids, out_ids)
        ctx.allgather(g_d, out_d)
        ctx.allgather(g_n, out_n)
        W.merge_shards_device(g_d.data_ptr(), g_ids.data_ptr(), g_n.data_ptr(), ws, NQ, K, m_d.data_ptr(),
                              m_ids.data_ptr(), m_n.data_ptr(), stream=ctx.stream)

    kern_ms, stats = [], []

    def step(timed):
        ix.search_batch_device(qt.data_ptr(), NQ, K, out_ids.data_ptr(), out_d.data_ptr(), out_n.data_ptr(),
                               ef=args.ef, mode="hnsw", stream=ctx.stream)
        if corpus:
            merge()

    ix.set_timing(True)
    elapsed = ctx.time_steps(step, args.steps, args.warmup, before_timed=ix.last_kernel_times)
    kern_ms.append(ix.last_kernel_times())   # per-batch averages over the timed steps
    stats.append(ix.last_batch_stats())
    fin = (m_ids, m_d) if corpus else (out_ids, out_d)
    hi_ids = fin[0].cpu().numpy().view(np.uint64).copy()
    hi_d = fin[1].cpu().numpy().copy()
    shard_ids = out_ids.cpu().numpy().view(np.uint64).copy()   # this rank's own shard answer
    shard_d = out_d.cpu().numpy().copy()
    # exact truths on the same queries (the exact path: ids bit-identical to
    # flatSearch; per shard + the same merge in the corpus layout), timed
    # once: SIFT-shaped data is integer-valued, so equal distances at the k
    # boundary send queries to the certificate's fallback
    ix.set_timing(False)
    torch.cuda.synchronize(ctx.dev)
    t0 = time.perf_counter()
    ix.search_batch_device(qt.data_ptr(), NQ, K, out_ids.data_ptr(), out_d.data_ptr(), out_n.data_ptr(), ef=0,
                           mode="exact", stream=ctx.stream)
    if corpus:
        merge()
    torch.cuda.synchronize(ctx.dev)
    exact_ms = 1000 * (time.perf_counter() - t0)
    exact_fb = ix.last_batch_stats()["fallbacks"]
    truth = (m_ids if corpus else out_ids).cpu().numpy().view(np.uint64)
    rec = float(np.mean([len(set(a) & set(b)) / K for a, b in zip(hi_ids.tolist(), truth.tolist())]))

    def recall_of(ids):
        return float(np.mean([len(set(a) & set(b)) / K for a, b in zip(ids.tolist(), truth.tolist())]))

    hnsw_ms = float(np.mean([k["hnsw_ms"] for k in kern_ms]))
    e, x = stats[-1]["dist_evals"], stats[-1]["expansions"]
    by = 4.0 * D * e + 4.0 * 2 * args.M * x   # 4*D*E + 4*deg_slots*X (deg0 = 2M)
    achieved = by / (hnsw_ms * 1e-3) / 1e9
    sweep = {}
    for ef in args.ef_sweep:   # the configs[2] ef sweep on the same graph and queries
        def step_e(timed, ef=ef):
            ix.search_batch_device(qt.data_ptr(), NQ, K, out_ids.data_ptr(), out_d.data_ptr(), out_n.data_ptr(),
                                   ef=ef, mode="hnsw", stream=ctx.stream)
            if corpus:
                merge()
        ix.set_timing(True)
        el = ctx.time_steps(step_e, args.steps, 1, before_timed=ix.last_kernel_times)
        km = ix.last_kernel_times()["hnsw_ms"]
        se = ix.last_batch_stats()
        got = (m_ids if corpus else out_ids).cpu().numpy().view(np.uint64)
        r_e = float(np.mean([len(set(a) & set(b)) / K for a, b in zip(got.tolist(), truth.tolist())]))
        b_e = 4.0 * D * se["dist_evals"] + 4.0 * 2 * args.M * se["expansions"]
        sweep[str(ef)] = {"value": round(NQ * (1 if corpus else ws) * args.steps / el, 1),
                          "ms_per_step": round(1000 * el / args.steps, 3), "recall@10": round(r_e, 4),
                          "kernel_ms": round(km, 3),
                          "hbm_frac_gpu_counts": round(b_e / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "dist_evals_per_query": round(se["dist_evals"] / NQ, 1)}
    ix.set_timing(False)
    if args.dump_ids:   # the shard's graph and answers, for the multi-rank parity test
        np.savez(args.dump_ids % {"rank": rank} if "%(rank)" in args.dump_ids else args.dump_ids,
                 ids=hi_ids, dists=hi_d, shard_ids=shard_ids, shard_dists=shard_d, lo=lo, n_local=n_local,
                 **{"g_" + k: np.asarray(v) for k, v in ix.download_graph().items()})
    units = NQ * (1 if corpus else ws)
    rows_per_rank = ctx.per_rank(n_local)
    res = {
        "metric": METRIC, "value": round(units * args.steps / elapsed, 1), "unit": "queries/s", "rows_per_rank": rows_per_rank,
        "ms_per_step": round(1000 * elapsed / args.steps, 3), "recall@10": round(rec, 4),
        "recall_truth": "exact path on the same queries (all of them)",
        "scaling": "strong" if corpus else "weak",
        "workload": "hnsw knnSearchByVector ef=%d, %s x %d-d %s, %d-query batch%s (M=%d, efConstruction=%d)"
                    % (args.ef, f"{N:,}", D, args.metric, NQ, "" if corpus else " per GPU", args.M, args.efc),
        "parallelism": (f"corpus sharded over {ws} GPU(s) by id range ({n_local:,} rows and their own graph per GPU), "
                        f"RCCL all-gather of per-shard top-k + device merge" if corpus else
                        f"{ws} GPU(s), each holding the graph and answering its own batch"),
        "data": {"sift": "SIFT-shaped (1024 centres + 24-d latent + noise, non-negative integers)",
                 "uniform": "U[0,1)", "gauss": "N(0,1)/sqrt(D)", "glove": GLOVE_DESC}[data],
        "graph": graph,
        "exact_same_data": {"ms_one_batch": round(exact_ms, 2), "fallback_queries": exact_fb,
                            "note": "the exact path on these queries, one untimed-loop call after the hnsw steps"},
        "roofline": {"bound": "hbm", "kernel": "wv_hnsw_kernel", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None, "kernel_ms": round(hnsw_ms, 3), "counts_from": "GPU counters",
                     "dist_evals_per_query": round(e / NQ, 1), "expansions_per_query": round(x / NQ, 1),
                     "fallback_queries": stats[-1]["fallbacks"]},
    }
    attach_traffic(res["roofline"], n_local, NQ, D, data)
    if sweep:
        res["ef_sweep"] = sweep
    if args.concurrency and ws == 1:
        res["concurrent_callers"] = concurrent_callers(args, ix, queries)
        if args.open_loop:
            res["open_loop"] = open_loop(args, ix, queries, res["concurrent_callers"])
    if not with_cpu and getattr(args, "counts_sample", 0) > 0 and base is not None:
        # SURVEY 8d's byte basis from the restatement's own evaluation counts
        # on a query sample of this shard's graph (no CPU timing): the GPU's
        # visited-cache re-evaluations are not counted as useful bytes
        O = _oracle()
        ref = O.Index(D, args.metric, args.M, args.efc, capacity=n_local, seed=1)
        ref.import_graph(base, ix.download_graph())
        ns_ = min(NQ, args.counts_sample)
        ost = ref.search_batch(queries[:ns_], K, args.ef, threads=args.cpu_threads)[3]
        e_q, x_q = ost["dist_evals"] / ns_, ost["expansions"] / ns_
        by = (4.0 * D * e_q + 4.0 * 2 * args.M * x_q) * NQ
        achieved = by / (hnsw_ms * 1e-3) / 1e9
        res["roofline"].update({"achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
                                "counts_from": f"CPU restatement (oracle/) on the same graph, {ns_}-query sample",
                                "dist_evals_per_query": round(e_q, 1), "expansions_per_query": round(x_q, 1),
                                "gpu_dist_evals_per_query": round(stats[-1]["dist_evals"] / NQ, 1)})
        del ref
    if base is None and getattr(args, "exact_counts_sample", 0) > 0:
        # corpora too large to restate on the host (configs[4]): the same
        # traversal counted on the GPU with an exact per-query visited bitmap
        # (WV_HNSW_UNIQUE_COUNTS) -- each node's layer-0 evaluation once, as
        # the reference's visited list allows, not the lossy cache's repeats
        ns_ = min(NQ, args.exact_counts_sample)
        os.environ["WV_HNSW_UNIQUE_COUNTS"] = "1"
        try:
            ix.search_batch_device(qt.data_ptr(), ns_, K, out_ids.data_ptr(), out_d.data_ptr(), out_n.data_ptr(),
                                   ef=args.ef, mode="hnsw", stream=ctx.stream)
            torch.cuda.synchronize(ctx.dev)
            su = ix.last_batch_stats()
        finally:
            del os.environ["WV_HNSW_UNIQUE_COUNTS"]
        e_q, x_q = su["dist_evals"] / ns_, su["expansions"] / ns_
        by = (4.0 * D * e_q + 4.0 * 2 * args.M * x_q) * NQ
        achieved = by / (hnsw_ms * 1e-3) / 1e9
        res["roofline"].update({"achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
                                "counts_from": f"GPU traversal with an exact per-query visited bitmap (each node's "
                                               f"evaluation counted once, as the reference's visited list), "
                                               f"{ns_}-query sample",
                                "dist_evals_per_query": round(e_q, 1), "expansions_per_query": round(x_q, 1),
                                "gpu_dist_evals_per_query": round(stats[-1]["dist_evals"] / NQ, 1)})
    if with_cpu:
        ref = O.Index(D, args.metric, args.M, args.efc, capacity=N, seed=1)
        ref.import_graph(base, ix.download_graph())   # the restatement searches the very same graph
        for ef, line in sweep.items():
            ri = ref.search_batch(queries, K, int(ef), threads=args.cpu_threads)[0]
            line["recall@10_cpu_restatement"] = round(
                float(np.mean([len(set(a) & set(b)) / K for a, b in zip(ri.tolist(), truth.tolist())])), 4)
        probe = min(NQ, 500)
        t0 = time.perf_counter()
        ref.search_batch(queries[:probe], K, args.ef, threads=args.cpu_threads)
        per_q = (time.perf_counter() - t0) / probe
        reps = max(1, int(args.cpu_seconds / max(per_q * NQ, 1e-9)))
        t0 = time.perf_counter()
        for _ in range(reps):
            oi, od, on, ost = ref.search_batch(queries, K, args.ef, threads=args.cpu_threads)
        cpu_t = (time.perf_counter() - t0) / reps
        n1 = int(min(NQ, max(100, args.cpu_seconds_t1 / max(per_q * args.cpu_threads, 1e-9))))
        t0 = time.perf_counter()
        ref.search_batch(queries[:n1], K, args.ef, threads=1)
        t1 = time.perf_counter() - t0
        # algorithmic bytes from the restatement's own count of distance
        # evaluations E and expansions X on the same graph / queries / ef
        # (SURVEY 8d), not from the GPU's counters
        e, x = ost["dist_evals"], ost["expansions"]
        by = 4.0 * D * e + 4.0 * 2 * args.M * x
        achieved = by / (hnsw_ms * 1e-3) / 1e9
        res["roofline"].update({"achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
                                "counts_from": "CPU restatement (oracle/) on the same graph",
                                "dist_evals_per_query": round(e / NQ, 1), "expansions_per_query": round(x / NQ, 1),
                                "gpu_dist_evals_per_query": round(stats[-1]["dist_evals"] / NQ, 1)})
        id_eq, d_eq, tie_ok = parity_stats(hi_ids, hi_d, oi, od)
        rec_cpu = float(np.mean([len(set(a) & set(b)) / K for a, b in zip(oi.tolist(), truth.tolist())]))
        res["parity_sample"] = {"queries": NQ, "id_match_frac": id_eq, "dists_bitwise_equal_frac": d_eq,
                                "tie_aware_identical_frac": tie_ok, "recall@10_gpu": round(rec, 4),
                                "recall@10_cpu_restatement": round(rec_cpu, 4)}
        res["cpu_baseline"] = {"value": round(NQ / cpu_t, 1), "unit": "queries/s", "cores": args.cpu_threads,
                               "host_cores": args.host_cores,
                               "kind": "port", "value_t1": round(n1 / t1, 1), "cores_t1": 1,
                               "sample": f"all {NQ} queries x {reps} passes (T={args.cpu_threads}), {n1} queries "
                                         f"(T=1); knnSearchByVector restated in C on the same graph (oracle/)"}
        if getattr(args, "filtered_fracs", None):
            res["filtered_hnsw"] = filtered_hnsw_legs(args, ctx, ix, ref, queries, qt, NQ, K, D, n_local)
        if getattr(args, "tomb_frac", 0) > 0:
            res["tombstoned"] = tombstoned_leg(args, ctx, ix, ref, queries, qt, NQ, K, D, n_local, res)
        if args.seq_build:
            # north_star: recall within 0.5 pt of the reference index -- whose
            # graph is built by inserting one node at a time (insert.go:103-217,
            # here the restatement's concurrent build) -- on identical data and ef
            del ref
            t0 = time.time()
            seq = O.Index(D, args.metric, args.M, args.efc, capacity=N, seed=1)
            seq.add_batch(base, threads=args.hnsw_build_threads)
            build_s = time.time() - t0
            si = seq.search_batch(queries, K, args.ef, threads=args.cpu_threads)[0]
            # the GPU-built graph's recall at the other ef too (before the
            # sequential graph replaces it on the device)
            efs = [args.ef] + ([128] if args.ef != 128 and 128 in args.ef_sweep else [])
            r_built = {args.ef: rec}
            for ef_ in efs[1:]:
                ix.search_batch_device(qt.data_ptr(), NQ, K, out_ids.data_ptr(), out_d.data_ptr(),
                                       out_n.data_ptr(), ef=ef_, mode="hnsw", stream=ctx.stream)
                torch.cuda.synchronize(ctx.dev)
                r_built[ef_] = recall_of(out_ids.cpu().numpy().view(np.uint64))
            ix.upload_graph(seq.export_graph())
            del seq
            r_seq_gpu = {}
            for ef_ in efs:
                ix.search_batch_device(qt.data_ptr(), NQ, K, out_ids.data_ptr(), out_d.data_ptr(),
                                       out_n.data_ptr(), ef=ef_, mode="hnsw", stream=ctx.stream)
                torch.cuda.synchronize(ctx.dev)
                r_seq_gpu[ef_] = recall_of(out_ids.cpu().numpy().view(np.uint64))
            r_seq = recall_of(si)
            res["sequential_build"] = {
                "recall@10_restatement_on_sequential_graph": round(r_seq, 4),
                "recall@10_gpu_on_sequential_graph": round(r_seq_gpu[args.ef], 4),
                "recall@10_gpu_built_graph": round(rec, 4),
                "delta_pt_gpu_built_vs_sequential": round(100 * (rec - r_seq), 2),
                "by_ef": {str(e): {"gpu_built": round(r_built[e], 4), "sequential": round(r_seq_gpu[e], 4),
                                   "delta_pt": round(100 * (r_built[e] - r_seq_gpu[e]), 2)} for e in efs},
                "sequential_build_s": round(build_s, 1), "threads": args.hnsw_build_threads}
    ix.close()
    return res


def filtered_hnsw_legs(args, ctx, ix, ref, queries, qt, NQ, K, D, n_local):
    """Filtered HNSW on the configs[0] graph (search.go:74-78 with forbidFlat,
    or |allow| >= flatSearchCutoff: the allow list is applied at layer 0,
    :282-298): a shared Bernoulli(p) list (seed 3), ef = the line's ef.  QPS,
    HBM fraction from the restatement's counts on the same graph, parity
    with the restatement (knnSearchByVector with the list), recall against
    the filtered exact answer, the restatement's own time on the host cores
    (cpu_baseline), and the rate of queries whose side set outgrew its HBM
    spill (answered by the exact filtered scan).  Lists below 40k rows
    (flatSearchCutoff) run as forbidFlat; the 1 % leg takes 1000 queries."""
    torch = ctx.torch
    out = {}
    for frac in args.filtered_fracs:
        nq = NQ if frac >= 0.05 else min(NQ, 1000)
        oi_, od_, on_ = _out_tensors(ctx, nq, K)
        a = argparse.Namespace(**vars(args))
        a.allow_frac = frac
        words, n_allowed = _allow_words(a, 0, n_local)
        allow_t = torch.from_numpy(words.view(np.int64)).to(ctx.dev)

        def step(timed, mode="hnsw"):
            ix.search_batch_device(qt.data_ptr(), nq, K, oi_.data_ptr(), od_.data_ptr(), on_.data_ptr(), ef=args.ef,
                                   mode=mode, stream=ctx.stream, allow_ptr=allow_t.data_ptr(), allow_nbits=n_local)

        ix.set_timing(True)
        el = ctx.time_steps(step, args.steps, args.warmup, before_timed=ix.last_kernel_times)
        km = ix.last_kernel_times()["hnsw_ms"]
        st = ix.last_batch_stats()
        ss = ix.last_side_stats()
        ix.set_timing(False)
        gi = oi_.cpu().numpy().view(np.uint64).copy()
        gd = od_.cpu().numpy().copy()
        step(False, mode="exact")
        torch.cuda.synchronize(ctx.dev)
        truth = oi_.cpu().numpy().view(np.uint64).copy()
        t0 = time.perf_counter()
        ri, rd, rn, rst = ref.search_batch(queries[:nq], K, args.ef, allow=words, threads=args.cpu_threads)
        cpu_s = time.perf_counter() - t0
        id_eq, d_eq, tie_ok = parity_stats(gi, gd, ri, rd)
        rec = float(np.mean([len(set(x) & set(y)) / K for x, y in zip(gi.tolist(), truth.tolist())]))
        rec_cpu = float(np.mean([len(set(x) & set(y)) / K for x, y in zip(ri.tolist(), truth.tolist())]))
        e, x = rst["dist_evals"], rst["expansions"]
        by = 4.0 * D * e + 4.0 * 2 * args.M * x
        achieved = by / (km * 1e-3) / 1e9
        leg = {
            "value": round(nq * args.steps / el, 1), "unit": "queries/s", "ms_per_step": round(1000 * el / args.steps, 3),
            "queries": nq, "allowed_rows": int(n_allowed), "ef": args.ef,
            "dispatch": "forbidFlat (|allow| < flatSearchCutoff 40000)" if n_allowed < 40000 else
                        "hnsw (|allow| >= flatSearchCutoff)",
            "recall@10_vs_filtered_exact": round(rec, 4), "recall@10_cpu_restatement": round(rec_cpu, 4),
            "exact_fallback_queries": int(st["fallbacks"]), "exact_fallback_rate": round(st["fallbacks"] / nq, 4),
            "side_state": {"lds_side_rows": ss["side_rows"], "spill_cap": ss["spill_cap"],
                           "light_pass_redone": ss["redone"], "spill_overflowed": ss["overflowed"]},
            "parity_sample": {"queries": nq, "id_match_frac": id_eq, "dists_bitwise_equal_frac": d_eq,
                              "tie_aware_identical_frac": tie_ok},
            "cpu_baseline": {"value": round(nq / cpu_s, 1), "unit": "queries/s", "cores": args.cpu_threads,
                             "kind": "port", "sample": f"the same {nq} queries and list, knnSearchByVector restated "
                                                       f"in C (oracle/), T={args.cpu_threads}"},
            "roofline": {"bound": "hbm", "kernel": "wv_hnsw_side_kernel", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None, "kernel_ms": round(km, 3),
                         "counts_from": "CPU restatement (oracle/) on the same graph and list",
                         "dist_evals_per_query": round(e / nq, 1), "expansions_per_query": round(x / nq, 1),
                         "gpu_dist_evals_per_query": round(st["dist_evals"] / nq, 1)}}
        attach_traffic(leg["roofline"], n_local, nq, D, args.hnsw_data, allow_frac=frac)
        out["allow_%g%%" % (100 * frac)] = leg
    return out


def tombstoned_leg(args, ctx, ix, ref, queries, qt, NQ, K, D, n_local, res):
    """The same line on a shard with a fraction of its ids tombstoned
    (delete.go:546-551: an update is a delete + insert and tombstones live
    until cleanup): tombstoned nodes are traversed but never returned
    (search.go:294-296, :347-349), so the side-register path runs (results
    in registers; the lossy visited cache at this selectivity, a rare
    overflow re-run with the exact bitmap).  QPS against the tombstone-free
    value, the lone caller's latency through the micro-batcher, and parity
    with the restatement under the same tombstones.  The tombstones are
    cleared afterwards."""
    torch = ctx.torch
    dead = np.nonzero(counter_uniform(5, 0, n_local, 1)[:, 0] < args.tomb_frac)[0]
    ix.add_tombstones(dead)
    oi_, od_, on_ = _out_tensors(ctx, NQ, K)

    def step(timed):
        ix.search_batch_device(qt.data_ptr(), NQ, K, oi_.data_ptr(), od_.data_ptr(), on_.data_ptr(), ef=args.ef,
                               mode="hnsw", stream=ctx.stream)

    ix.set_timing(True)
    el = ctx.time_steps(step, args.steps, args.warmup, before_timed=ix.last_kernel_times)
    km = ix.last_kernel_times()["hnsw_ms"]
    st, ss = ix.last_batch_stats(), ix.last_side_stats()
    ix.set_timing(False)
    gi = oi_.cpu().numpy().view(np.uint64).copy()
    gd = od_.cpu().numpy().copy()
    for t in dead.tolist():
        ref.add_tombstone(int(t))
    ri, rd, rn, rst = ref.search_batch(queries, K, args.ef, threads=args.cpu_threads)
    for t in dead.tolist():
        ref.remove_tombstone(int(t))
    id_eq, d_eq, tie_ok = parity_stats(gi, gd, ri, rd)
    leaked = int(np.isin(gi[gi != np.uint64(0xFFFFFFFFFFFFFFFF)], dead.astype(np.uint64)).sum())
    a1 = argparse.Namespace(**vars(args))
    a1.concurrency = [1]
    lone = concurrent_callers(a1, ix, queries).get("1", {})
    ix.set_tombstones([])
    e, x = rst["dist_evals"], rst["expansions"]
    by = 4.0 * D * e + 4.0 * 2 * args.M * x
    achieved = by / (km * 1e-3) / 1e9
    free = res.get("value")
    val = NQ * args.steps / el
    roof = {"bound": "hbm", "kernel": "wv_hnsw_side_kernel", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel_ms": round(km, 3),
            "counts_from": "CPU restatement (oracle/) with the same tombstones",
            "dist_evals_per_query": round(e / NQ, 1), "expansions_per_query": round(x / NQ, 1),
            "gpu_dist_evals_per_query": round(st["dist_evals"] / NQ, 1)}
    attach_traffic(roof, n_local, NQ, D, args.hnsw_data, allow_frac="tomb:%g" % args.tomb_frac)
    return {"value": round(val, 1), "unit": "queries/s", "ms_per_step": round(1000 * el / args.steps, 3),
            "tombstoned_ids": int(len(dead)), "tomb_frac": args.tomb_frac,
            "vs_tombstone_free_value": round(val / free, 4) if free else None,
            "tombstoned_ids_returned": leaked, "exact_fallback_queries": int(st["fallbacks"]),
            "side_state": {"lds_side_rows": ss["side_rows"], "light_pass_redone": ss["redone"],
                           "spill_overflowed": ss["overflowed"]},
            "parity_sample": {"queries": NQ, "id_match_frac": id_eq, "dists_bitwise_equal_frac": d_eq,
                              "tie_aware_identical_frac": tie_ok},
            "lone_caller_through_batcher": lone,
            "roofline": roof}


def concurrent_callers(args, ix, queries):
    """The production path: T native threads each calling SearchByVector for
    one query at a time (index.go:988-1028 -> shard_read.go:246-252) through
    the library's micro-batcher (wv_batcher_search, AUTO dispatch at the
    index's searchTimeEF) -- QPS and per-call latency.  The callers run in
    tests/native/libwvload.so (measurement infrastructure)."""
    import ctypes as C
    path = os.path.join(ROOT, "tests", "native", "libwvload.so")
    if not os.path.exists(path):
        return {"error": "tests/native/libwvload.so not built"}
    lib = C.CDLL(path)
    lib.wvl_concurrent.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int,
                                   C.c_int, C.c_void_p]
    q = np.ascontiguousarray(queries, dtype=np.float32)
    ix.update_user_config(ef=args.ef)   # searchTimeEF = the line's ef
    out = {}
    for t in args.concurrency:
        r = np.zeros(6, np.float64)
        rc = lib.wvl_concurrent(C.c_void_p(ix._h.value if hasattr(ix._h, "value") else ix._h), q.ctypes.data,
                                q.shape[0], q.shape[1], args.k, t, args.concurrency_seconds, args.max_batch, 0,
                                r.ctypes.data)
        if rc:
            out[str(t)] = {"error": f"status {rc}"}
            continue
        out[str(t)] = {"value": round(r[0], 1), "unit": "queries/s", "p50_us": round(r[1], 1),
                       "p99_us": round(r[2], 1), "mean_batch": round(r[3], 1), "requests": int(r[4]),
                       "seconds": round(r[5], 2)}
    ix.update_user_config(ef=-1)
    out["note"] = (f"T threads x one query per call (k={args.k}, ef={args.ef}), wv_batcher_search: two workers, "
                   f"max_batch {args.max_batch}, latency-first dispatch (no linger); host query in, host result out")
    return out


def open_loop(args, ix, queries, closed):
    """Open-loop arrivals through the micro-batcher: Poisson requests at 10 %
    and 50 % of the closed-loop capacity (the largest caller count's QPS),
    each issued at its time by a pool of native threads -- the reference
    answers every SearchByVector on its own (shard_read.go:252), so an
    arrival must not wait for callers that are not coming (wv_batcher.cpp:
    the refill wait runs only while the last batch's callers resubmit).
    Latency from the scheduled arrival (no coordinated omission)."""
    import ctypes as C
    path = os.path.join(ROOT, "tests", "native", "libwvload.so")
    lib = C.CDLL(path)
    if not hasattr(lib, "wvl_open_loop"):
        return {"error": "libwvload.so lacks wvl_open_loop"}
    lib.wvl_open_loop.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int,
                                  C.c_int, C.c_void_p]
    caps = [v["value"] for v in closed.values() if isinstance(v, dict) and "value" in v]
    if not caps:
        return {"error": "no closed-loop capacity"}
    cap = max(caps)
    q = np.ascontiguousarray(queries, dtype=np.float32)
    ix.update_user_config(ef=args.ef)
    out = {"capacity_qps": round(cap, 1)}
    for f in args.open_loop:
        rate = f * cap
        r = np.zeros(8, np.float64)
        rc = lib.wvl_open_loop(C.c_void_p(ix._h.value if hasattr(ix._h, "value") else ix._h), q.ctypes.data,
                               q.shape[0], q.shape[1], args.k, rate, args.open_loop_seconds, args.max_batch, 512,
                               r.ctypes.data)
        if rc:
            out[f"{f:.0%}"] = {"error": f"status {rc}"}
            continue
        out[f"{f:.0%}"] = {"offered_qps": round(rate, 1), "achieved_qps": round(r[0], 1), "p50_us": round(r[1], 1),
                           "p99_us": round(r[2], 1), "p999_us": round(r[3], 1), "max_us": round(r[4], 1),
                           "mean_batch": round(r[5], 1), "requests": int(r[6]), "late_starts": int(r[7])}
    ix.update_user_config(ef=-1)
    out["note"] = ("Poisson arrivals (seed 7) at the given share of the closed-loop capacity, 512 pool threads, "
                   f"k={args.k}, ef={args.ef}; latency from the scheduled arrival; late_starts = requests issued "
                   ">50 us after their time (pool saturated)")
    return out


def group_leg(args):
    """Child process (no torch.distributed): one process drives `--group-devices`
    through libwvgpu.so's in-process group (wv_group_*, the layout a single Go
    server uses): the corpus sharded by id range, per-shard top-k gathered to
    the first device over RCCL (ncclCommInitAll) and merged there.  Timed
    through the host entry point (query upload and result download included)."""
    import weaviate_amd as W
    devs = [int(x) for x in args.group_devices.split(",")]
    N, D, NQ, K = args.rows, args.dim, args.nq, args.k
    gen = {"uniform": counter_uniform, "gauss": counter_gauss, "sift": counter_sift, "glove": counter_glove}[args.data]
    base = gen(1, 0, N, D)
    queries = gen(2, 0, NQ, D)
    g = W.GPUGroup(devs, D, args.metric, capacity=N, layout="shard")
    g.upload_vectors(base)
    del base
    for _ in range(args.warmup):
        g.search_batch(queries, K, mode="exact")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ids, ds, n = g.search_batch(queries, K, mode="exact")
    dt = time.perf_counter() - t0
    res = {"value": round(NQ * args.steps / dt, 1), "unit": "queries/s", "ms_per_step": round(1e3 * dt / args.steps, 3),
           "members": len(devs), "uses_rccl": g.info()["uses_rccl"],
           "workload": f"exact {K}-NN, {N:,} x {D}-d {args.metric}, {NQ}-query batch, corpus sharded over "
                       f"{len(devs)} devices in ONE process (wv_group_search_batch, host buffers in and out)"}
    if args.dump_ids and os.path.exists(args.dump_ids):
        ref = np.load(args.dump_ids)
        res["ids_equal_single_gpu"] = bool(np.array_equal(ids, ref["ids"]) and
                                           np.array_equal(ds.view(np.uint32), ref["dists"].view(np.uint32)))
    g.close()
    print(json.dumps(res), flush=True)


def run_group_leg_child(args, ws, final_ids, final_d):
    """Rank 0 after every rank left the process group: the in-process group
    leg in a child process, bounded by a timeout (its failure is reported, not
    fatal to the bench line)."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        ref = os.path.join(td, "rank0.npz")
        np.savez(ref, ids=final_ids, dists=final_d)
        env = {k: v for k, v in os.environ.items()
               if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                            "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
        cmd = [sys.executable, os.path.abspath(__file__), "--group-leg", "--group-devices",
               ",".join(str(i) for i in range(ws)), "--rows", str(args.rows), "--dim", str(args.dim), "--nq",
               str(args.nq), "--k", str(args.k), "--metric", args.metric, "--data", args.data, "--steps",
               str(args.steps), "--warmup", str(args.warmup), "--dump-ids", ref]
        try:
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
        except subprocess.TimeoutExpired:
            return {"error": "timed out after 240 s"}
        if p.returncode != 0:
            return {"error": f"exit {p.returncode}", "stderr_tail": p.stderr[-600:]}
        try:
            return json.loads(p.stdout.strip().splitlines()[-1])
        except Exception:
            return {"error": "no JSON line", "stdout_tail": p.stdout[-600:]}


def main():
    global GLOVE_NOISE
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["exact", "hnsw"], default="exact")
    ap.add_argument("--split", choices=["query", "corpus"], default="",
                    help="N>1: query = every GPU holds the corpus and answers its own batch (default, weak scaling); "
                         "corpus = id-range shards + RCCL all-gather + device merge (strong scaling)")
    ap.add_argument("--rows", type=int, default=1_000_000, help="corpus rows N (all shards)")
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--nq", type=int, default=10_000, help="queries per batch (per GPU with --split query)")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--ef", type=int, default=64)
    ap.add_argument("--ef-sweep", default="", help="hnsw: comma-separated ef values timed after the main line "
                                                   "(configs[2]: 32,64,128,256)")
    ap.add_argument("--metric", default="l2-squared")
    ap.add_argument("--data", choices=["auto", "uniform", "gauss", "sift", "glove"], default="auto",
                    help="uniform: U[0,1) (tie-free, configs[1]); gauss: N(0,1)/sqrt(D) (GloVe/Deep/C4-shaped); "
                         "sift: clustered non-negative integers (SIFT-shaped, configs[0]); "
                         "auto: uniform for exact, sift for hnsw")
    ap.add_argument("--glove-noise", type=float, default=GLOVE_NOISE,
                    help="glove data: full-rank residual relative to the latent part")
    ap.add_argument("--concurrency", default="1,8,64,256",
                    help="hnsw: concurrent single-query caller counts timed through the micro-batcher ('' = skip)")
    ap.add_argument("--concurrency-seconds", type=float, default=2.0)
    ap.add_argument("--open-loop", default="0.1,0.5",
                    help="hnsw: open-loop Poisson arrival rates as shares of the closed-loop capacity ('' = skip)")
    ap.add_argument("--open-loop-seconds", type=float, default=1.5)
    ap.add_argument("--max-batch", type=int, default=1024, help="micro-batcher: queries per launch")
    ap.add_argument("--allow-frac", type=float, default=0.0,
                    help="exact mode: shared allow list, Bernoulli(p) over ids (seed 3, BASELINE configs[3])")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time (T=all)")
    ap.add_argument("--cpu-seconds-t1", type=float, default=5.0, help="target CPU-baseline sample time (T=1)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (GOMAXPROCS-equivalent); 0 = every CPU this process may use")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hnsw-line", action="store_true",
                    help="skip the configs[0] hnsw line that the exact workload reports beside its value")
    ap.add_argument("--no-corpus-leg", action="store_true",
                    help="N>1 exact: skip the corpus-sharded (RCCL merge) leg reported beside the query split")
    ap.add_argument("--seq-build", action="store_true",
                    help="hnsw at N=1: also build the restatement's insert-by-insert graph and report its recall "
                         "beside the GPU-built graph's (north_star's 0.5-pt criterion; ~40 s of CPU at 1M; on by "
                         "default for the C1 line beside the exact value)")
    ap.add_argument("--no-seq-build", action="store_true", help="skip the C1 line's sequential-build recall check")
    ap.add_argument("--c5-rows", type=int, default=100_000_000,
                    help="configs[4] corpus rows, sharded N ways (100M / N rows and graph per GPU)")
    ap.add_argument("--c5-weak", action="store_true",
                    help="the configs[4] line with 12.5M rows per GPU (weak scaling) instead of the fixed corpus")
    ap.add_argument("--no-c5-line", action="store_true",
                    help="skip the configs[4] line (100M x 96 corpus sharded over the N GPUs, hnsw + RCCL merge)")
    ap.add_argument("--tomb-frac", type=float, default=0.01,
                    help="C1 line: also time the shard with this fraction of ids tombstoned (0 = skip)")
    ap.add_argument("--no-filtered-hnsw", action="store_true",
                    help="skip the filtered-HNSW legs (allow 10 / 50 %%, forbidFlat) on the configs[0] graph")
    ap.add_argument("--no-c4-line", action="store_true",
                    help="skip the configs[3] line (10M x 768 dot, allow lists 100/50/10/1 %%, sharded over the N GPUs)")
    ap.add_argument("--c4-rows", type=int, default=10_000_000)
    ap.add_argument("--c4-nq", type=int, default=1000)
    ap.add_argument("--c4-fracs", default="1,0.5,0.1,0.01", help="configs[3] allow-list selectivities")
    ap.add_argument("--c4-cpu-seconds", type=float, default=4.0)
    ap.add_argument("--c4-cpu-seconds-t1", type=float, default=2.0)
    ap.add_argument("--no-c3-line", action="store_true",
                    help="skip the configs[2] GloVe-shaped hnsw ef-sweep line reported beside the default value")
    ap.add_argument("--hnsw-build-threads", type=int, default=16)
    ap.add_argument("--M", type=int, default=64, help="hnsw maxConnections (layer-0 degree 2M)")
    ap.add_argument("--efc", type=int, default=128, help="hnsw efConstruction")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL over xGMI, the product path); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--dump-ids", default="", help="rank 0 saves the final ids/dists (npz) for cross-N checks")
    ap.add_argument("--graph-build", choices=["cpu", "gpu"], default="gpu",
                    help="hnsw graph: wv_index_build_graph on the GPU (default) or the CPU restatement's "
                         "sequential build (reference-equivalent, slow at 1M)")
    ap.add_argument("--batch-div", type=int, default=64, help="GPU build: batch = inserted / batch_div")
    ap.add_argument("--graph-cache", default="", help="npz path: load the hnsw graph if present, else build and save")
    ap.add_argument("--no-wide-line", action="store_true", help="skip the k=100 / SearchByVectorDistance lines")
    ap.add_argument("--no-group-leg", action="store_true",
                    help="N>1 exact: skip the in-process multi-GPU group leg (wv_group, RCCL gather) run by rank 0")
    ap.add_argument("--group-leg", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--group-devices", default="0", help=argparse.SUPPRESS)
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from build_hash import host_cores_info
    args.host_cores = host_cores_info()
    if args.cpu_threads <= 0:
        args.cpu_threads = args.host_cores["cores"]
    args.ef_sweep = [int(x) for x in args.ef_sweep.split(",") if x]
    args.c4_fracs = [float(x) for x in args.c4_fracs.split(",") if x]
    args.concurrency = [int(x) for x in args.concurrency.split(",") if x]
    args.open_loop = [float(x) for x in args.open_loop.split(",") if x]
    GLOVE_NOISE = args.glove_noise
    if args.group_leg:
        if args.data == "auto":
            args.data = "uniform"
        return group_leg(args)

    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    ws, rank, _ = dist_env()
    if ws != args.gpus:
        print(json.dumps({"error": f"--gpus {args.gpus} but WORLD_SIZE={ws}: launch with --nproc-per-node "
                                   f"{args.gpus} or without a launcher"}), flush=True)
        sys.exit(2)
    if not args.split:
        # the north-star layout (id-range shards + RCCL merge) for the
        # sharded configs -- configs[3] (10M x 768 dot) and configs[4] (100M x
        # 96 hnsw) -- and for any corpus past 8M rows; the query split for
        # configs[0]/[1]'s 1M rows, which one GPU holds whole
        sharded_cfg = args.rows >= 8_000_000 or (args.dim >= 512 and args.metric == "dot")
        args.split = "corpus" if (ws == 1 or sharded_cfg) else "query"
    if args.data == "auto":
        args.data = "sift" if args.workload == "hnsw" else "uniform"
    args.hnsw_data = args.data if args.workload == "hnsw" else "sift"

    import weaviate_amd as W
    _heartbeat()
    ctx = Ctx(args)
    with_cpu = rank == 0 and ws == 1 and not args.no_cpu_baseline

    if args.workload == "hnsw":
        h = run_hnsw(args, ctx, W, with_cpu)
        result = {"metric": METRIC, "value": h["value"], "unit": "queries/s", "n_gpus": ws,
                  "devices": ctx.n_devices, "steps": args.steps, "warmup": args.warmup,
                  "ms_per_step": h["ms_per_step"], "higher_is_better": True, "scaling": h["scaling"],
                  "vs_baseline": None, "dtype": "f32", "data": "synthetic: counter-based " + h["data"],
                  "config": {"workload": h["workload"], "N": args.rows, "dim": args.dim, "nq": args.nq,
                             "k": args.k, "metric": args.metric, "mode": "hnsw", "split": args.split,
                             "parallelism": h["parallelism"]},
                  "recall@10": h["recall@10"], "graph": h["graph"], "roofline": h["roofline"]}
        for key in ("parity_sample", "cpu_baseline", "ef_sweep", "concurrent_callers", "sequential_build"):
            if key in h:
                result[key] = h[key]
    else:
        phase("exact headline (configs[1])")
        e, st = run_exact(args, ctx, W)
        result = {
            "metric": METRIC, "value": e["value"], "unit": "queries/s", "n_gpus": ws, "devices": ctx.n_devices,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": e["ms_per_step"], "higher_is_better": True,
            "scaling": e["scaling"], "vs_baseline": None,
            "dtype": e["dtype"],
            "data": "synthetic: counter-based %s float32 corpus (seed 1) and queries (seed 2)" % {
                "uniform": "U[0,1)", "gauss": "N(0,1)/sqrt(D)", "glove": GLOVE_DESC,
                "sift": "SIFT-shaped (1024 centres + 24-d latent + noise, non-negative integers)"}[args.data],
            "config": {"workload": e["workload"], "N": args.rows, "dim": args.dim, "nq": args.nq, "k": args.k,
                       "metric": args.metric, "mode": "exact", "recall@10": 1.0, "split": args.split,
                       "parallelism": e["parallelism"]},
            "roofline": e["roofline"],
        }
        if with_cpu:
            phase("exact CPU baseline + parity sample")
            O = _oracle()
            result["cpu_baseline"], result["parity_sample"] = exact_cpu_baseline(args, st, O)
        if ws == 1 and args.allow_frac == 0 and not args.no_wide_line:
            phase("wide k / SearchByVectorDistance")
            result["wide_k"] = wide_k_line(args, ctx, st, W)
        if args.dump_ids and rank == 0:
            np.savez(args.dump_ids, ids=st["final_ids"], dists=st["final_d"])
        rank0_final = (st["final_ids"], st["final_d"])
        # N > 1: the north-star layout beside the query split -- id-range
        # shards, RCCL all-gather, device merge -- on rank 0's batch, whose
        # merged answer must equal rank 0's whole-corpus answer bit for bit
        if ws > 1 and args.split == "query" and not args.no_corpus_leg:
            rank0_ids, rank0_d = st["final_ids"], st["final_d"]
            st["ix"].close()
            a2 = argparse.Namespace(**vars(args))
            a2.split = "corpus"
            c, cst = run_exact(a2, ctx, W)
            result["corpus_sharded"] = {
                "value": c["value"], "unit": "queries/s", "ms_per_step": c["ms_per_step"], "scaling": "strong",
                "parallelism": c["parallelism"], "kernel_ms": c["roofline"]["kernel_ms"],
                "ids_equal_query_split": bool(rank == 0 and np.array_equal(cst["final_ids"], rank0_ids)
                                              and np.array_equal(cst["final_d"].view(np.uint32),
                                                                 rank0_d.view(np.uint32)))}
            cst["ix"].close()
        else:
            st["ix"].close()
        if not args.no_hnsw_line and args.metric == "l2-squared":
            # (the C1 line at N = 1 also reports north_star's criterion: recall
            # within 0.5 pt of the insert-by-insert graph; --no-seq-build skips it)
            a1 = argparse.Namespace(**vars(args))
            a1.seq_build = (args.seq_build or (not args.no_seq_build and args.rows == 1_000_000)) and ws == 1
            a1.filtered_fracs = [] if args.no_filtered_hnsw else [0.1, 0.5, 0.01]
            a1.dump_ids = ""   # (--dump-ids holds the exact line's answers)
            phase("configs[0] hnsw line")
            h = run_hnsw(a1, ctx, W, with_cpu)
            h.pop("metric", None)
            result["hnsw_c1"] = h
        if not args.no_c3_line and ws == 1 and (args.rows, args.dim, args.metric) == (1_000_000, 128, "l2-squared"):
            # configs[2]: GloVe-100-shaped 1.2M x 100 cosine, hnsw ef sweep 32-256
            a3 = argparse.Namespace(**vars(args))
            a3.rows, a3.dim, a3.metric, a3.hnsw_data = 1_200_000, 100, "cosine-dot", "glove"
            a3.ef, a3.ef_sweep, a3.concurrency, a3.split = 64, [32, 64, 128, 256], [], "corpus"
            a3.cpu_seconds, a3.cpu_seconds_t1, a3.graph_build, a3.dump_ids = 4.0, 2.0, "gpu", ""
            # north_star's 0.5-pt recall check against the insert-by-insert
            # graph at this line's ef and 128 (~50 s of CPU at 1.2M rows)
            a3.seq_build = not args.no_seq_build and ws == 1
            phase("configs[2] hnsw ef sweep")
            h = run_hnsw(a3, ctx, W, with_cpu)
            h.pop("metric", None)
            result["hnsw_c3"] = h
        if not args.no_c4_line and args.rows == 1_000_000 and args.metric == "l2-squared":
            try:
                phase("configs[3] exact 10M x 768 dot")
                result["exact_c4"] = c4_line(args, ctx, W, with_cpu)
            except Exception as e:   # reported, not fatal to the headline line
                result["exact_c4"] = {"error": f"{type(e).__name__}: {e}"}
        if not args.no_c5_line and args.rows == 1_000_000 and args.metric == "l2-squared":
            # configs[4]'s layout: a Deep/SIFT-shaped 96-d corpus sharded by id
            # range over the N GPUs, every GPU building and searching the graph
            # of its shard, per-shard top-k all-gathered over RCCL and merged on
            # the device (index.go:967-1044).  The corpus is the fixed 100M
            # rows at every N (100M / N rows and graph per GPU, strong
            # scaling; N = 1 holds all of it: 38.4 GB of rows + a 51 GB
            # layer-0 CSR in 288 GB).  The rows are generated on the device
            # and the graph built there: linear, 14.2 s per 12.5M rows
            # (profiles/r05/build_scaling_probe.log).  --c5-weak: 12.5M rows
            # per GPU instead.
            a5 = argparse.Namespace(**vars(args))
            c5_fixed = not args.c5_weak
            c5_rows = args.c5_rows if c5_fixed else 12_500_000 * ws
            a5.rows, a5.dim, a5.metric, a5.hnsw_data = c5_rows, 96, "l2-squared", "sift"
            # (ef 128: recall@10 0.963 over the 100M corpus on one GPU, where
            # ef 64 gives 0.893 -- the metric is QPS at recall >= 0.95)
            a5.ef, a5.ef_sweep, a5.concurrency, a5.split = 128, [64], [], "corpus"
            a5.graph_build, a5.dump_ids, a5.seq_build = "gpu", "", False
            a5.device_data = True
            a5.counts_sample, a5.exact_counts_sample = 0, 1000
            try:
                phase("configs[4] hnsw over the 100M corpus")
                h = run_hnsw(a5, ctx, W, False)
                h.pop("metric", None)
                if c5_fixed:
                    h["scaling"] = f"strong (fixed {c5_rows:,}-row corpus, {c5_rows // ws:,} rows per GPU)"
                else:
                    h["scaling"] = "weak (12.5M rows per GPU; the 100M corpus at N = 8)"
                h["value_units"] = (f"queries/s over the whole {a5.rows:,}-row corpus"
                                    + (" (every rank searches the batch over its shard)" if ws > 1 else " on one GPU"))
                result["hnsw_c5_sharded"] = h
            except Exception as e:   # reported, not fatal to the headline line
                result["hnsw_c5_sharded"] = {"error": f"{type(e).__name__}: {e}"}
    result["distributed"] = ctx.info()
    if ws > 1:
        ctx.barrier()
        ctx.dist.destroy_process_group()
        # the other ranks exit here and leave their GPUs idle for the group leg
        if (rank == 0 and args.workload == "exact" and not args.no_group_leg and args.split == "query"
                and ctx.n_devices == ws and args.allow_frac == 0):
            result["group_in_process"] = run_group_leg_child(args, ws, *rank0_final)
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()

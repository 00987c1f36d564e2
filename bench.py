"""Headline benchmark: exact top-10 queries/sec over 10M x 1536 fp32 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4|c5]
                    [--ntotal N] [--batch B] [--k K] [--metric ip|l2] [--no-cpu-baseline]

Ranks: under torchrun (WORLD_SIZE set) this process is one rank.  Started
directly with --gpus N > 1, it is a launcher: it starts N fresh rank processes
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, 127.0.0.1
rendezvous), never touches HIP itself, and exits with their status.  Rank 0
prints the JSON line with n_gpus = the world size RCCL saw and the head-count
of an all-gather over every rank.

Workloads (BASELINE.json configs; the default is the one the metric is quoted on):
  c3  10M x 1536 fp32, batch 4096, top-10 IP.  One step = one exact search of the
      batch over the whole corpus, row-sharded over the N ranks (one process per
      GPU) with an RCCL all-gather + GPU merge of the per-shard lists.
  c2  1M x 1536 fp32, batch 1024, top-10 IP (same path, smaller corpus).
  c4  graph_refresher self-join: 1M student rows, cosine top-50 excluding self;
      the corpus is replicated and the query rows are split over the ranks.
  c5  50M x 1536 bf16-stored corpus (row-sharded), batches of 8 queries with a
      1 % remove + 1 % append mutation every 10 batches (seed 91011); recall@10
      of the final index against fp32 exact search on 1000 queries (1 GPU).
Corpus and queries are generated on the device by the counter-based generator
(no dataset exists offline) and are resident in HBM before the timed region.

Rank 0 prints ONE JSON line.  Besides the driver's fields:
  roofline      the dominant kernel: algorithmic work per launch (FLOP for the
                MFMA kernels, bytes for the HBM-bound GEMV) / mean launch time from
                HIP events recorded on the launch stream (vs_timer_*), against the
                fp32 (157.3 TFLOP/s) / bf16 (2.5 PFLOP/s) matrix peak or 8 TB/s HBM;
                `traffic` is the PMC-measured HBM bytes per launch when a rocprofv3
                summary for this workload exists in profiles/ (tools/pmc_summary.py)
  batch1        (c3/c2) the B=1 latency path (gemv_topk, HBM-bound), same corpus
  cpu_baseline  (c3/c2, N=1) the faiss-semantics CPU port (oracle/flat.knn_faiss_fp32:
                blocked numpy-BLAS sgemm + top-k, all host threads) on a bounded
                sample, extrapolated linearly in N (a flat scan is linear in N)
"""

from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "book-recommendation-engine_amd"))
sys.path.insert(0, ROOT)

METRIC_NAME = "exact top-10 queries/sec at 10M×1536 fp32 (1/8 GPU) + % HBM/MFMA roofline"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: Peak FP32 (matrix)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: Peak BF16 MFMA (dense)
# MI355X_MICROARCH.md, MFMA table: I8 32x32x32 takes the cycles of BF16 32x32x16
# (2x K), so the dense int8 MFMA rate is twice the bf16 one
I8_MFMA_PEAK_TOPS = 2.0 * BF16_MFMA_PEAK_TFLOPS
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak (spec)
HBM_KERNELS = ("gemv_topk", "skinny_topk")


def mfma_kind(kname: str, esz: int) -> str:
    if kname == "gemm_topk_x1_i8":  # one int8 MFMA product per fp32 product
        return "mfma_x1_i8"
    if kname == "gemm_topk_x1":  # one bf16 MFMA product per fp32 product
        return "mfma_x1"
    return "mfma32" if esz == 4 else "mfma16"


def is_x1(kname: str) -> bool:
    return kname.startswith("gemm_topk_x1")


def x1_dominant(ctx, work_total, kms, nl):
    """The filter engine's first stage runs on the int8 or the bf16 plane per
    search (the library's adaptive order).  Returns the plane that took most of
    the timed kernel time: (timer name, its share of the algorithmic work, its
    kernel ms, its dispatches, per-plane record).  A pass whose later launches
    are dump launches times its first (list) launch apart ("<name>_list"): the
    roofline is the dump kernel's own time.  Each span's work is the share of
    its pass's database tiles the library recorded for it (a list launch
    covers less than a dump launch)."""
    mi, ni, si = ctx.lib.timer_read_kernel_share("gemm_topk_x1_i8")
    mil, nil, sil = ctx.lib.timer_read_kernel_share("gemm_topk_x1_i8_list")
    mip, _ = ctx.lib.timer_read_kernel("gemm_topk_x1_i8_pass")
    mb, nb, sb = ctx.lib.timer_read_kernel_share("gemm_topk_x1")
    mbl, nbl, sbl = ctx.lib.timer_read_kernel_share("gemm_topk_x1_list")
    mbp, _ = ctx.lib.timer_read_kernel("gemm_topk_x1_pass")
    # launches of a pass cover unequal parts of it (the list launch a quarter
    # chunk, or 1/8 of a split pass): work in proportion to the tiles each
    # span covered (the library's per-span shares, in passes)
    per = work_total / max(1e-12, si + sil + sb + sbl)
    split = {"i8": {"dispatches": ni, "kernel_ms": round(mi, 3)},
             "i8_list_launches": {"dispatches": nil, "kernel_ms": round(mil, 3)},
             "i8_whole_passes": {"kernel_ms": round(mip, 3)},
             "bf16": {"dispatches": nb, "kernel_ms": round(mb, 3)},
             "bf16_list_launches": {"dispatches": nbl, "kernel_ms": round(mbl, 3)},
             "bf16_whole_passes": {"kernel_ms": round(mbp, 3)}}
    # the whole pass of the dominant plane: its list and dump launches plus the
    # cut and replay kernels between them (one span per pass), over the work
    # of all its launches
    if mi + mil >= mb + mbl:
        split["whole_pass"] = (per * (si + sil), mip)
        return "gemm_topk_x1_i8", per * si, mi, ni, split
    split["whole_pass"] = (per * (sb + sbl), mbp)
    return "gemm_topk_x1", per * sb, mb, nb, split


def rocprof_prefix(kname: str):
    """rocprof's name of a timed kernel: gemm_topk_x1<KR, MODE, DUMP, EL> with EL
    1 = int8, 0 = bf16 (the plane is the last template argument); the PMC
    lookup takes the instantiation with the most dispatches (the dump launches
    where a pass has them)."""
    if kname == "gemm_topk_x1_i8":
        return "void vs::gemm_topk_x1<", "el=1"
    if kname == "gemm_topk_x1":
        return "void vs::gemm_topk_x1<", "el=0"
    # the small-batch plane pass: skinny_plane_topk<KL, EL, NQG, NT>, EL 1 = int8
    if kname == "skinny_plane_topk_i8":
        return "void vs::skinny_plane_topk<", "<8, 1,"
    if kname == "skinny_plane_topk":
        return "void vs::skinny_plane_topk<", "<8, 0,"
    return "void vs::" + kname + "<", ""


def kernel_matches(name: str, must: str) -> bool:
    """`must` is a substring of the rocprof name, or "el=<plane>": the x1
    kernel's fourth template argument (gemm_topk_x1<KR, MODE, DUMP, EL[, HYB]>)."""
    if not must.startswith("el="):
        return must in name
    i, j = name.find("<"), name.find(">(")
    args = [a.strip() for a in name[i + 1:j].split(",")] if 0 <= i < j else []
    return len(args) >= 4 and args[3] == must[3:]

DEFAULTS = {
    "c3": dict(ntotal=10_000_000, batch=4096, k=10, metric="ip", dtype="f32"),
    "c2": dict(ntotal=1_000_000, batch=1024, k=10, metric="ip", dtype="f32"),
    "c4": dict(ntotal=1_000_000, batch=0, k=50, metric="cos", dtype="f32"),
    "c5": dict(ntotal=50_000_000, batch=8, k=10, metric="ip", dtype="bf16"),
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--workload", choices=sorted(DEFAULTS), default="c3")
    p.add_argument("--ntotal", type=int, default=None)
    p.add_argument("--d", type=int, default=1536)
    p.add_argument("--batch", type=int, default=None)
    p.add_argument("--k", type=int, default=None)
    p.add_argument("--metric", choices=["ip", "l2"], default=None)
    p.add_argument("--data", choices=["uniform", "clustered"], default="uniform",
                   help="c2/c3 corpus: counter-based uniform rows (default) or unit-norm "
                        "clustered rows like text embeddings (1024 centroids, noise 0.5; "
                        "one GPU only) to measure the filter engine's fallback rate")
    p.add_argument("--batch1-steps", type=int, default=20)
    p.add_argument("--wide-k", default="30,60",
                   help="the service's wide k values (service.py:627 k = 30, :529-531 "
                        "k = 60) for the wide-k leg, comma-separated")
    p.add_argument("--wide-k-batch", type=int, default=4096)
    p.add_argument("--wide-k-steps", type=int, default=3)
    p.add_argument("--any-k", type=int, default=100,
                   help="k of the any-k leg (the agent-chosen k of search_catalog, "
                        "mcp_book_server.py:115,142): batch 1 and the full batch through "
                        "the paged exact engine; 0 skips it")
    p.add_argument("--clustered-steps", type=int, default=3,
                   help="C3 on one GPU: after the headline, the same search over unit-norm "
                        "clustered rows (text-embedding-like, --data clustered) timed for "
                        "this many steps as the `clustered` record; 0 skips it")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-rows", type=int, default=1_000_000)
    p.add_argument("--cpu-queries", type=int, default=1024)
    p.add_argument("--recall-queries", type=int, default=1000)
    p.add_argument("--cpu-batch1-rows", type=int, default=1_000_000)
    p.add_argument("--dry-run", action="store_true",
                   help="launcher/collective rehearsal on CPU (gloo, no GPU, no kernel): "
                        "each step all-gathers a (batch, k) list like the sharded search; "
                        "the line carries dry_run=true and is not a measurement")
    a = p.parse_args(argv)
    for key, val in DEFAULTS[a.workload].items():
        if getattr(a, key, None) is None:
            setattr(a, key, val)
    if a.steps is None:
        a.steps = {"c3": 5, "c2": 10, "c4": 2, "c5": 30}[a.workload]
    return a


def pmc_traffic(workload: str, kernel_prefix: str, must_contain: str = ""):
    """HBM bytes per launch of the benched kernel from the newest PMC summary in
    profiles/ (tools/pmc_summary.py).  Among the instantiations whose full
    rocprof name starts with `kernel_prefix` and contains `must_contain` (the
    x1 kernel's plane), and among each one's launch geometries (grid sizes:
    full passes vs the staged engine's small gathered ones), the (name, grid)
    with the most dispatches is the dominant kernel; its bytes are returned
    with a source string naming the file, the full name, the grid and the
    dispatch count."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc_{workload}.json")))
    for path in reversed(files):  # newest tag first
        with open(path, encoding="utf-8") as f:
            summ = json.load(f)
        best = None
        for name, rec in summ.get("kernels", {}).items():
            if not (name.startswith(kernel_prefix) and kernel_matches(name, must_contain)):
                continue
            groups = rec.get("by_grid") or {"?": rec}
            dump = kernel_matches(name, "el=1") or kernel_matches(name, "el=0")
            dump = dump and ", true, " in name.split("(")[0]  # DUMP = the third argument
            for grid, g in groups.items():
                # the most dispatches; a dump launch over a list launch on a tie
                # (a split pass: one of each per search)
                key = (g["dispatches"], dump)
                if best is None or key > best[0]:
                    best = (key, g["hbm_bytes_per_launch"], name, grid)
        if best is not None:
            (n, _), hbm, name, grid = best
            return hbm, (f"{os.path.relpath(path, ROOT)}: {name.split('(')[0]} grid {grid}, "
                         f"{n} dispatches")
    return None, None


def cpu_baseline(shard, args, xq_host):
    """faiss-semantics CPU port timed on a bounded sample of the same workload."""
    from threadpoolctl import threadpool_info

    from oracle import flat

    n = min(args.cpu_rows, shard.ntotal)
    xb = shard.reconstruct_n(0, n)  # the same synthetic rows, copied to host
    xq = xq_host[: args.cpu_queries]
    metric = flat.METRIC_INNER_PRODUCT if args.metric == "ip" else flat.METRIC_L2
    flat.knn_faiss_fp32(xb[:1000], xq[:8], args.k, metric)  # warm BLAS threads
    t0 = time.perf_counter()
    flat.knn_faiss_fp32(xb, xq, args.k, metric)
    dt = time.perf_counter() - t0
    threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    qps_full = xq.shape[0] / dt * n / args.ntotal
    affinity = len(os.sched_getaffinity(0))
    res = {
        "value": round(qps_full, 3),
        "unit": "queries/s",
        "cores": int(threads),
        # the BLAS pool runs at the thread count the GPU pool grants one GPU's job
        # (OMP_NUM_THREADS, set by the box; its rules: "leave them", worker pools
        # sized to the box's CPU share, 16 per GPU) although the affinity mask
        # shows every host CPU; the all-CPU figure is a linear extrapolation
        "thread_cap": {"threads_used": int(threads),
                       "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
                       "reason": "the GPU pool's CPU share for a one-GPU job"},
        "value_all_host_cpus_extrapolated": round(qps_full * affinity / max(1, int(threads)), 3),
        "kind": "port",
        "sample": f"{xq.shape[0]} queries x {n} rows (first rows of the same corpus), "
                  f"{dt:.2f} s; extrapolated x{n}/{args.ntotal} rows (flat scan is linear in N)",
        "impl": "oracle/flat.py knn_faiss_fp32: faiss BLAS branch restated "
                "(numpy sgemm blocks + top-k), faiss-cpu not installable offline",
        "cpu_model": cpu_model(),
        "host_cpus_affinity": affinity,
    }
    # the reference's live shape: one query (mcp_book_server.py:142 -> faiss
    # sequential branch, nq < 20: one thread scans every row with a size-k heap)
    if args.cpu_batch1_rows > 0:
        from oracle import cfaiss

        n1 = min(args.cpu_batch1_rows, n)
        q1 = xq[:1]
        cfaiss.knn_seq(xb[:1000], q1, args.k, metric)  # load / warm
        t0 = time.perf_counter()
        cfaiss.knn_seq(xb[:n1], q1, args.k, metric)
        dt1 = time.perf_counter() - t0
        ms_full = dt1 * 1e3 * args.ntotal / n1
        res["batch1"] = {
            "ms_per_query": round(ms_full, 3), "qps": round(1e3 / ms_full, 4), "cores": 1,
            "kind": "port",
            "sample": f"1 query x {n1} rows, {dt1:.3f} s; extrapolated x{args.ntotal}/{n1} rows",
            "impl": "oracle/faiss_flat.c oracle_knn_seq: faiss's sequential branch (fp32 "
                    "scalar sums + heap) on one thread, as faiss runs nq=1 (the parity "
                    "oracle's strict summation order: slower than faiss)",
        }
        # faiss-speed stand-in: the same scan with faiss's reassociated SIMD sums
        cfaiss.knn_seq_simd(xb[:1000], q1, args.k, metric)
        t0 = time.perf_counter()
        _, Is = cfaiss.knn_seq_simd(xb[:n1], q1, args.k, metric)
        dts = time.perf_counter() - t0
        _, Ic = cfaiss.knn_seq(xb[:n1], q1, args.k, metric)
        ms_simd = dts * 1e3 * args.ntotal / n1
        res["batch1"]["faiss_speed"] = {
            "ms_per_query": round(ms_simd, 3), "qps": round(1e3 / ms_simd, 4), "cores": 1,
            "kind": "port",
            "sample": f"1 query x {n1} rows, {dts:.3f} s; extrapolated x{args.ntotal}/{n1} rows",
            "impl": "oracle/faiss_flat_simd.c: faiss fvec_inner_product/L2sqr's reassociated "
                    "AVX2 sums (16 lanes, FMA) + the same heap, one thread, -O3; the faiss-"
                    "speed stand-in (timing only)",
            "labels_match_scalar": bool((Is == Ic).all()),
        }
    return res


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo", encoding="utf-8") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def launch_ranks(argv, n: int) -> int:
    """Start n rank processes of this script and wait for them (the driver's
    `bench.py --gpus N` form).  The parent imports nothing that touches HIP, so
    each rank initialises its own GPU in a fresh process."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                    "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    try:
        for p in procs:
            code = p.wait()
            if code != 0 and rc == 0:
                rc = code
                for q in procs:  # one rank failed: the others would wait forever
                    if q.poll() is None:
                        q.terminate()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc if rc >= 0 else 1


class Ctx:
    def __init__(self, args):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.args = torch, dist, args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dry = bool(args.dry_run)
        if self.world != args.gpus:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE={self.world}; using WORLD_SIZE",
                  file=sys.stderr)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        if self.dry:
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dev = torch.device("cpu")
            self.lib = None
            self.stream = 0
        else:
            # Test hooks (tests/test_gpu_world2.py; the driver sets neither):
            # VS_BENCH_DEVICE puts every rank on one device, VS_BENCH_BACKEND=gloo
            # runs the collectives on host tensors (RCCL refuses two ranks on one
            # GPU), so the N > 1 data path runs on a one-GPU box.
            if os.environ.get("VS_BENCH_DEVICE") is not None:
                self.local = int(os.environ["VS_BENCH_DEVICE"])
            torch.cuda.set_device(self.local)
            if os.environ.get("VS_BENCH_BACKEND", "nccl") == "gloo":
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            else:
                dist.init_process_group("nccl", rank=self.rank, world_size=self.world,
                                        device_id=torch.device("cuda", self.local))
            from vsearch import _lib

            self.dev = torch.device("cuda", self.local)
            self.lib = _lib
            self.stream = torch.cuda.current_stream().cuda_stream
        self.backend = dist.get_backend()
        # collectives run on device tensors over RCCL, on host tensors over gloo
        self.cdev = self.dev if self.backend == "nccl" else torch.device("cpu")
        # head-count over the collective itself: every rank reports (rank, device)
        me = torch.tensor([1, self.rank, -1 if self.dry else self.local], dtype=torch.int64,
                          device=self.cdev)
        allv = [torch.zeros_like(me) for _ in range(self.world)]
        dist.all_gather(allv, me)
        self.ranks_seen = int(sum(int(v[0]) for v in allv))
        self.devices = [int(v[2]) for v in allv]

    def synchronize(self):
        if not self.dry:
            self.torch.cuda.synchronize()

    def sync_all(self):
        self.dist.barrier()
        self.synchronize()

    def max_over_ranks(self, x: float) -> float:
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def queries(self, n, d, row0=50_000_000, seed=5678):
        q = self.torch.empty((n, d), dtype=self.torch.float32, device="cuda")
        self.lib.check(self.lib.load().vs_fill_synthetic(
            ctypes.c_void_p(q.data_ptr()), n, d, seed, row0, ctypes.c_void_p(self.stream)))
        self.torch.cuda.synchronize()
        return q

    def timed(self, fn, steps, warmup):
        """W untimed steps; K timed steps bracketed by barrier + synchronize;
        max over ranks.  Returns (seconds, kernel_ms_total, kernel_launches, last)."""
        last = None
        for _ in range(warmup):
            last = fn(-1)
        self.synchronize()
        if self.lib:
            self.lib.timer_reset()
            self.lib.timer_enable(True)
        self.sync_all()
        t0 = time.perf_counter()
        for i in range(steps):
            last = fn(i)
        self.synchronize()
        self.dist.barrier()
        t1 = time.perf_counter()
        kms, nl = 0.0, 0
        if self.lib:
            self.lib.timer_enable(False)
            kms, nl = self.lib.timer_read()
        return self.max_over_ranks(t1 - t0), kms, nl, last


def dump_record(d, o):
    """The filter pass's dump launches over the timed steps (vs_gemm_x1.hip
    header): rows stored below the lists' floors (one (row, raw sum) slot
    each) and lane lists out of slots."""
    return {"on": os.environ.get("VS_X1_DUMP", "1") != "0", "rows_dumped": d,
            "lists_out_of_slots": o}


def base_result(args, ctx, value, elapsed, unit="queries/s"):
    return {
        "metric": METRIC_NAME,
        "value": round(value, 3),
        "unit": unit,
        "n_gpus": ctx.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "ranks_seen": ctx.ranks_seen,
        "devices": ctx.devices,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32" if args.dtype == "f32" else "bf16",
        "data": "synthetic: counter-based splitmix64 rows in [-1,1) generated on device "
                "(corpus seed 1234, queries seed 5678)",
    }


def roofline(kind, work_total, kms, nl, unit_desc, kernel, traffic, traffic_src):
    """Roofline record of the dominant kernel over the timed region.

    work_total  algorithmic FLOP (MFMA kinds) or bytes (hbm) of all timed steps
    kms, nl     summed HIP-event time (ms) of those launches and their dispatch
                count (gemm_topk_x3 cuts one search into several dispatches)
    achieved = work_total / kernel time = work per dispatch / mean dispatch time,
    the figure rocprofv3's per-kernel average duration reproduces."""
    if kind == "mfma32":
        peak, unit, bound, scale = FP32_MFMA_PEAK_TFLOPS, "TFLOP/s", "mfma", 1e12
    elif kind == "mfma16":
        peak, unit, bound, scale = BF16_MFMA_PEAK_TFLOPS, "TFLOP/s", "mfma", 1e12
    elif kind == "mfma_x1":
        peak, unit, bound, scale = BF16_MFMA_PEAK_TFLOPS, "TFLOP/s", "mfma", 1e12
    elif kind == "mfma_x1_i8":
        peak, unit, bound, scale = I8_MFMA_PEAK_TOPS, "TFLOP/s", "mfma", 1e12
    else:
        peak, unit, bound, scale = HBM_PEAK_GBS, "GB/s", "hbm", 1e9
    secs = kms / 1e3
    achieved = work_total / secs / scale if secs > 0 else 0.0
    nl = max(1, nl)
    r = {"bound": bound, "kernel": kernel, "achieved": round(achieved, 3), "peak": peak,
         "unit": unit, "frac": round(achieved / peak, 4) if peak else None,
         "traffic": traffic,
         "per_launch": f"{unit_desc}; {work_total / nl:.4g} "
                       f"{'FLOP' if bound == 'mfma' else 'B'} per dispatch, "
                       f"mean dispatch {kms / nl:.3f} ms over {nl} dispatches"}
    if traffic is not None:
        r["traffic_note"] = ("PMC HBM bytes per dispatch (2*FETCH_SIZE + WRITE_SIZE, "
                             "gfx950 correction; Infinity-Cache hits included)")
    if kind == "mfma_x1":
        r["peak_note"] = ("filter pass of the filter-and-verify engine: one bf16 MFMA product "
                          "per fp32 product (bf16 copies of rows and queries), against the dense "
                          "bf16 peak; candidates are then rescored exactly in fp64 and a "
                          "rigorous error bound proves the exact top-k is among them")
    if kind == "mfma_x1_i8":
        r["peak_note"] = ("filter pass of the filter-and-verify engine: one int8 MFMA product "
                          "per fp32 product (int8 codes of rows and queries, one fp32 scale per "
                          "row; 2*N*d int8 multiply-adds per query, counted as FLOP) against the "
                          "dense int8 MFMA peak (2x bf16, MI355X_MICROARCH.md); candidates are "
                          "then rescored exactly in fp64 and a rigorous error bound proves the "
                          "exact top-k is among them")
    if kind in HELD_CLOCK_CEILING:
        c = HELD_CLOCK_CEILING[kind]
        r["held_clock_ceiling"] = {
            "value": c, "frac": round(achieved / c, 4),
            "source": "tools/mfma_ceiling.hip: the same MFMAs at the filter kernel's occupancy "
                      "with no loads (mean of 5 runs on one MI355X, profiles/r05k/mfma_ceiling.json)"}
    if traffic_src:
        r["traffic_source"] = traffic_src
    return r


# The most the filter kernel's MFMA stream reaches on this chip at the clock it
# holds under that load (TFLOP/s; nominal peaks above): int8 0.895, bf16 0.986.
HELD_CLOCK_CEILING = {"mfma_x1_i8": 4473.7, "mfma_x1": 2464.2}


def add_whole_pass(rf, split, scale):
    """`roofline` describes the dump launches alone (the kernel rocprofv3's mean
    is checked against); `whole_pass` puts the same plane's whole filter pass
    beside it: list + dump launches + the cut / replay kernels between them,
    over the algorithmic work of all the pass's launches."""
    work, ms = split.pop("whole_pass")
    rf["scope"] = "dump launches of the filter pass only (the dominant kernel)"
    if ms > 0:
        ach = work / (ms / 1e3) / scale
        rf["whole_pass"] = {"achieved": round(ach, 3), "frac": round(ach / rf["peak"], 4),
                            "kernel_ms": round(ms, 3),
                            "scope": "list + dump launches + x1_qcut / x1_replay kernels"}


class ClusteredRows:
    """Unit-norm rows like text embeddings: row i = normalize(c[i % 1024] + 0.5 * n_i),
    centroids c and noise n_i standard normal / sqrt(d) (the clustered
    variant).  Deterministic per 1M-row chunk; queries use another noise seed."""

    def __init__(self, torch, d, seed, noise_seed=None, ncent=1024, sigma=0.5):
        self.torch, self.d, self.sigma = torch, d, sigma
        self.noise_seed = seed + 1 if noise_seed is None else noise_seed
        g = torch.Generator(device="cuda").manual_seed(seed)
        c = torch.randn((ncent, d), generator=g, device="cuda")
        self.cent = c / c.norm(dim=1, keepdim=True)

    def rows(self, r0, n):
        torch = self.torch
        g = torch.Generator(device="cuda").manual_seed(self.noise_seed * 1_000_003 + r0)
        idx = torch.arange(r0, r0 + n, device="cuda") % self.cent.shape[0]
        x = self.cent[idx] + self.sigma * torch.randn((n, self.d), generator=g,
                                                      device="cuda") / self.d ** 0.5
        return (x / x.norm(dim=1, keepdim=True)).contiguous()


def run_knn(args, ctx):
    import numpy as np

    from vsearch import faiss as vfaiss
    from vsearch.sharded import ShardedIndexFlat

    torch = ctx.torch
    metric = vfaiss.METRIC_INNER_PRODUCT if args.metric == "ip" else vfaiss.METRIC_L2
    index = ShardedIndexFlat(args.d, metric, device=ctx.local, dtype=args.dtype)
    B, d, k = args.batch, args.d, args.k
    if args.data == "clustered":
        if ctx.world != 1:
            raise SystemExit("--data clustered runs on one GPU")
        gen = ClusteredRows(torch, d, seed=1234)
        for r0 in range(0, args.ntotal, 1 << 20):
            x = gen.rows(r0, min(1 << 20, args.ntotal - r0))
            index.shard.add_device(x.data_ptr(), x.shape[0], stream=ctx.stream)
            torch.cuda.synchronize()
            del x
        index._sync_counts()
        xq = ClusteredRows(torch, d, seed=1234, noise_seed=5678).rows(0, B)
    else:
        index.add_synthetic(args.ntotal, seed=1234)
        xq = ctx.queries(B, d)
    n_shard = index.shard.ntotal

    ctx.lib.filter_stats(reset=True)
    elapsed, kms, nl, (D, I) = ctx.timed(
        lambda i: index.search_device(xq, k, stream=ctx.stream), args.steps, args.warmup)
    fw = ctx.lib.filter_wide_stats()
    f2 = ctx.lib.filter_second_stats()
    we, wr = ctx.lib.filter_wide_sets()
    dmp = ctx.lib.filter_dump_stats()
    fq, ff = ctx.lib.filter_stats(reset=True)
    Dh, Ih = D.cpu().numpy(), I.cpu().numpy()
    sane = bool((Ih >= 0).all() and (Ih < args.ntotal).all())
    sane &= bool((np.diff(Dh, axis=1) <= 0).all() if metric == vfaiss.METRIC_INNER_PRODUCT
                 else (np.diff(Dh, axis=1) >= 0).all())
    flops = 2.0 * n_shard * d * B
    esz = 4 if args.dtype == "f32" else 2
    kname = ctx.lib.timer_kernel()
    exact_check = None
    if is_x1(kname):
        # the same queries through the exact fp32 MFMA engine: ids must agree up to
        # exact fp32 near-ties (the verify step makes the filter engine exact; this
        # re-checks it live; the two round their fp32 scores differently)
        nchk = min(B, 256)
        index.shard.set_engine("fp32")
        De, Ie = index.search_device(xq[:nchk].contiguous(), k, stream=ctx.stream)
        index.shard.set_engine("auto")
        De, Ie = De.cpu().numpy(), Ie.cpu().numpy()
        diff = Ie != Ih[:nchk]
        rows = int(diff.any(axis=1).sum())
        dsc = np.abs(De - Dh[:nchk])
        tol = 1e-5 * np.maximum(1.0, np.abs(De))
        beyond = int((diff & (dsc > tol)).any(axis=1).sum())
        exact_check = {"queries": nchk, "engine": "fp32", "rows_with_id_mismatch": rows,
                       "rows_beyond_tie_tolerance": beyond,
                       "max_abs_score_diff": float(dsc.max())}
        sane &= beyond == 0
    gemv = kname in HBM_KERNELS  # the small-batch kernels are HBM-bound
    # PMC summaries are single-GPU profiles: per-dispatch bytes of a 1/N shard differ
    work = flops * args.steps
    split = None
    if is_x1(kname):
        kname, work, kms, nl, split = x1_dominant(ctx, work, kms, nl)
    plane = {"gemm_topk_x1_i8": "i8", "gemm_topk_x1": "bf16"}.get(kname)
    # clustered data runs the bf16 plane at full size: its own PMC summary
    pmc_key = (args.workload + ("cl" if args.data == "clustered" else "")
               + ("l2" if args.metric == "l2" else ""))
    traffic, tsrc = (pmc_traffic(pmc_key, *rocprof_prefix(kname))
                     if ctx.world == 1 else (None, None))
    if gemv:
        rf = roofline("hbm", n_shard * d * esz * args.steps, kms, nl,
                      f"{n_shard}*{d}*{esz} B per search (batch {B} over the rank's shard)",
                      kname, traffic, tsrc)
    else:
        rf = roofline(mfma_kind(kname, esz), work, kms, nl,
                      f"2*{n_shard}*{d}*{B} FLOP per search (whole batch over the rank's shard)",
                      kname, traffic, tsrc)
        if split:
            add_whole_pass(rf, split, scale=1e12)
            rf["first_stage_planes"] = split

    batch1 = None
    if args.batch1_steps > 0 and not gemv:
        q1 = xq[:1].contiguous()
        t1, k1, n1, _ = ctx.timed(lambda i: index.search_device(q1, k, stream=ctx.stream),
                                  args.batch1_steps, 3)
        kern1 = k1 / max(1, n1) / 1e3
        kname1 = ctx.lib.timer_kernel()
        # the small-batch filter pass streams a filter plane (int8: 1 B per
        # element, bf16: 2), the exact kernels the stored rows
        esz1 = {"skinny_plane_topk_i8": 1, "skinny_plane_topk": 2}.get(kname1, esz)
        bytes1 = n_shard * d * esz1
        batch1 = {"ms_per_query": round(t1 / args.batch1_steps * 1e3, 4),
                  "qps": round(args.batch1_steps / t1, 2), "kernel": kname1,
                  "kernel_ms": round(kern1 * 1e3, 4),
                  "bytes_per_query": bytes1,
                  "achieved_GBs": round(bytes1 / kern1 / 1e9, 1) if kern1 > 0 else None,
                  "frac_hbm_peak": round(bytes1 / kern1 / 1e9 / HBM_PEAK_GBS, 4)
                  if kern1 > 0 else None}
        if kname1.startswith("skinny_plane"):
            # beside it, the exact stream over the stored rows (VS_SMALL_FILTER=0)
            prev = os.environ.get("VS_SMALL_FILTER")
            os.environ["VS_SMALL_FILTER"] = "0"
            try:
                t2, k2, n2, _ = ctx.timed(lambda i: index.search_device(q1, k, stream=ctx.stream),
                                          args.batch1_steps, 3)
            finally:
                if prev is None:
                    del os.environ["VS_SMALL_FILTER"]
                else:
                    os.environ["VS_SMALL_FILTER"] = prev
            kern2 = k2 / max(1, n2) / 1e3
            batch1["exact_stream"] = {"ms_per_query": round(t2 / args.batch1_steps * 1e3, 4),
                                      "kernel": ctx.lib.timer_kernel(),
                                      "kernel_ms": round(kern2 * 1e3, 4),
                                      "frac_hbm_peak": round(n_shard * d * esz / kern2 / 1e9 /
                                                             HBM_PEAK_GBS, 4) if kern2 > 0 else None}

    # The service's wide searches (service.py:627 k = 30, :529-531 k = 60 over
    # a coalesced batch): inner product's rule reads the 2k - 1 best, i.e. 64
    # and 128 candidates per query in the filter pass (the two-page exact
    # engine only for what the filter cannot settle).  Measured apart so that
    # each k has a number beside the headline; not part of `value`.
    wide = None
    if (args.wide_k_steps > 0 and metric == vfaiss.METRIC_INNER_PRODUCT and args.wide_k
            and not gemv):
        wide = []
        bw = min(args.wide_k_batch, B)
        qw = xq[:bw].contiguous()
        for kw in [int(v) for v in str(args.wide_k).split(",") if v]:
            ctx.lib.filter_stats(reset=True)
            tw, kmw, nw, (Dw, Iw) = ctx.timed(
                lambda i: index.search_device(qw, kw, stream=ctx.stream), args.wide_k_steps, 1)
            # the plane the searches' first pass ran on (the adaptive order may
            # start on bf16) and that pass's dump launches and whole-pass spans
            wk = ctx.lib.timer_kernel()
            if is_x1(wk):
                wk, _, wmi, wni, wsplit = x1_dominant(ctx, 0.0, kmw, nw)
                wmp = wsplit["whole_pass"][1]
            else:
                wmi, wni, wmp = kmw, nw, 0.0
            ww = ctx.lib.filter_wide_stats()
            w2 = ctx.lib.filter_second_stats()
            wwe, wwr = ctx.lib.filter_wide_sets()
            wq, wf = ctx.lib.filter_stats(reset=True)
            Iwh = Iw.cpu().numpy()
            wide.append({"k": kw, "batch": bw, "steps": args.wide_k_steps,
                         "ms_per_search": round(tw / args.wide_k_steps * 1e3, 3),
                         "queries_per_s": round(args.wide_k_steps * bw / tw, 1),
                         "kernel": wk,
                         "kernel_ms_per_dispatch": round(wmi / max(1, wni), 3),
                         "first_pass_ms_per_search": round(wmp / args.wide_k_steps, 3),
                         "filter_queries": wq, "wide_checked": ww,
                         "wide_set_mean": round(wwe / ww, 1) if ww else 0.0,
                         "wide_rescored_mean": round(wwr / ww, 1) if ww else 0.0,
                         "to_bf16_stage": w2, "exact_redo_queries": wf,
                         "result_sane": bool((Iwh >= 0).all() and (Iwh < args.ntotal).all())})

    # Any k (faiss answers every k; the agent picks search_catalog's k,
    # mcp_book_server.py:115,142): k past one 64-entry page runs the paged exact
    # engine (vs_api.hip run_paged), at batch 1 (the live tool) and at the full
    # batch.  Measured apart; not part of `value`.
    anyk = None
    if args.any_k > 0 and not gemv:
        anyk = []
        for bk, steps in ((1, 3), (B, 1)):
            qk = xq[:bk].contiguous()
            tk, kmk, nk, (Dk, Ik) = ctx.timed(
                lambda i: index.search_device(qk, args.any_k, stream=ctx.stream), steps, 1)
            Ikh, Dkh = Ik.cpu().numpy(), Dk.cpu().numpy()
            ok = bool((Ikh >= 0).all() and (Ikh < args.ntotal).all())
            ok &= bool((np.diff(Dkh, axis=1) <= 0).all() if metric == vfaiss.METRIC_INNER_PRODUCT
                       else (np.diff(Dkh, axis=1) >= 0).all())
            kk = ctx.lib.timer_kernel()
            staged = is_x1(kk) or kk.startswith("skinny_plane")
            anyk.append({"k": args.any_k, "batch": bk, "steps": steps,
                         "ms_per_search": round(tk / steps * 1e3, 3),
                         "queries_per_s": round(steps * bk / tk, 1),
                         "kernel": kk,
                         "kernel_ms_per_search": round(kmk / steps, 3),
                         "engine": ("staged filter and verify, up to 1024 candidates per query "
                                    "(inner product k <= 512, L2 k <= 1023)" if staged else
                                    "paged exact (vs_api.hip run_paged): ceil(k / 64) pages of "
                                    "64 lexicographic entries, more where inner product's tie "
                                    "rule needs them"),
                         "result_sane": ok})

    if ctx.rank == 0:
        cpu = None
        if not args.no_cpu_baseline and ctx.world == 1 and args.dtype == "f32":
            cpu = cpu_baseline(index.shard, args, xq.cpu().numpy())
        res = base_result(args, ctx, args.steps * B / elapsed, elapsed)
        if args.data == "clustered":
            res["data"] = ("synthetic: unit-norm clustered rows (1024 centroids + 0.5 noise, "
                           "torch generator seed 1234; queries noise seed 5678)")
        res["config"] = {
            "workload": f"{args.workload.upper()}: {args.ntotal}x{d} {args.dtype} exact flat "
                        f"{'inner-product' if args.metric == 'ip' else 'L2'}, batch {B}, top-{k}",
            "ntotal": args.ntotal, "d": d, "batch": B, "k": k, "metric": args.metric,
            "parallelism": f"row-shard x{ctx.world} + RCCL all-gather top-k merge",
            "kernel": kname}
        res["roofline"] = rf
        if fq:
            res["filter_verify"] = {"plane": plane, "queries": fq, "wide_checked": fw,
                                    "wide_set_mean": round(we / fw, 1) if fw else 0.0,
                                    "wide_rescored_mean": round(wr / fw, 1) if fw else 0.0,
                                    "to_bf16_stage": f2,
                                    "fallback_queries": ff,
                                    "fallback_rate": round(ff / fq, 6), "exact_check": exact_check,
                                    "dump_launches": dump_record(*dmp)}
        res["batch1"] = batch1
        res["wide_k"] = wide
        res["any_k"] = anyk
        res["cpu_baseline"] = cpu
        # the filter planes the index kept (a memory shortage drops bf16, then
        # both: the exact fp32 engine alone, an order of magnitude slower)
        res["filter_planes"] = list(index.shard.filter_planes)
        res["result_sane"] = sane
        return res
    return None


def clustered_record(res):
    """The headline-shaped summary of a clustered run (run_knn with --data
    clustered), for the `clustered` record beside the uniform headline."""
    fv = res.get("filter_verify") or {}
    rf = res.get("roofline") or {}
    return {"value": res["value"], "unit": res["unit"], "ms_per_step": res["ms_per_step"],
            "steps": res["steps"], "data": res["data"], "kernel": rf.get("kernel"),
            "roofline": {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac",
                                                 "kernel_ms_per_dispatch", "whole_pass")
                         if k in rf},
            "first_stage_planes": rf.get("first_stage_planes"),
            "to_bf16_stage": fv.get("to_bf16_stage"),
            "exact_redo_queries": fv.get("fallback_queries"),
            "exact_check": fv.get("exact_check"),
            "filter_planes": res.get("filter_planes"),
            "result_sane": res.get("result_sane")}


def run_selfjoin(args, ctx):
    """C4: graph_refresher self-join (cosine top-k excluding self); the corpus is
    replicated on every rank and the query rows are split.  Each step ends with
    the writer's input on rank 0: every rank's (similarity, label) rows are
    gathered there over RCCL (graph_refresher/main.py:386-389 inserts them from
    one process), padded to the largest block."""
    from vsearch import faiss as vfaiss
    from vsearch.sharded import shard_bounds

    torch = ctx.torch
    N, d, k = args.ntotal, args.d, args.k
    index = vfaiss.IndexFlat(d, vfaiss.METRIC_INNER_PRODUCT, device=ctx.local, dtype=args.dtype)
    index.reserve(N)
    index.add_synthetic(N, seed=1234)
    lo, hi = shard_bounds(N, ctx.world, ctx.rank)
    nq = hi - lo
    nmax = -(-N // ctx.world)  # largest block
    Dp = torch.full((nmax, k), -3.0e38, dtype=torch.float32, device="cuda")
    Ip = torch.full((nmax, k), -1, dtype=torch.int64, device="cuda")
    D, I = Dp[:nq], Ip[:nq]
    gD = [torch.empty_like(Dp) for _ in range(ctx.world)] if ctx.rank == 0 else None
    gI = [torch.empty_like(Ip) for _ in range(ctx.world)] if ctx.rank == 0 else None

    def step(i):
        index.selfjoin_device(k, lo, nq, D.data_ptr(), I.data_ptr(), stream=ctx.stream)
        if ctx.world > 1:  # the rows go to the one writer process
            if ctx.backend == "nccl":
                ctx.dist.gather(Dp, gD, dst=0)
                ctx.dist.gather(Ip, gI, dst=0)
            else:  # gloo (test hook): host tensors
                hD = [t.cpu() for t in gD] if gD else None
                hI = [t.cpu() for t in gI] if gI else None
                ctx.dist.gather(Dp.cpu(), hD, dst=0)
                ctx.dist.gather(Ip.cpu(), hI, dst=0)
                if ctx.rank == 0:
                    for t, h in zip(gD, hD):
                        t.copy_(h)
                    for t, h in zip(gI, hI):
                        t.copy_(h)
        return None

    ctx.lib.filter_stats(reset=True)
    elapsed, kms, nl, _ = ctx.timed(step, args.steps, args.warmup)
    fw = ctx.lib.filter_wide_stats()
    f2 = ctx.lib.filter_second_stats()
    we, wr = ctx.lib.filter_wide_sets()
    dmp = ctx.lib.filter_dump_stats()
    fq, ff = ctx.lib.filter_stats(reset=True)
    Ih = I.cpu()
    sane = bool(((Ih >= 0) & (Ih < N)).all()) and not bool(
        (Ih == torch.arange(lo, hi)[:, None]).any())
    flops_step = 2.0 * N * d * nq
    kname = ctx.lib.timer_kernel()
    exact_check = None
    if is_x1(kname):
        # the first 256 students again through the fp32 MFMA engine: ids must agree
        nchk = min(nq, 256)
        De = torch.empty((nchk, k), dtype=torch.float32, device="cuda")
        Ie = torch.empty((nchk, k), dtype=torch.int64, device="cuda")
        index.set_engine("fp32")
        index.selfjoin_device(k, lo, nchk, De.data_ptr(), Ie.data_ptr(), stream=ctx.stream)
        index.set_engine("auto")
        torch.cuda.synchronize()
        diff = Ie.cpu() != Ih[:nchk]
        rows = int(diff.any(dim=1).sum())
        # a label may differ only where the two similarities tie within fp32 error
        # (the fp32 engine's own rounding; DESIGN.md §4.1 tolerance)
        dsim = (De - D[:nchk]).abs().cpu()
        beyond = int((diff & (dsim > 1e-5)).any(dim=1).sum())
        exact_check = {"students": nchk, "engine": "fp32", "rows_with_id_mismatch": rows,
                       "rows_beyond_tie_tolerance": beyond,
                       "max_abs_sim_diff": float(dsim.max())}
        sane &= beyond == 0
    work = flops_step * args.steps
    split = None
    if is_x1(kname):
        kname, work, kms, nl, split = x1_dominant(ctx, work, kms, nl)
    plane = {"gemm_topk_x1_i8": "i8", "gemm_topk_x1": "bf16"}.get(kname)
    traffic, tsrc = pmc_traffic(args.workload, *rocprof_prefix(kname))
    esz = 4 if args.dtype == "f32" else 2
    rf = roofline(mfma_kind(kname, esz), work, kms, nl,
                  f"2*{N}*{d}*{nq} FLOP per step ({nq} query rows per rank)",
                  kname, traffic, tsrc)
    if split:
        add_whole_pass(rf, split, scale=1e12)
        rf["first_stage_planes"] = split
    if ctx.rank == 0:
        # the writer's rows: (a, b, sim) with sim >= threshold (main.py:350-354),
        # counted from the gathered arrays of the last step (not timed)
        if ctx.world > 1:
            Sall = torch.cat([g[:shard_bounds(N, ctx.world, r)[1] - shard_bounds(N, ctx.world, r)[0]]
                              for r, g in enumerate(gD)])
            Iall = torch.cat([g[:shard_bounds(N, ctx.world, r)[1] - shard_bounds(N, ctx.world, r)[0]]
                              for r, g in enumerate(gI)])
        else:
            Sall, Iall = D, I
        writer = {"rows_gathered_on_rank0": int(Sall.shape[0]),
                  "edges_sim_ge_0.75": int(((Iall >= 0) & (Sall >= 0.75)).sum().item()),
                  "edges_total": int((Iall >= 0).sum().item())}
        res = base_result(args, ctx, args.steps * N / elapsed, elapsed, unit="students/s")
        res["config"] = {"workload": f"C4: self-join {N}x{d} cosine top-{k} excluding self",
                         "ntotal": N, "d": d, "k": k,
                         "parallelism": f"replicated corpus, query rows split x{ctx.world}, "
                                        "RCCL gather of the rows to rank 0 (the writer)"}
        res["writer"] = writer
        res["roofline"] = rf
        if fq:
            res["filter_verify"] = {"plane": plane, "students": fq, "wide_checked": fw,
                                    "wide_set_mean": round(we / fw, 1) if fw else 0.0,
                                    "wide_rescored_mean": round(wr / fw, 1) if fw else 0.0,
                                    "to_bf16_stage": f2,
                                    "fallback_students": ff,
                                    "fallback_rate": round(ff / fq, 6),
                                    "exact_check": exact_check,
                                    "dump_launches": dump_record(*dmp)}
        res["result_sane"] = sane
        res["cpu_baseline"] = None
        return res
    return None


def run_c5(args, ctx):
    """C5: bf16-stored corpus, interleaved mutations and small query batches,
    recall@10 against fp32 exact search on the final corpus."""
    import numpy as np

    from vsearch import faiss as vfaiss
    from vsearch.sharded import ShardedIndexFlat

    torch = ctx.torch
    metric = vfaiss.METRIC_INNER_PRODUCT if args.metric == "ip" else vfaiss.METRIC_L2
    N, d, k, B = args.ntotal, args.d, args.k, args.batch
    index = ShardedIndexFlat(d, metric, device=ctx.local, dtype=args.dtype)
    index.add_synthetic(N, seed=1234)
    rng = np.random.default_rng(91011)
    xq = ctx.queries(max(B, args.recall_queries), d)
    nmut = max(1, N // 100)
    mut_time = 0.0
    mut_rounds = []  # (remove ms, append ms) per mutation round
    # The workload's mutations are inputs: every removal list (labels of the
    # N-row index; each round removes and appends nmut, so the size stays N)
    # is drawn before the timed region, and the harness's record of which
    # generator row every label holds (for recall) is replayed after it.
    muts = [np.sort(rng.choice(N, nmut, replace=False)).astype(np.int64)
            for i in range(args.steps) if i % 10 == 9]
    done = []

    def step(i):
        nonlocal mut_time
        if i >= 0 and i % 10 == 9:  # 1 % removes + 1 % appends every 10 batches
            # the searches already queued finish first (the removal waits for the
            # index's readers anyway): the time below is the mutation's own
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rm = muts[len(done)]
            index.remove_ids(rm)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            g0 = N + len(done) * nmut
            index.append_synthetic_ids(np.arange(g0, g0 + nmut, dtype=np.int64), seed=1234)
            done.append(rm)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            mut_time += t2 - t0
            mut_rounds.append((round((t1 - t0) * 1e3, 2), round((t2 - t1) * 1e3, 2)))
        j = (max(i, 0) * B) % (xq.shape[0] - B + 1)
        return index.search_device(xq[j:j + B], k, stream=ctx.stream)

    elapsed, kms, nl, _ = ctx.timed(step, args.steps, args.warmup)
    gen = np.arange(N, dtype=np.int64)  # generator row of every current label
    for r, rm in enumerate(done):
        g0 = N + r * nmut
        gen = np.concatenate([np.delete(gen, rm), np.arange(g0, g0 + nmut, dtype=np.int64)])
    assert index.ntotal == gen.size
    n_shard = index.shard.ntotal
    kname = ctx.lib.timer_kernel()
    # the small-batch filter pass streams the index's int8 plane (1 B per
    # element; the verification then reads a few candidate rows), the exact
    # kernels the stored rows (bf16: 2 B)
    esz = {"skinny_plane_topk_i8": 1, "skinny_plane_topk": 2}.get(
        kname, 2 if args.dtype == "bf16" else 4)
    traffic, tsrc = pmc_traffic(args.workload, "void vs::" + kname + "<")
    rf = roofline("hbm", n_shard * d * esz * args.steps, kms, nl,
                  f"{n_shard}*{d}*{esz} B per search (batch {B} over the rank's shard)",
                  kname, traffic, tsrc)
    recall = None
    if ctx.world == 1 and args.recall_queries > 0:
        nr = args.recall_queries
        q = xq[:nr].contiguous()
        Dg, Ig = index.search_device(q, k, stream=ctx.stream)
        Ig = Ig.cpu().numpy()
        # fp32 exact reference over the same (mutated) corpus, rebuilt chunk by chunk
        chunk = 4_000_000
        parts_D, parts_I = [], []
        # the reference chunks keep no filter planes (rows only: beside the
        # bf16 index and its int8 plane, HBM holds 4M fp32 rows but not their
        # planes too); their exact fp32 engine answers
        prev = os.environ.get("VS_FILTER")
        os.environ["VS_FILTER"] = "none"
        for a in range(0, gen.size, chunk):
            ref = vfaiss.IndexFlat(d, metric, device=ctx.local)
            ref.add_synthetic_ids(gen[a:a + chunk], seed=1234)
            ref.set_id_base(a)
            Dr = torch.empty((nr, k), dtype=torch.float32, device="cuda")
            Ir = torch.empty((nr, k), dtype=torch.int64, device="cuda")
            ref.search_device(q.data_ptr(), nr, k, Dr.data_ptr(), Ir.data_ptr(), ctx.stream)
            torch.cuda.synchronize()
            parts_D.append(Dr)
            parts_I.append(Ir)
            del ref
        if prev is None:
            del os.environ["VS_FILTER"]
        else:
            os.environ["VS_FILTER"] = prev
        Dm = torch.empty((nr, k), dtype=torch.float32, device="cuda")
        Im = torch.empty((nr, k), dtype=torch.int64, device="cuda")
        Dall = torch.stack(parts_D).contiguous()
        Iall = torch.stack(parts_I).contiguous()
        ctx.lib.check(ctx.lib.load().vs_merge_topk(
            ctypes.c_void_p(Dall.data_ptr()), ctypes.c_void_p(Iall.data_ptr()), len(parts_D), nr,
            k, k, metric, ctypes.c_void_p(Dm.data_ptr()), ctypes.c_void_p(Im.data_ptr()),
            ctypes.c_void_p(ctx.stream)))
        torch.cuda.synchronize()
        Im = Im.cpu().numpy()
        recall = float(np.mean([len(set(Ig[i]) & set(Im[i])) / k for i in range(nr)]))
    mt = ctx.max_over_ranks(mut_time)
    if ctx.rank == 0:
        res = base_result(args, ctx, args.steps * B / elapsed, elapsed)
        if args.data == "clustered":
            res["data"] = ("synthetic: unit-norm clustered rows (1024 centroids + 0.5 noise, "
                           "torch generator seed 1234; queries noise seed 5678)")
        res["config"] = {"workload": f"C5: {N}x{d} {args.dtype}-stored flat "
                                     f"{'IP' if args.metric == 'ip' else 'L2'}, batch {B}, "
                                     f"top-{k}, 1% remove + 1% append every 10 batches",
                         "ntotal": N, "d": d, "batch": B, "k": k,
                         "parallelism": f"row-shard x{ctx.world} + RCCL all-gather top-k merge",
            "kernel": kname}
        res["roofline"] = rf
        res["recall_at_10_vs_fp32"] = recall
        res["recall_queries"] = args.recall_queries if recall is not None else 0
        res["mutation_seconds_in_timed_region"] = round(mt, 3)
        res["mutation_rounds_remove_append_ms"] = mut_rounds
        res["cpu_baseline"] = None
        return res
    return None


def run_dry(args, ctx):
    """Launcher / collective rehearsal without a GPU (see --dry-run)."""
    torch = ctx.torch
    B, k = max(1, args.batch or 1), args.k
    kin = min(2 * k - 1, 64) if args.metric == "ip" else k
    D = torch.zeros((B, kin), dtype=torch.float32)
    outs = [torch.empty_like(D) for _ in range(ctx.world)]
    elapsed, _, _, _ = ctx.timed(lambda i: ctx.dist.all_gather(outs, D), args.steps, args.warmup)
    if ctx.rank == 0:
        res = base_result(args, ctx, args.steps * B / elapsed, elapsed)
        res["dry_run"] = True
        res["data"] = "none: dry run (gloo all-gather of a (batch, 2k-1) list per step, no kernel)"
        res["config"] = {"workload": f"dry run of {args.workload.upper()}", "batch": B, "k": k,
                         "parallelism": f"row-shard x{ctx.world} (gloo rehearsal)"}
        return res
    return None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    ctx = Ctx(args)
    if args.dry_run:
        res = run_dry(args, ctx)
    elif args.workload in ("c3", "c2"):
        res = run_knn(args, ctx)
        if (args.workload == "c3" and args.data == "uniform" and ctx.world == 1
                and args.clustered_steps > 0 and args.dtype == "f32"):
            # embedding-like rows beside the uniform headline (the headline's
            # index is gone with run_knn's frame): same shape, same engine
            import copy
            import gc

            gc.collect()
            ca = copy.copy(args)
            ca.data, ca.steps, ca.warmup = "clustered", args.clustered_steps, 1
            ca.batch1_steps, ca.wide_k_steps, ca.any_k, ca.no_cpu_baseline = 0, 0, 0, True
            cres = run_knn(ca, ctx)
            if res is not None and cres is not None:
                res["clustered"] = clustered_record(cres)
    elif args.workload == "c4":
        res = run_selfjoin(args, ctx)
    else:
        res = run_c5(args, ctx)
    if ctx.rank == 0 and res is not None:
        print(json.dumps(res), flush=True)
    ctx.dist.barrier()
    ctx.dist.destroy_process_group()


if __name__ == "__main__":
    main()

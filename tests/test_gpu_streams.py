"""GPU: concurrent device-resident searches on two streams of one index.

Per-call scratch comes from a chunk cache shared by every stream (vs_api.hip
Scratch / scratch_chunk_get): a chunk carries the event of its last use and a
taker on another stream waits for it on the device.  Two host threads, each on
its own non-blocking stream, search the same index with different query sets
over and over (the filter engine: int8 -> bf16 -> fp32 stages, many scratch
buffers per search); every result must equal the one-stream result of the same
queries, so a chunk handed across streams before its last use finished shows
up as a wrong list."""

import threading

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def test_two_streams_share_scratch_chunks():
    import torch

    from vsearch import faiss as vfaiss
    from vsearch.synth import synthetic_rows

    n, d, nq, k = 300_000, 1536, 512, 10
    index = vfaiss.IndexFlatIP(d)
    index.add_synthetic(n, seed=77)
    qs = [torch.from_numpy(synthetic_rows(50_000_000 + 10_000 * t, nq, d, 90 + t)).cuda()
          for t in range(2)]
    ref = []
    for q in qs:  # one stream, synchronous: the reference lists
        D, I = index.search(q.cpu().numpy(), k)
        ref.append((D, I))
    errors = []
    barrier = threading.Barrier(2, timeout=60)

    def worker(t):
        try:
            st = torch.cuda.Stream()
            D = torch.empty((nq, k), dtype=torch.float32, device="cuda")
            I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
            barrier.wait()
            for _ in range(12):
                with torch.cuda.stream(st):
                    index.search_device(qs[t].data_ptr(), nq, k, D.data_ptr(), I.data_ptr(),
                                        stream=st.cuda_stream)
                    Ih = I.cpu().numpy()  # ordered after the search on st
                    Dh = D.cpu().numpy()
                if not (Ih == ref[t][1]).all() or not np.allclose(Dh, ref[t][0], rtol=1e-6, atol=0):
                    errors.append((t, int((Ih != ref[t][1]).sum())))
                    return
        except Exception as e:  # pragma: no cover - reported below
            errors.append((t, repr(e)))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    torch.cuda.synchronize()
    assert not errors, errors


def test_writer_of_one_index_does_not_drain_another():
    """Writers wait for their own index's readers only (vs_api.hip ReaderMark /
    wait_readers): remove_ids on a small index A returns while a queue of long
    searches of index B is still running on another stream, and both results
    stay exact.  (Storage growth frees the old buffers with hipFree; the time
    it takes beside B's queue is printed, not asserted.)"""
    import time

    import torch

    from oracle import flat
    from vsearch import faiss as vfaiss
    from vsearch.synth import synthetic_rows

    d, k = 1536, 10
    big = vfaiss.IndexFlatIP(d)
    big.add_synthetic(2_000_000, seed=5)
    xq = torch.from_numpy(synthetic_rows(50_000_000, 4096, d, 6)).cuda()
    D = torch.empty((4096, k), dtype=torch.float32, device="cuda")
    I = torch.empty((4096, k), dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    rng = np.random.default_rng(7)
    xa = rng.standard_normal((20_000, 64)).astype(np.float32)
    small = vfaiss.IndexFlatIP(64)
    small.add(xa)
    small.search(xa[:100], k)  # a reader mark of A's own
    # warm-up: B's search once, timed alone
    with torch.cuda.stream(st):
        big.search_device(xq.data_ptr(), 4096, k, D.data_ptr(), I.data_ptr(), stream=st.cuda_stream)
    st.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(st):
        big.search_device(xq.data_ptr(), 4096, k, D.data_ptr(), I.data_ptr(), stream=st.cuda_stream)
    st.synchronize()
    one = time.perf_counter() - t0
    reps = max(8, int(0.5 / max(one, 1e-3)))
    t0 = time.perf_counter()
    with torch.cuda.stream(st):  # a queue of B searches, ~0.5 s of device work
        for _ in range(reps):
            big.search_device(xq.data_ptr(), 4096, k, D.data_ptr(), I.data_ptr(),
                              stream=st.cuda_stream)
    t_q = time.perf_counter()
    probe = torch.cuda.Stream(priority=-1)  # diagnostic: a high-priority torch stream
    with torch.cuda.stream(probe):
        z = torch.ones(1024, device="cuda") * 2
    probe.synchronize()
    t_probe = time.perf_counter() - t_q
    t_q = time.perf_counter()
    rm = np.arange(0, 20_000, 3, dtype=np.int64)
    assert small.remove_ids(rm) == rm.size
    t_rm = time.perf_counter() - t_q
    t_g = time.perf_counter()
    small.add(xa[:10_000])  # 16,667 + 10,000 rows: past the first capacity -> growth
    t_grow = time.perf_counter() - t_g
    st.synchronize()
    total = time.perf_counter() - t0
    print(f"B queue {reps} x {one * 1e3:.1f} ms = {total * 1e3:.0f} ms; remove_ids on A "
          f"{t_rm * 1e3:.1f} ms; growth of A {t_grow * 1e3:.1f} ms; high-priority torch "
          f"probe {t_probe * 1e3:.1f} ms ({float(z[0])})")
    assert t_rm < 0.25 * reps * one, (t_rm, reps * one)
    # both indexes still exact
    xr, _ = flat.remove_ids(xa, rm)
    xr = np.concatenate([xr, xa[:10_000]])
    Da, Ia = small.search(xa[:300], k)
    Dr, Ir = flat.knn_exact(xr, xa[:300], k, flat.METRIC_INNER_PRODUCT)
    assert not flat.mismatches(Da, Ia, Dr, Ir, flat.METRIC_INNER_PRODUCT, xr, xa[:300], strict=True)
    Db, Ib = big.search(xq[:512].cpu().numpy(), k)
    assert (Ib == I[:512].cpu().numpy()).all()


def test_tail_wait_keeps_device_results(monkeypatch):
    """Device-output searches read their first stage's leftover count and
    enqueue the later stages only when queries remain (vs_api.hip
    tail_wait_on).  With queries beside 200 near-copies of their own direction
    (the int8 checks hand them on: the later stages run) and without (nothing
    left: the search ends after its first stage), the lists equal those of
    VS_TAIL_WAIT=0 (every launch kept) and of the host-output path."""
    import torch

    from vsearch import faiss as vfaiss

    rng = np.random.default_rng(5)
    d = 256
    xb = rng.uniform(-1, 1, (300_000, d)).astype(np.float32)
    hard = rng.uniform(-1, 1, (8, d)).astype(np.float32)
    pos = rng.choice(xb.shape[0], (8, 200), replace=False)
    for j in range(8):
        xb[pos[j]] = (hard[j] * (1.0 + 0.02 * rng.uniform(0, 1, (200, 1)))
                      + 0.01 * rng.standard_normal((200, d))).astype(np.float32)
    index = vfaiss.IndexFlatIP(d)
    index.add(xb)
    st = torch.cuda.Stream()
    for nq, nh in ((512, 8), (512, 0), (16, 3), (1, 0)):
        xq = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
        xq[:nh] = hard[:nh] + 0.01 * rng.standard_normal((nh, d)).astype(np.float32)
        q = torch.from_numpy(xq).cuda()
        out = {}
        for tw in ("1", "0"):
            monkeypatch.setenv("VS_TAIL_WAIT", tw)
            D = torch.empty(nq, 10, device="cuda")
            I = torch.empty(nq, 10, dtype=torch.int64, device="cuda")
            st.wait_stream(torch.cuda.current_stream())  # q's copy
            with torch.cuda.stream(st):
                index.search_device(q.data_ptr(), nq, 10, D.data_ptr(), I.data_ptr(),
                                    stream=st.cuda_stream)
            st.synchronize()
            out[tw] = (D.cpu().numpy(), I.cpu().numpy())
        monkeypatch.delenv("VS_TAIL_WAIT")
        Dh, Ih = index.search(xq, 10)
        for tw in ("1", "0"):
            assert np.array_equal(out[tw][1], Ih), (nq, nh, tw)
            assert np.array_equal(out[tw][0], Dh), (nq, nh, tw)

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

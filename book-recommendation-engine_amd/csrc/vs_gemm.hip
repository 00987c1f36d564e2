// vs_gemm.hip — fused MFMA distance + top-k kernel (large query batches), for
// fp32 rows (v_mfma_f32_32x32x2_f32) and bf16 rows (v_mfma_f32_32x32x16_bf16).
// List semantics and key conventions: vs_device.h / vs_internal.h.
#include "vs_device.h"

namespace vs {

// ---------------------------------------------------------------------------
// GEMM path.
//
// Workgroup = 256 threads (4 waves), tile = 128 database rows x 128 queries.
// Wave w owns queries [32w, 32w+32) of the tile against all 128 rows: four
// 32x32 accumulators (database subtiles s = 0..3).  In v_mfma_f32_32x32x2_f32 the
// A operand is the database row block (row i = lane&31) and the B operand the
// query block (column j = lane&31), so after the K loop lane l holds, for query
// column l&31, the scores of rows (r&3) + 8(r>>2) + 4(l>>5) of each subtile: a
// lane sees one query only, and can keep that query's top-k in its own
// registers with no cross-lane traffic.  Each query therefore owns two lists per
// workgroup (lane halves h = 0, 1); the merge kernel combines them.
//
// K loop: BK = 32 floats per stage, double-buffered in LDS and filled with
// global_load_lds_dwordx4 (no VGPR staging).  An LDS row is 128 B = 8 chunks of
// 16 B; chunk c of row r is stored at c ^ ((r >> 1) & 7), which makes the
// ds_read_b128 fragment reads conflict-free (each 16-lane read group lands on 16
// distinct 16-B slots).  glds writes LDS lane-linearly, so the swizzle is applied
// to the per-lane GLOBAL source address instead.
//
// Fragment k-order: every lane reads one 16-B chunk per operand per step (chunk
// c = 2*step + h of the 128-B stage row).  fp32: the chunk holds 4 floats and
// feeds 4 x32x32x2 MFMAs (instruction t uses k = 4h + t of the 8-wide step);
// bf16: the chunk holds 8 bf16 = exactly the 32x32x16 operand of lane l
// (k = 8h + j).  A and B use the same mapping, so the product is the plain dot
// product; the summation order differs from faiss's sgemm, inside the
// documented fp32 tolerance.  Each stage moves 128 B per row: 32 floats or 64 bf16.
//
// Workgroup -> (query tile, split) mapping is XCD-aware: consecutive logical ids
// (which share a database split and differ in query tile) are packed onto one XCD
// so the 4 MiB L2 there serves each database tile to all query tiles in flight.
//
// FLOOR (KP = 64 only, every metric): the lists admit only entries that come
// strictly after the query's floor (fkey[q], fid[q]) in (key, row) order — page
// p + 1 of a query's lexicographic order starts after page p's last entry
// (vs_api.hip run_paged: any k, and faiss's inner-product tie rule, which reads
// up to 2k - 1 entries).  Every page of a search runs this instantiation (page 1
// with the floor (-inf, -1)), so a row's key is bit-identical in all pages.
template <int KP, int MODE, typename T, bool FLOOR = false>
__global__ __launch_bounds__(256, (KP >= 64 ? 1 : 2)) void gemm_topk(
    const T* __restrict__ X, const float* __restrict__ xaux, const T* __restrict__ Q,
    const float* __restrict__ qaux, int64_t ld, int nstage, int ntotal, int ntiles, int nsplit,
    int nqt, int64_t self0, float* __restrict__ pkey, int* __restrict__ pid,
    const int* __restrict__ qlist, const int* __restrict__ qcount,
    const float* __restrict__ fkey, const int* __restrict__ fid) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 2, "fp32 or bf16 rows");
  // [buf][X|Q][128 rows][128 B]; viewed as floats (32 per row) for addressing.
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * kBN * kBK];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int h = lane >> 5;
  const int c32 = lane & 31;

  // Bijective XCD remap (blocks b and b+8 are dispatched to the same XCD).
  const int nblk = gridDim.x;
  const int b = blockIdx.x;
  int lb;
  {
    const int xcd = b & 7, slot = b >> 3, qq = nblk >> 3, rr = nblk & 7;
    lb = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + slot;
  }
  const int qt = lb % nqt;
  const int sp = lb / nqt;
  const int t0 = (int)((int64_t)sp * ntiles / nsplit);
  const int t1 = (int)((int64_t)(sp + 1) * ntiles / nsplit);

  // gathered batch (the exact redo of flagged queries): slot s is query row
  // qlist[s]; tiles past the device-side count have nothing to do
  const int nf = qlist ? *qcount : 0;
  if (qlist && qt * kBQ >= nf) return;  // uniform
  const int qloc = 32 * w + c32;
  const int gq = qt * kBQ + qloc;
  const int qsrc = qlist ? qlist[min(gq, nf - 1)] : gq;
  float qa = 0.0f;
  if constexpr (MODE == MODE_L2 || MODE == MODE_COS) qa = qaux[qsrc];
  const int selfrow = self0 >= 0 ? (int)(self0 + qsrc) : -1;
  float fk = 0.0f;
  int fi = 0;
  if constexpr (FLOOR) {
    fk = fkey[qsrc];
    fi = fid[qsrc];
  }

  float lk[KP];
  int li[KP];
  list_init<KP, int>(lk, li);

  const T* Qblk = qlist ? Q : Q + (int64_t)qt * kBQ * ld;
  // glds geometry: a wave instruction moves 8 rows x 128 B; wave w stages row
  // groups g = 4w..4w+3 of both operands.  The per-lane source offset is 32-bit
  // on a wave-uniform base (saddr form); the swizzle (row >> 1) & 7 depends on
  // the group only through g & 1, so two lane offsets cover all four groups.
  const int srow = lane >> 3;
  const int sphys = lane & 7;
  const uint32_t ldb = (uint32_t)ld * (uint32_t)sizeof(T);  // row stride in bytes
  uint32_t soff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int row = par * 8 + srow;  // any group with g & 1 == par has this swizzle
    const int c = sphys ^ ((row >> 1) & 7);
    soff[par] = (uint32_t)(w * 32 + srow) * ldb + (uint32_t)c * 16u;
  }
  // query source offsets (per lane): contiguous tile rows, or the gathered rows
  // (64-bit: a gathered row of a 65,536-query batch can sit past 4 GiB of
  // query bytes once d * esize exceeds 64 KiB)
  uint64_t qoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (qlist) {
      const int slot = qt * kBQ + w * 32 + i * 8 + srow;
      const int src = qlist[min(slot, nf - 1)];
      const int row = (w * 4 + i) * 8 + srow;  // the LDS row decides the swizzle
      qoff[i] = (uint64_t)src * ldb + (uint32_t)(sphys ^ ((row >> 1) & 7)) * 16u;
    } else {
      qoff[i] = soff[i & 1] + (uint32_t)(i * 8) * ldb;
    }
  }
  // fragment-read geometry: (row >> 1) & 7 is the same for every subtile.
  const int fsw = (c32 >> 1) & 7;

  for (int t = t0; t < t1; ++t) {
    const char* Xblk = (const char*)(X + (int64_t)t * kBN * ld);
    f32x16 acc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[s][r] = 0.0f;
    }

    auto stage = [&](int buf, int kb) {
      float* dX = smem + buf * (2 * kBN * kBK);
      float* dQ = dX + kBN * kBK;
      const char* xs = Xblk + kb;
      const char* qs = (const char*)Qblk + kb;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int g = w * 4 + i;
        const uint32_t o = soff[i & 1] + (uint32_t)(i * 8) * ldb;
        __builtin_amdgcn_global_load_lds(xs + o, VS_LDS(dX + g * 256), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(qs + qoff[i], VS_LDS(dQ + g * 256), 16, 0, 0);
      }
    };

    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int st = 0; st < nstage; ++st) {
      if (st + 1 < nstage) stage((st + 1) & 1, (st + 1) * 128);
      const float* cX = smem + (st & 1) * (2 * kBN * kBK);
      const float* cQ = cX + kBN * kBK;
#pragma unroll
      for (int kc = 0; kc < 4; ++kc) {
        const int coff = ((kc * 2 + h) ^ fsw) * 4;
        const f32x4 bq = *(const f32x4*)(cQ + qloc * kBK + coff);
        f32x4 ax[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) ax[s] = *(const f32x4*)(cX + (32 * s + c32) * kBK + coff);
        if constexpr (sizeof(T) == 4) {
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
              acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(ax[s][tt], bq[tt], acc[s], 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s)
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ax[s]),
                                                            __builtin_bit_cast(bf16x8, bq),
                                                            acc[s], 0, 0, 0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }

    // Epilogue, one 32-row subtile at a time.  Phase A (unrolled, branch-free):
    // scores -> keys, and a 16-bit mask of the values that beat the lane's
    // current worst entry (the threshold only tightens while inserting, so the
    // value it had at the start of the subtile admits a superset).  Phase B (rare
    // after the first tiles): the lane parks the 16 keys in a private column of
    // the (now idle) staging LDS and inserts the flagged ones, so the insertion
    // code exists once per subtile instead of once per value.
    const int r0 = t * kBN;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float tk = lk[KP - 1];
      const int ti = li[KP - 1];
      uint32_t m = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rb = r0 + 32 * s + 8 * j + 4 * h;
        f32x4 xa = {0.f, 0.f, 0.f, 0.f};
        if constexpr (MODE == MODE_L2 || MODE == MODE_COS) xa = *(const f32x4*)(xaux + rb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = rb + i;
          const float v = acc[s][j * 4 + i];
          float key;
          if constexpr (MODE == MODE_IP) {
            key = -v;
          } else if constexpr (MODE == MODE_L2) {
            key = l2_from_ip(qa, xa[i], v);
          } else {
            key = -(v * (qa * xa[i]));
          }
          acc[s][j * 4 + i] = key;
          bool cand = row < ntotal && row != selfrow && lex_less(key, row, tk, ti);
          if constexpr (FLOOR) cand = cand && lex_less(fk, fi, key, row);
          m |= (uint32_t)cand << (j * 4 + i);
        }
      }
      if (m) {
#pragma unroll
        for (int r = 0; r < 16; ++r) smem[r * 256 + tid] = acc[s][r];
        do {
          const int bi = __builtin_ctz(m);
          m &= m - 1;
          const int row = r0 + 32 * s + (bi & 3) + 8 * (bi >> 2) + 4 * h;
          list_insert<KP, int>(lk, li, smem[bi * 256 + tid], row);
        } while (m);
      }
    }
    // The next tile's first stage overwrites the LDS the epilogue may have used.
    __syncthreads();
  }

  const int P = nsplit * 2;
  float* ok = pkey + ((int64_t)gq * P + sp * 2 + h) * KP;
  int* oi = pid + ((int64_t)gq * P + sp * 2 + h) * KP;
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    ok[j] = lk[j];
    oi[j] = li[j];
  }
}

template <int KP, int MODE, bool FLOOR = false>
static hipError_t gemm_dispatch_mode(const void* X, const float* xaux, const void* Q,
                                     const float* qaux, int64_t ld, int esize, int ntotal,
                                     int nq_pad, int nsplit, int64_t self0, Partials part,
                                     hipStream_t st, const int* qlist, const int* qcount,
                                     const float* fkey = nullptr, const int* fid = nullptr) {
  const int ntiles = (ntotal + kBN - 1) / kBN;
  const int nqt = nq_pad / kBQ;
  const int nblk = nqt * nsplit;
  const int nstage = (int)(ld * esize / 128);
  if (esize == 4)
    hipLaunchKernelGGL((gemm_topk<KP, MODE, float, FLOOR>), dim3(nblk), dim3(256), 0, st,
                       (const float*)X, xaux, (const float*)Q, qaux, ld, nstage, ntotal, ntiles,
                       nsplit, nqt, self0, part.key, part.id, qlist, qcount, fkey, fid);
  else
    hipLaunchKernelGGL((gemm_topk<KP, MODE, uint16_t, FLOOR>), dim3(nblk), dim3(256), 0, st,
                       (const uint16_t*)X, xaux, (const uint16_t*)Q, qaux, ld, nstage, ntotal,
                       ntiles, nsplit, nqt, self0, part.key, part.id, qlist, qcount, fkey, fid);
  return hipGetLastError();
}

template <int KP>
static hipError_t gemm_dispatch(int mode, const void* X, const float* xaux, const void* Q,
                                const float* qaux, int64_t ld, int esize, int ntotal, int nq_pad,
                                int nsplit, int64_t self0, Partials part, hipStream_t st,
                                const int* qlist, const int* qcount) {
  switch (mode) {
    case MODE_IP:
      return gemm_dispatch_mode<KP, MODE_IP>(X, xaux, Q, qaux, ld, esize, ntotal, nq_pad, nsplit, self0,
                                             part, st, qlist, qcount);
    case MODE_L2:
      return gemm_dispatch_mode<KP, MODE_L2>(X, xaux, Q, qaux, ld, esize, ntotal, nq_pad, nsplit, self0,
                                             part, st, qlist, qcount);
    case MODE_COS:
      return gemm_dispatch_mode<KP, MODE_COS>(X, xaux, Q, qaux, ld, esize, ntotal, nq_pad,
                                              nsplit, self0, part, st, qlist, qcount);
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_gemm_topk(int KP, int mode, const void* X, const float* xaux, const void* Q,
                            const float* qaux, int64_t ld, int esize, int ntotal, int nq_pad,
                            int nsplit, int64_t self0, Partials part, hipStream_t st,
                            const int* qlist, const int* qcount, const float* fkey,
                            const int* fid) {
  if (nq_pad % kBQ != 0 || (ld * esize) % 128 != 0 || part.KP != KP || part.P != 2 * nsplit ||
      (esize != 4 && esize != 2) || ((qlist == nullptr) != (qcount == nullptr)) ||
      ((fkey == nullptr) != (fid == nullptr)))
    return hipErrorInvalidValue;
  if (fkey) {  // a page after a floor (the paged engine, 64-entry lists)
    if (KP != 64) return hipErrorInvalidValue;
    switch (mode) {
      case MODE_IP:
        return gemm_dispatch_mode<64, MODE_IP, true>(X, xaux, Q, qaux, ld, esize, ntotal, nq_pad,
                                                     nsplit, self0, part, st, qlist, qcount, fkey,
                                                     fid);
      case MODE_L2:
        return gemm_dispatch_mode<64, MODE_L2, true>(X, xaux, Q, qaux, ld, esize, ntotal, nq_pad,
                                                     nsplit, self0, part, st, qlist, qcount, fkey,
                                                     fid);
      case MODE_COS:
        return gemm_dispatch_mode<64, MODE_COS, true>(X, xaux, Q, qaux, ld, esize, ntotal, nq_pad,
                                                      nsplit, self0, part, st, qlist, qcount, fkey,
                                                      fid);
      default:
        return hipErrorInvalidValue;
    }
  }
  switch (KP) {
    case 8:
      return gemm_dispatch<8>(mode, X, xaux, Q, qaux, ld, esize, ntotal, nq_pad, nsplit, self0, part, st, qlist, qcount);
    case 16:
      return gemm_dispatch<16>(mode, X, xaux, Q, qaux, ld, esize, ntotal, nq_pad, nsplit, self0, part, st, qlist, qcount);
    case 32:
      return gemm_dispatch<32>(mode, X, xaux, Q, qaux, ld, esize, ntotal, nq_pad, nsplit, self0, part, st, qlist, qcount);
    case 64:
      return gemm_dispatch<64>(mode, X, xaux, Q, qaux, ld, esize, ntotal, nq_pad, nsplit, self0, part, st, qlist, qcount);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace vs

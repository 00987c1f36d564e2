// The held-clock MFMA ceiling at the filter pass's occupancy (VERDICT r04
// "next" 2): one workgroup of 8 waves per CU (two per SIMD, 160 KB of LDS
// declared so no second workgroup fits), every wave issuing the filter
// kernel's 16 MFMAs per step into 8 32x32 accumulators — and nothing else: no
// loads, no LDS, no barriers.  What it reaches is the most the filter kernel's
// tile can reach on this chip at the clock the chip holds under MFMA load;
// bench.py's roofline fraction against the nominal peak reads against it.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_ceiling tools/mfma_ceiling.hip
//   tools/mfma_ceiling            # prints one JSON line per plane
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int kLds = 160 * 1024;

template <bool I8>
__global__ __launch_bounds__(512) void mfma_loop(int iters, int* out) {
  extern __shared__ char lds[];  // occupancy only: never touched
  (void)lds;
  const int lane = threadIdx.x & 63;
  i32x4 a = {lane, lane * 3, lane * 5, lane * 7};
  i32x4 b = {lane * 11, lane * 13, lane * 17, lane * 19};
  if constexpr (I8) {
    i32x16 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = i32x16{};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[j], 0, 0, 0);
    }
    int r = 0;
    for (int j = 0; j < 8; ++j)
      for (int e = 0; e < 16; ++e) r ^= acc[j][e];
    if (r == 0x7fffffff) out[blockIdx.x] = r;  // keeps the loop; never true in practice
  } else {
    f32x16 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = f32x16{};
    const bf16x8 ab = __builtin_bit_cast(bf16x8, a), bb = __builtin_bit_cast(bf16x8, b);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, acc[j], 0, 0, 0);
    }
    float r = 0.f;
    for (int j = 0; j < 8; ++j)
      for (int e = 0; e < 16; ++e) r += acc[j][e];
    if (r == 1.2345f) out[blockIdx.x] = 1;
  }
}

template <bool I8>
void run(int cus, int iters, double peak) {
  int* out = nullptr;
  CHECK(hipMalloc(&out, sizeof(int) * cus));
  CHECK(hipFuncSetAttribute((const void*)mfma_loop<I8>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  mfma_loop<I8><<<cus, 512, kLds>>>(iters / 10, out);  // warm the clock
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f, sum = 0.f;
  const int reps = 5;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0));
    mfma_loop<I8><<<cus, 512, kLds>>>(iters, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
    sum += ms;
  }
  // per wave and iteration: 16 MFMAs of 32x32 outputs x K (32 int8 / 16 bf16), 2 ops per MAC
  const double ops = (double)cus * 8 * iters * 16 * 32.0 * 32.0 * (I8 ? 32 : 16) * 2;
  const double mean = sum / reps;
  // cycles per step and SIMD at 2.4 GHz nominal: two waves x 16 MFMAs
  printf("{\"plane\": \"%s\", \"cus\": %d, \"iters\": %d, \"mean_ms\": %.3f, \"best_ms\": %.3f, "
         "\"tops_mean\": %.1f, \"peak_tops\": %.1f, \"frac_of_peak\": %.4f, "
         "\"implied_clock_ghz\": %.3f}\n",
         I8 ? "int8" : "bf16", cus, iters, mean, best, ops / (mean * 1e-3) / 1e12, peak,
         ops / (mean * 1e-3) / 1e12 / peak, 2.4 * ops / (mean * 1e-3) / 1e12 / peak);
  CHECK(hipFree(out));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  run<true>(cus, iters, 5000.0);
  run<false>(cus, iters, 2500.0);
  return 0;
}

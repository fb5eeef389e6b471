// Philox4x32-10 throughput ceiling on gfx950: the compute roof of the
// draw-stream kernel (bench.py "compute_roofline").  Every lane runs
// independent Philox blocks back to back (10 rounds, 2 v_mad_u64_u32 + 4 xor
// per round, key schedule in SGPRs) and folds the four words into a
// compare-count so nothing is dead code.  Prints one JSON line.
//
//   hipcc --offload-arch=gfx950 -O3 tools/philox_peak.hip -o tools/philox_peak && tools/philox_peak
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__global__ void __launch_bounds__(256) philox_blocks(uint32_t *out, int iters, uint32_t k0, uint32_t k1) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    uint32_t a = t, b = 0, c = (uint32_t)i, d = 0, kk0 = k0, kk1 = k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * a, p1 = (uint64_t)0xCD9E8D57u * c;
      const uint32_t n0 = (uint32_t)(p1 >> 32) ^ b ^ kk0, n2 = (uint32_t)(p0 >> 32) ^ d ^ kk1;
      a = n0; b = (uint32_t)p1; c = n2; d = (uint32_t)p0;
      kk0 += 0x9E3779B9u; kk1 += 0xBB67AE85u;
    }
    acc += (a < 123456u) + (b < 123456u) + (c < 123456u) + (d < 123456u);
  }
  out[t] = acc;
}

int main() {
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int blocks = pr.multiProcessorCount * 32, iters = 512;
  uint32_t *out;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    CK(hipEventRecord(e0));
    philox_blocks<<<blocks, 256>>>(out, iters, 1u, 2u);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;  // rep 0 warms up
  }
  const double n = (double)blocks * 256 * iters;
  printf("{\"device\": \"%s\", \"cus\": %d, \"philox_blocks_per_s\": %.6e, \"draws_per_s\": %.6e, \"ms\": %.4f, "
         "\"blocks\": %.0f}\n",
         pr.gcnArchName, pr.multiProcessorCount, n / (best * 1e-3), 4 * n / (best * 1e-3), best, n);
  CK(hipFree(out));
  return 0;
}

// Philox4x32-10 throughput ceiling on gfx950: the compute roof of the
// draw-stream kernel (bench.py "compute_roofline").  Every lane runs
// independent Philox blocks back to back (10 rounds, 2 v_mad_u64_u32 per
// round, key schedule in SGPRs) and folds the four words into a
// compare-count so nothing is dead code.  Variants:
//   xor2   : the two xors of a round as two v_xor_b32 (what plain C compiles to)
//   bitop3 : one gfx950 v_bitop3_b32 (LUT 0x96 = a^b^c) per output word
//   mullohi: bitop3, with v_mul_hi_u32 + v_mul_lo_u32 instead of v_mad_u64_u32
// each at 1 and 2 independent chains per lane.  The peak is the best variant.
// Prints one JSON line.
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

template <int V>
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  if constexpr (V == 0) return a ^ b ^ c;
  else return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

template <int V>
__device__ __forceinline__ void mul(uint32_t m, uint32_t x, uint32_t &hi, uint32_t &lo) {
  if constexpr (V == 2) {
    hi = __umulhi(m, x);
    lo = m * x;
  } else {
    const uint64_t p = (uint64_t)m * x;
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
  }
}

template <int V, int CH>
__global__ void __launch_bounds__(256) philox_blocks(uint32_t *out, int iters, uint32_t k0, uint32_t k1) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    uint32_t a[CH], b[CH], c[CH], d[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      a[u] = t * CH + u;
      b[u] = 0;
      c[u] = (uint32_t)i;
      d[u] = 0;
    }
    uint32_t kk0 = k0, kk1 = k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        uint32_t h0, l0, h1, l1;
        mul<V>(0xD2511F53u, a[u], h0, l0);
        mul<V>(0xCD9E8D57u, c[u], h1, l1);
        a[u] = x3<V>(h1, b[u], kk0);
        c[u] = x3<V>(h0, d[u], kk1);
        b[u] = l1;
        d[u] = l0;
      }
      kk0 += 0x9E3779B9u;
      kk1 += 0xBB67AE85u;
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) acc += (a[u] < 123456u) + (b[u] < 123456u) + (c[u] < 123456u) + (d[u] < 123456u);
  }
  out[t] = acc;
}

template <int V, int CH>
static int run(const hipDeviceProp_t &pr, uint32_t *out, double &rate) {
  const int blocks = pr.multiProcessorCount * 32, iters = 512 / CH;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    CK(hipEventRecord(e0));
    philox_blocks<V, CH><<<blocks, 256>>>(out, iters, 1u, 2u);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;  // rep 0 warms up
  }
  rate = (double)blocks * 256 * iters * CH / (best * 1e-3);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return 0;
}

int main() {
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  uint32_t *out;
  CK(hipMalloc(&out, (size_t)pr.multiProcessorCount * 32 * 256 * 4));
  double r[6];
  if (run<0, 1>(pr, out, r[0]) || run<0, 2>(pr, out, r[1]) || run<1, 1>(pr, out, r[2]) ||
      run<1, 2>(pr, out, r[3]) || run<2, 1>(pr, out, r[4]) || run<2, 2>(pr, out, r[5]))
    return 1;
  double best = 0;
  for (double x : r) best = x > best ? x : best;
  printf("{\"device\": \"%s\", \"cus\": %d, \"philox_blocks_per_s\": %.6e, \"draws_per_s\": %.6e, "
         "\"variants\": {\"xor2_1\": %.4e, \"xor2_2\": %.4e, \"bitop3_1\": %.4e, \"bitop3_2\": %.4e, "
         "\"mullohi_1\": %.4e, \"mullohi_2\": %.4e}}\n",
         pr.gcnArchName, pr.multiProcessorCount, best, 4 * best, r[0], r[1], r[2], r[3], r[4], r[5]);
  CK(hipFree(out));
  return 0;
}

// Probe (diagnostic, not product): issue cost of v_pk_fma_f32 against two v_fma_f32 on gfx950, one wave
// alone and two waves per SIMD: 8 independent accumulator chains, 512 steps, s_memtime around the loop.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));

template <bool kPacked>
__global__ void k_issue(float* out, unsigned long long* cyc, float a0) {
  v2f acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = v2f{a0 + i, a0 - i};
  const v2f m = v2f{1.0001f, 0.9999f}, c = v2f{0.5f, 0.25f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int s = 0; s < 512; ++s) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (kPacked) {
        acc[i] = __builtin_elementwise_fma(acc[i], m, c);
      } else {
        acc[i].x = __builtin_fmaf(acc[i].x, m.x, c.x);
        acc[i].y = __builtin_fmaf(acc[i].y, m.y, c.y);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  for (int i = 0; i < 8; ++i) r += acc[i].x + acc[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 4096 * 64 * 4);
  (void)hipMalloc(&cyc, 4096 * 8);
  unsigned long long h[4096];
  for (int waves_per_simd : {1, 2}) {
    const int nb = 1024 * waves_per_simd;  // 1024 SIMDs
    for (int packed = 0; packed < 2; ++packed) {
      for (int rep = 0; rep < 2; ++rep) {
        if (packed) k_issue<true><<<nb, 64>>>(out, cyc, 1.f);
        else k_issue<false><<<nb, 64>>>(out, cyc, 1.f);
        (void)hipDeviceSynchronize();
      }
      (void)hipMemcpy(h, cyc, nb * 8, hipMemcpyDeviceToHost);
      double s = 0;
      for (int b = 0; b < nb; ++b) s += (double)h[b];
      const double per = s / nb / (512.0 * 8);
      printf("waves/SIMD %d %s: %.2f cycles per step of 2 fp32 FMAs (8 independent chains)\n", waves_per_simd,
             packed ? "v_pk_fma_f32" : "2x v_fma_f32", per);
    }
  }
  return 0;
}

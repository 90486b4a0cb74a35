// Probe (diagnostic, not product): layout and numerics of v_mfma_f32_32x32x1_2b_f32 on gfx950.
// 1) layout: two K steps, A = la + 1 then 1, B = 1 then 100 (lb + 1): D = (la + 1) + 100 (lb + 1)
//    decodes which A lane / B lane feed each (register, lane) of D.
// 2) numerics: 27 K steps of random data vs an fmaf chain over k ascending in the decoded layout.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
typedef float f32x32 __attribute__((ext_vector_type(32)));

__global__ void k_layout(float* out) {
  const int l = threadIdx.x;
  f32x32 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x1f32((float)(l + 1), 1.0f, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x1f32(1.0f, 100.0f * (float)(l + 1), c, 0, 0, 0);
  for (int v = 0; v < 32; ++v) out[v * 64 + l] = c[v];
}

__global__ void k_chain(const float* a, const float* b, float* out, int K) {
  const int l = threadIdx.x;
  f32x32 c = {};
  for (int k = 0; k < K; ++k) c = __builtin_amdgcn_mfma_f32_32x32x1f32(a[k * 64 + l], b[k * 64 + l], c, 0, 0, 0);
  for (int v = 0; v < 32; ++v) out[v * 64 + l] = c[v];
}

int main() {
  float *d_out, *d_a, *d_b;
  const int K = 27;
  hipMalloc(&d_out, 32 * 64 * 4);
  hipMalloc(&d_a, K * 64 * 4);
  hipMalloc(&d_b, K * 64 * 4);
  float out[32 * 64];
  k_layout<<<1, 64>>>(d_out);
  hipMemcpy(out, d_out, sizeof(out), hipMemcpyDeviceToHost);
  int la_of[32][64], lb_of[32][64], bad = 0;
  for (int v = 0; v < 32; ++v)
    for (int l = 0; l < 64; ++l) {
      int x = (int)out[v * 64 + l];
      int lb = x / 100 - 1, la = x % 100 - 1;
      la_of[v][l] = la; lb_of[v][l] = lb;
      // hypothesis: block = v / 16 (A, B lanes of that block), j = l % 32 (B lane), i = 8 ((v % 16) / 4) + 4 (l / 32) + v % 4
      int blk = v / 16, j = l % 32, i = 8 * ((v % 16) / 4) + 4 * (l / 32) + v % 4;
      if (la != 32 * blk + i || lb != 32 * blk + j) {
        if (bad < 8) printf("layout mismatch v=%d l=%d: A lane %d B lane %d (hyp %d %d)\n", v, l, la, lb, 32 * blk + i, 32 * blk + j);
        ++bad;
      }
    }
  printf("layout: %d mismatches vs hypothesis (block=v/16, row i=8((v%%16)/4)+4(l/32)+v%%4, col j=l%%32)\n", bad);
  float a[K * 64], b[K * 64];
  srand(7);
  int nbad = 0;
  for (int trial = 0; trial < 50; ++trial) {
    for (int t = 0; t < K * 64; ++t) {
      a[t] = ((float)rand() / RAND_MAX - 0.5f) * powf(2.f, (float)(rand() % 20 - 10));
      b[t] = ((float)rand() / RAND_MAX - 0.5f) * powf(2.f, (float)(rand() % 20 - 10));
      if (rand() % 9 == 0) a[t] = 0.f;
      if (rand() % 13 == 0) b[t] = -0.f;
    }
    hipMemcpy(d_a, a, sizeof(a), hipMemcpyHostToDevice);
    hipMemcpy(d_b, b, sizeof(b), hipMemcpyHostToDevice);
    k_chain<<<1, 64>>>(d_a, d_b, d_out, K);
    hipMemcpy(out, d_out, sizeof(out), hipMemcpyDeviceToHost);
    for (int v = 0; v < 32; ++v)
      for (int l = 0; l < 64; ++l) {
        float acc = 0.f;
        for (int k = 0; k < K; ++k) acc = fmaf(a[k * 64 + la_of[v][l]], b[k * 64 + lb_of[v][l]], acc);
        uint32_t x, y;
        memcpy(&x, &acc, 4);
        memcpy(&y, &out[v * 64 + l], 4);
        if (x != y) {
          if (nbad < 8) printf("numerics mismatch trial %d v=%d l=%d: fmaf chain %.9g mfma %.9g\n", trial, v, l, acc, out[v * 64 + l]);
          ++nbad;
        }
      }
  }
  printf("numerics: %d of %d outputs differ from the host fmaf chain (50 trials, K=%d)\n", nbad, 50 * 32 * 64, K);
  return (bad || nbad) ? 1 : 0;
}

// Probe (diagnostic, not product): layout and numerics of v_mfma_f32_32x32x2_f32 (single block,
// K = 2 per instruction) on gfx950.  Layout as mfma_2b_probe; numerics: S instructions of random
// data (and of 0/1 B operands, the subtree-sum use) against four accumulation hypotheses per
// instruction: H1 fma(a1,b1,fma(a0,b0,c)), H2 fma(a0,b0,fma(a1,b1,c)), H3 one rounding of
// a0 b0 + a1 b1 + c (double), H4 (a0 b0 + a1 b1 rounded) + c.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <cstdint>
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_layout(float* out) {
  const int l = threadIdx.x;
  f32x16 c = {};
  // A = lane + 1, B = 100 (lane + 1) * [k == lane/32]: D[i][j] = sum_k A[i][k] B[k][j]
  c = __builtin_amdgcn_mfma_f32_32x32x2f32((float)(l + 1), 100.0f * (float)(l + 1), c, 0, 0, 0);
  for (int v = 0; v < 16; ++v) out[v * 64 + l] = c[v];
}

__global__ void k_chain(const float* a, const float* b, float* out, int S) {
  const int l = threadIdx.x;
  f32x16 c = {};
  for (int s = 0; s < S; ++s) c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s * 64 + l], b[s * 64 + l], c, 0, 0, 0);
  for (int v = 0; v < 16; ++v) out[v * 64 + l] = c[v];
}

static uint32_t bits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }

int main() {
  float *d_out, *d_a, *d_b;
  const int S = 12;
  hipMalloc(&d_out, 16 * 64 * 4);
  hipMalloc(&d_a, S * 64 * 4);
  hipMalloc(&d_b, S * 64 * 4);
  float out[16 * 64];
  k_layout<<<1, 64>>>(d_out);
  hipMemcpy(out, d_out, sizeof(out), hipMemcpyDeviceToHost);
  // hypothesis: A lane for (i, k) = i + 32 k, B lane for (k, j) = j + 32 k, D[i][j] at v, l with
  // i = 8 (v / 4) + 4 (l / 32) + v % 4, j = l % 32
  int bad = 0;
  for (int v = 0; v < 16; ++v)
    for (int l = 0; l < 64; ++l) {
      const int i = 8 * (v / 4) + 4 * (l / 32) + v % 4, j = l % 32;
      double want = 0.0;
      for (int k = 0; k < 2; ++k) want += (double)(i + 32 * k + 1) * 100.0 * (double)(j + 32 * k + 1);
      if ((double)out[v * 64 + l] != (float)want) {
        if (bad < 6) printf("layout mismatch v=%d l=%d got %.1f want %.1f\n", v, l, out[v * 64 + l], want);
        ++bad;
      }
    }
  printf("layout: %d mismatches vs hypothesis\n", bad);
  float a[S * 64], b[S * 64];
  for (int mode = 0; mode < 2; ++mode) {
    srand(11 + mode);
    long nh[4] = {0, 0, 0, 0}, tot = 0;
    for (int trial = 0; trial < 40; ++trial) {
      for (int t = 0; t < S * 64; ++t) {
        a[t] = ((float)rand() / RAND_MAX - 0.5f) * powf(2.f, (float)(rand() % 24 - 12));
        b[t] = mode == 0 ? ((float)rand() / RAND_MAX - 0.5f) * powf(2.f, (float)(rand() % 24 - 12))
                         : (float)(rand() & 1);
      }
      hipMemcpy(d_a, a, sizeof(a), hipMemcpyHostToDevice);
      hipMemcpy(d_b, b, sizeof(b), hipMemcpyHostToDevice);
      k_chain<<<1, 64>>>(d_a, d_b, d_out, S);
      hipMemcpy(out, d_out, sizeof(out), hipMemcpyDeviceToHost);
      for (int v = 0; v < 16; ++v)
        for (int l = 0; l < 64; ++l) {
          const int i = 8 * (v / 4) + 4 * (l / 32) + v % 4, j = l % 32;
          float h[4] = {0.f, 0.f, 0.f, 0.f};
          for (int s = 0; s < S; ++s) {
            const float a0 = a[s * 64 + i], a1 = a[s * 64 + 32 + i], b0 = b[s * 64 + j], b1 = b[s * 64 + 32 + j];
            h[0] = fmaf(a1, b1, fmaf(a0, b0, h[0]));
            h[1] = fmaf(a0, b0, fmaf(a1, b1, h[1]));
            h[2] = (float)((double)a0 * b0 + (double)a1 * b1 + (double)h[2]);
            h[3] = (float)((double)a0 * b0 + (double)a1 * b1) + h[3];
          }
          for (int q = 0; q < 4; ++q) nh[q] += bits(h[q]) == bits(out[v * 64 + l]);
          ++tot;
        }
    }
    printf("%s B: outputs matching H1 %ld, H2 %ld, H3 %ld, H4 %ld of %ld\n", mode == 0 ? "random" : "0/1", nh[0], nh[1],
           nh[2], nh[3], tot);
  }
  return bad ? 1 : 0;
}

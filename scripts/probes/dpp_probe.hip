// Probe (diagnostic, not product): DPP row_newbcast:n (dpp_ctrl 0x150 + n) and v_permlane16_swap on
// gfx950 -- the PGS gather of one lane's value to its 32-lane half.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  const int l = threadIdx.x;
  const int b3 = __builtin_amdgcn_update_dpp(0, l, 0x150 + 3, 0xF, 0xF, false);
  const int b12 = __builtin_amdgcn_update_dpp(0, l, 0x150 + 12, 0xF, 0xF, false);
  const auto p = __builtin_amdgcn_permlane16_swap(b3, b3, false, false);
  out[l] = b3; out[64 + l] = b12; out[128 + l] = p[0]; out[192 + l] = p[1];
}
int main() {
  int* d; int h[256];
  (void)hipMalloc(&d, sizeof(h));
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    const int row = l / 16, half = l / 32;
    if (h[l] != 16 * row + 3) ++bad;
    if (h[64 + l] != 16 * row + 12) ++bad;
    if (h[128 + l] != 32 * half + 3) ++bad;       // row 0 of the half's value everywhere
    if (h[192 + l] != 32 * half + 16 + 3) ++bad;  // row 1 of the half's value everywhere
  }
  for (int t = 0; t < 4; ++t) { for (int l = 0; l < 64; l += 8) printf("%d ", h[64 * t + l]); printf("\n"); }
  printf("dpp probe: %d mismatches\n", bad);
  return bad != 0;
}

// Traffic calibration for roofline.traffic (DESIGN.md §3 "Traffic"): rocprofv3's FETCH_SIZE / WRITE_SIZE
// are calibrated on gfx950 only for 16-B-per-lane streaming accesses (MI355X_MICROARCH.md, "HBM").
// k_step touches its state with a different pattern: field-major [field][N] rows, two envs per 64-lane
// wave, lane k of env half h reading / writing field k of env 2b + h (4 B per lane, an 8-B run per field
// row per wave), workgroups spread over the XCDs by xcd_block, the state updated in place and the same
// buffers reused launch after launch.  This probe moves a KNOWN byte count with exactly that pattern and,
// for comparison, with the calibrated streaming pattern, so the counters can be converted to bytes:
//   k_pattern<1>: k_step's pattern (xcd_block mapping), F fields x N envs, read + write in place
//   k_pattern<0>: the same without the XCD remap (workgroup b -> envs 2b, 2b + 1)
//   k_stream:     16 B per lane, grid-stride, read + write in place, same bytes
//   k_wonly_field<1>: k_step's pattern, stores only (a buffer the kernel never reads: the side buffer,
//                 body_pos, rewards) -- known read bytes 0, so any FETCH_SIZE is fill traffic
//   k_wonly_rows: env-major 59-float rows (the observation), two envs per wave, stores only
// Each kernel runs `reps` times back to back on the same buffers (the bench's regime).  Run under
//   rocprofv3 --pmc FETCH_SIZE  and  rocprofv3 --pmc WRITE_SIZE   (separate passes)
// and reduce with scripts/traffic_calib.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

// the same mapping as csrc/allsteps_kernels.hip xcd_block
__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, slot = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + slot;
}

template <int kRemap>
__global__ __launch_bounds__(64) void k_pattern(float* st, int n, int nf) {
  const int el = threadIdx.x >> 5, lane = threadIdx.x & 31;
  const int pair = kRemap ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int e = pair * 2 + el;
  if (e >= n) return;
  for (int f = lane; f < nf; f += 32) {
    const float v = st[(size_t)f * n + e];
    st[(size_t)f * n + e] = v * 0.5f + 1.0f;
  }
}

template <int kRemap>
__global__ __launch_bounds__(64) void k_wonly_field(float* out, int n, int nf) {
  const int el = threadIdx.x >> 5, lane = threadIdx.x & 31;
  const int pair = kRemap ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int e = pair * 2 + el;
  if (e >= n) return;
  for (int f = lane; f < nf; f += 32) out[(size_t)f * n + e] = (float)(f + e);
}

__global__ __launch_bounds__(64) void k_wonly_rows(float* out, int n) {
  const int el = threadIdx.x >> 5, lane = threadIdx.x & 31;
  const int e = xcd_block(blockIdx.x, gridDim.x) * 2 + el;
  if (e >= n) return;
  float* row = out + (size_t)e * 59;
  row[lane] = (float)lane;
  if (lane < 59 - 32) row[32 + lane] = (float)(lane + 32);
}

__global__ __launch_bounds__(256) void k_stream(float4* st, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = st[i];
    v.x = v.x * 0.5f + 1.0f; v.y = v.y * 0.5f + 1.0f; v.z = v.z * 0.5f + 1.0f; v.w = v.w * 0.5f + 1.0f;
    st[i] = v;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 4096;
  const int nf = argc > 2 ? std::atoi(argv[2]) : 32;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 20;
  if (n <= 0 || n % 2 || nf <= 0 || nf > 256 || ((size_t)n * nf) % 4) {
    std::fprintf(stderr, "bad sizes n=%d nf=%d\n", n, nf);
    return 2;
  }
  const size_t count = (size_t)n * nf;
  float* st = nullptr;
  CHECK(hipMalloc(&st, count * sizeof(float)));
  CHECK(hipMemset(st, 0, count * sizeof(float)));
  const int blocks = n / 2;
  for (int r = 0; r < reps; ++r) k_pattern<1><<<blocks, 64>>>(st, n, nf);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  for (int r = 0; r < reps; ++r) k_pattern<0><<<blocks, 64>>>(st, n, nf);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  const size_t n4 = count / 4;
  const int sb = (int)((n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048);
  for (int r = 0; r < reps; ++r) k_stream<<<sb, 256>>>(reinterpret_cast<float4*>(st), n4);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float* wo = nullptr;
  const size_t wcount = (size_t)n * (nf > 59 ? nf : 59);
  CHECK(hipMalloc(&wo, wcount * sizeof(float)));
  for (int r = 0; r < reps; ++r) k_wonly_field<1><<<blocks, 64>>>(wo, n, nf);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  for (int r = 0; r < reps; ++r) k_wonly_rows<<<blocks, 64>>>(wo, n);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  CHECK(hipFree(wo));
  std::printf("{\"n\": %d, \"fields\": %d, \"reps\": %d, \"bytes_read\": %zu, \"bytes_written\": %zu, "
              "\"wonly_field_bytes\": %zu, \"wonly_rows_bytes\": %zu}\n", n, nf, reps, count * sizeof(float),
              count * sizeof(float), count * sizeof(float), (size_t)n * 59 * sizeof(float));
  CHECK(hipFree(st));
  return 0;
}

// ppo_kernels.hip -- the non-GEMM half of one PPO minibatch step (include/ppo.h), gfx950.
//
// Restates rl_games 1.6.1 (absent offline): a2c_continuous.py calc_gradients
// (actor_loss / critic_loss / bound_loss / entropy, policy_kl, update_mu_sigma), running_mean_std.py
// (train-mode update + normalise), torch clip_grad_norm_ + torch.optim.Adam, schedulers.py
// AdaptiveScheduler.  Gradients are the analytic derivatives of those losses (the autograd graph of
// the reference reduces to them); tests/test_gpu_learning.py checks them against torch autograd.
//
// Everything is deterministic (fixed-order block partials, no float atomics), so ranks that replay
// the same update on the same data stay bit-identical (multi_gpu_mode allgather).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "ppo.h"
#include "ppo_loss.h"

namespace {

thread_local char g_err[256] = "";

int fail(int code, const char* what) {
    snprintf(g_err, sizeof(g_err), "%s", what);
    return code;
}

}  // namespace

namespace ppo_detail {
void set_error(const char* msg) { snprintf(g_err, sizeof(g_err), "%s", msg); }
}  // namespace ppo_detail

namespace {

int launched(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
        return -2;
    }
    return 0;
}

constexpr int kWave = 64;
constexpr float kLog2Pi = 1.8378770664093453f;

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {  // round to nearest even
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7f800000u) == 0x7f800000u) return uint16_t((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
    u += 0x7fffu + ((u >> 16) & 1u);
    return uint16_t(u >> 16);
}

__device__ __forceinline__ float f16_to_f32(uint16_t h) { return float(__builtin_bit_cast(_Float16, h)); }

__device__ __forceinline__ uint16_t f32_to_f16(float f) {  // v_cvt_f16_f32: round to nearest even, inf past 65504
    return __builtin_bit_cast(uint16_t, static_cast<_Float16>(f));
}

// element types of the low-precision buffers: PPO_DT_F32 (0), PPO_DT_BF16 (1), PPO_DT_F16 (2)
template <int T>
__device__ __forceinline__ float lp_to_f32(uint16_t h) { return T == PPO_DT_F16 ? f16_to_f32(h) : bf16_to_f32(h); }
template <int T>
__device__ __forceinline__ uint16_t f32_to_lp(float f) { return T == PPO_DT_F16 ? f32_to_f16(f) : f32_to_bf16(f); }

__device__ __forceinline__ float load_as_f32(const void* p, int64_t i, int dtype) {
    if (dtype == PPO_DT_BF16) return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
    if (dtype == PPO_DT_F16) return f16_to_f32(static_cast<const uint16_t*>(p)[i]);
    return static_cast<const float*>(p)[i];
}

__device__ __forceinline__ void store_from_f32(void* p, int64_t i, int dtype, float x) {
    if (dtype == PPO_DT_BF16)
        static_cast<uint16_t*>(p)[i] = f32_to_bf16(x);
    else if (dtype == PPO_DT_F16)
        static_cast<uint16_t*>(p)[i] = f32_to_f16(x);
    else
        static_cast<float*>(p)[i] = x;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
    return x;
}

// ------------------------------------------------------------------------------ obs normaliser

constexpr int kStatRows = 256;
constexpr int kStatPhases = 4;

__global__ void __launch_bounds__(64 * kStatPhases) k_obs_stats(const float* __restrict__ x,
                                                                const int32_t* __restrict__ mb_idx, int mb_rows,
                                                                int cols, double* __restrict__ partials) {
    __shared__ double red[2][kStatPhases][64];
    const int c = threadIdx.x % 64, ph = threadIdx.x / 64;
    const int64_t base = int64_t(*mb_idx) * mb_rows;
    const int r0 = blockIdx.x * kStatRows;
    const int r1 = min(r0 + kStatRows, mb_rows);
    // four independent chains per thread (rows r, r + 4, r + 8, r + 12 of a 16-row step), so four
    // loads are in flight and the fp64 adds do not serialise on one accumulator; combined in a fixed
    // order (deterministic)
    double sa[4] = {0.0, 0.0, 0.0, 0.0}, qa[4] = {0.0, 0.0, 0.0, 0.0};
    if (c < cols) {
        int r = r0 + ph;
        for (; r + 3 * kStatPhases < r1; r += 4 * kStatPhases) {
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = x[(base + r + u * kStatPhases) * cols + c];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                sa[u] += v[u];
                qa[u] += v[u] * v[u];
            }
        }
        for (; r < r1; r += kStatPhases) {
            const double v = x[(base + r) * cols + c];
            sa[0] += v;
            qa[0] += v * v;
        }
    }
    const double s = (sa[0] + sa[1]) + (sa[2] + sa[3]);
    const double ss = (qa[0] + qa[1]) + (qa[2] + qa[3]);
    red[0][ph][c] = s;
    red[1][ph][c] = ss;
    __syncthreads();
    if (ph < 2) {
        double t = 0.0;
        for (int q = 0; q < kStatPhases; ++q) t += red[ph][q][c];
        partials[(blockIdx.x * 2 + ph) * 64 + c] = t;
    }
}

// 4 waves: wave w sums the partial blocks b = w, w + 4, ... (eight loads in flight per lane), the four
// sums are combined in a fixed order, then wave 0 applies the running-moment update
__global__ void __launch_bounds__(256) k_obs_stats_update(const double* __restrict__ partials, int nblk, int cols,
                                                          int mb_rows, double* __restrict__ mean,
                                                          double* __restrict__ var, double* __restrict__ count) {
    __shared__ double red[2][4][64];
    const int c = threadIdx.x % 64, w = threadIdx.x / 64;
    {
        double s = 0.0, ss = 0.0;
        if (c < cols) {
            int b = w;
            for (; b + 12 < nblk; b += 16) {
                double v[4], q[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    v[u] = partials[((b + 4 * u) * 2 + 0) * 64 + c];
                    q[u] = partials[((b + 4 * u) * 2 + 1) * 64 + c];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    s += v[u];
                    ss += q[u];
                }
            }
            for (; b < nblk; b += 4) {
                s += partials[(b * 2 + 0) * 64 + c];
                ss += partials[(b * 2 + 1) * 64 + c];
            }
        }
        red[0][w][c] = s;
        red[1][w][c] = ss;
    }
    __syncthreads();
    if (w != 0) return;
    const double cnt = *count;  // every lane reads before lane 0 writes (single wave, in-order)
    if (c < cols) {
        const double s = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
        const double ss = (red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c]);
        const double n = double(mb_rows);
        const double bm = s / n;
        const double bv = fmax(ss - n * bm * bm, 0.0) / (n - 1.0);  // torch.var: unbiased
        const double d = bm - mean[c];
        const double tot = cnt + n;
        const double m2 = var[c] * cnt + bv * n + d * d * cnt * n / tot;
        mean[c] = mean[c] + d * n / tot;
        var[c] = m2 / tot;
    }
    __builtin_amdgcn_wave_barrier();
    if (c == 0) *count = cnt + double(mb_rows);
}

// (64 x 4)-thread blocks over 16-row tiles: a thread owns columns c and c + 64 of the tile's rows 4k + ty,
// so the column's mean and 1 / sqrt(var + eps) denominators are read and formed once per thread and
// no element needs a 64-bit index division (the one-thread-per-element form spent most of its time there)
constexpr int kNormCols = 64, kNormRowThreads = 4, kNormTileRows = 16;
__global__ void __launch_bounds__(kNormCols * kNormRowThreads) k_obs_normalize(
    const float* __restrict__ x, const int32_t* __restrict__ mb_idx, int mb_rows, int cols,
    const double* __restrict__ mean, const double* __restrict__ var, float eps, void* __restrict__ out, int out_cols,
    int out_stride, int out_dtype) {
    const int r0 = blockIdx.x * kNormTileRows;
    const int64_t xbase = int64_t(*mb_idx) * mb_rows;
    for (int c = threadIdx.x; c < out_cols; c += kNormCols) {
        const bool in = c < cols;
        // rl_games: (x - mean.float()) / sqrt(var.float() + eps), then clamp
        const float mf = in ? float(mean[c]) : 0.f;
        const float den = in ? sqrtf(float(var[c]) + eps) : 1.f;
#pragma unroll
        for (int k = 0; k < kNormTileRows / kNormRowThreads; ++k) {
            const int r = r0 + kNormRowThreads * k + threadIdx.y;
            if (r >= mb_rows) break;
            float y = 0.f;
            if (in) {
                const float v = x[(xbase + r) * cols + c];
                y = (v - mf) / den;
                y = fminf(fmaxf(y, -5.f), 5.f);
            }
            store_from_f32(out, int64_t(r) * out_stride + c, out_dtype, y);
        }
    }
}

// ------------------------------------------------------------------------------ PPO losses


template <int A>
__global__ void __launch_bounds__(ppo_detail::kLossThreads) k_loss_grad(ppo_detail::LossRowArgs p) {
    __shared__ float s_red[ppo_detail::loss_lds_floats(A)];
    ppo_detail::loss_block<A, ppo_detail::kLossThreads>(p, blockIdx.x, s_red);
}

__global__ void __launch_bounds__(64) k_loss_finalize(const float* __restrict__ partials, int nblk, int A, int mb_rows,
                                                      float entropy_coef, const float* __restrict__ grad_scale,
                                                      float* __restrict__ g_hb,
                                                      float* __restrict__ g_ls, float* __restrict__ stats,
                                                      const int32_t* __restrict__ stat_idx, float* __restrict__ kl_out) {
    const int NV = 2 * A + 1 + PPO_LOSS_NSTAT;
    const int k = blockIdx.x;  // one wave per value, lanes stride over the block partials (fixed order)
    // four independent chains per lane (four loads in flight), combined in a fixed order
    float sa[4] = {0.f, 0.f, 0.f, 0.f};
    int b = threadIdx.x;
    for (; b + 3 * kWave < nblk; b += 4 * kWave) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = partials[int64_t(b + u * kWave) * NV + k];
#pragma unroll
        for (int u = 0; u < 4; ++u) sa[u] += v[u];
    }
    for (; b < nblk; b += kWave) sa[0] += partials[int64_t(b) * NV + k];
    float s = (sa[0] + sa[1]) + (sa[2] + sa[3]);
    s = wave_sum(s);
    if (threadIdx.x != 0) return;
    ppo_detail::loss_finalize_value(k, s, A, mb_rows, entropy_coef, grad_scale, g_hb, g_ls, stats, stat_idx, kl_out);
}

// ------------------------------------------------------------------------------ ELU backward

constexpr int kEluRows = 128;
constexpr int kEluThreads = 1024;

template <int T>
__device__ __forceinline__ void load4(const void* p, int64_t i, float (&x)[4]) {
    if (T) {
        const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p) + i);
        x[0] = lp_to_f32<T>(uint16_t(u.x & 0xffffu));
        x[1] = lp_to_f32<T>(uint16_t(u.x >> 16));
        x[2] = lp_to_f32<T>(uint16_t(u.y & 0xffffu));
        x[3] = lp_to_f32<T>(uint16_t(u.y >> 16));
    } else {
        const float4 u = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
        x[0] = u.x;
        x[1] = u.y;
        x[2] = u.z;
        x[3] = u.w;
    }
}

// four adjacent columns per thread (8-B bf16 / fp16, 16-B fp32 loads), row phases across the block
template <int DH_T, int H_T, int DZ_T>
__global__ void __launch_bounds__(kEluThreads) k_elu_bwd(const void* __restrict__ dh, const void* __restrict__ h,
                                                         void* __restrict__ dz, int rows, int cols,
                                                         float* __restrict__ partials) {
    __shared__ float red[kEluThreads * 4];
    const int quads = cols / 4;
    const int nph = kEluThreads / quads;
    const int cq = threadIdx.x % quads, ph = threadIdx.x / quads;
    const int r0 = blockIdx.x * kEluRows;
    const int r1 = min(r0 + kEluRows, rows);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (ph < nph) {
#pragma unroll 2
        for (int r = r0 + ph; r < r1; r += nph) {
            const int64_t i = int64_t(r) * cols + 4 * cq;
            float g[4], hv[4], z[4];
            load4<DH_T>(dh, i, g);
            load4<H_T>(h, i, hv);
#pragma unroll
            for (int k = 0; k < 4; ++k) z[k] = hv[k] > 0.f ? g[k] : g[k] * (hv[k] + 1.f);
            if (DZ_T) {
                uint16_t b[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    b[k] = f32_to_lp<DZ_T>(z[k]);
                    z[k] = lp_to_f32<DZ_T>(b[k]);  // bias grad from the stored (GEMM-visible) dz
                }
                *reinterpret_cast<uint2*>(static_cast<uint16_t*>(dz) + i) =
                    make_uint2(uint32_t(b[0]) | (uint32_t(b[1]) << 16), uint32_t(b[2]) | (uint32_t(b[3]) << 16));
            } else {
                *reinterpret_cast<float4*>(static_cast<float*>(dz) + i) = make_float4(z[0], z[1], z[2], z[3]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[k] += z[k];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[4 * threadIdx.x + k] = acc[k];
    __syncthreads();
    for (int c = threadIdx.x; c < cols; c += kEluThreads) {
        float t = 0.f;
        for (int q = 0; q < nph; ++q) t += red[4 * (q * quads) + c];
        partials[int64_t(blockIdx.x) * cols + c] = t;
    }
}

// ------------------------------------------------------------------------------ rollout policy head

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

__device__ __forceinline__ float u01(uint32_t u) { return float(u >> 8) * 5.9604644775390625e-8f + 2.98023223876953125e-8f; }

template <int A>
__global__ void __launch_bounds__(256) k_policy_sample(const float* __restrict__ head, const float* __restrict__ logstd,
                                                       int rows, uint64_t seed, const int64_t* __restrict__ step_ctr,
                                                       const double* __restrict__ vm, const double* __restrict__ vv,
                                                       float veps, float* __restrict__ act, float* __restrict__ nlp,
                                                       float* __restrict__ val, float* __restrict__ mus,
                                                       float* __restrict__ sigmas) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const uint64_t sc = uint64_t(*step_ctr);
    const uint2 key = make_uint2(uint32_t(seed), uint32_t(seed >> 32));
    const float* h = head + int64_t(r) * (A + 1);
    float q = 0.f, sum_ls = 0.f;
    float z[(A + 3) / 4 * 4];
#pragma unroll
    for (int c = 0; c < (A + 3) / 4; ++c) {
        const uint4 b = philox4x32_10(make_uint4(uint32_t(r), uint32_t(c), uint32_t(sc), uint32_t(sc >> 32)), key);
        // Box-Muller, two normals per uniform pair
        float s0, c0, s1, c1;
        __sincosf(6.283185307179586f * u01(b.y), &s0, &c0);
        __sincosf(6.283185307179586f * u01(b.w), &s1, &c1);
        const float r0 = sqrtf(-2.f * __logf(u01(b.x))), r1 = sqrtf(-2.f * __logf(u01(b.z)));
        z[4 * c + 0] = r0 * c0;
        z[4 * c + 1] = r0 * s0;
        z[4 * c + 2] = r1 * c1;
        z[4 * c + 3] = r1 * s1;
    }
#pragma unroll
    for (int j = 0; j < A; ++j) {
        const float ls = logstd[j];
        const float sg = expf(ls);
        const float mu = h[j];
        const float a = mu + sg * z[j];
        const float d = (a - mu) / sg;
        q += d * d;
        sum_ls += ls;
        act[int64_t(r) * A + j] = a;
        mus[int64_t(r) * A + j] = mu;
        sigmas[int64_t(r) * A + j] = sg;
    }
    nlp[r] = 0.5f * q + 0.5f * kLog2Pi * float(A) + sum_ls;
    float v = h[A];
    if (vm) v = sqrtf(float(vv[0]) + veps) * fminf(fmaxf(v, -5.f), 5.f) + float(vm[0]);
    val[r] = v;
}

__global__ void k_counter_add(int64_t* ctr, int64_t inc) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *ctr += inc;
}

// ------------------------------------------------------------------------------ rollout bookkeeping

constexpr int kPostThreads = 256;

__global__ void __launch_bounds__(kPostThreads) k_rollout_post(const float* __restrict__ rew,
                                                               const uint8_t* __restrict__ done,
                                                               const uint8_t* __restrict__ tout,
                                                               const float* __restrict__ val, int n, float scale,
                                                               float shift, float gamma, int boot,
                                                               float* __restrict__ shaped_out, float* __restrict__ cr,
                                                               float* __restrict__ cs, float* __restrict__ cl,
                                                               float* __restrict__ partials) {
    __shared__ float red[kPostThreads / kWave][4];
    const int i = blockIdx.x * kPostThreads + threadIdx.x;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (i < n) {
        const float r = rew[i];
        float sh = (r + shift) * scale;  // DefaultRewardsShaper
        if (boot && tout[i]) sh = sh + gamma * val[i] * 1.f;  // value_bootstrap on time-outs
        shaped_out[i] = sh;
        const float r1 = cr[i] + r, s1 = cs[i] + sh, l1 = cl[i] + 1.f;
        const bool d = done[i] != 0;
        if (d) {
            v[0] = r1;
            v[1] = s1;
            v[2] = l1;
            v[3] = 1.f;
        }
        cr[i] = d ? 0.f : r1;  // current_* *= not_dones
        cs[i] = d ? 0.f : s1;
        cl[i] = d ? 0.f : l1;
    }
    const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float t = wave_sum(v[k]);
        if (lane == 0) red[w][k] = t;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        float t = 0.f;
        for (int q = 0; q < kPostThreads / kWave; ++q) t += red[q][threadIdx.x];
        partials[blockIdx.x * 4 + threadIdx.x] = t;
    }
}

__global__ void __launch_bounds__(64) k_meter_update(const float* __restrict__ partials, int nblk, float max_size,
                                                     float* __restrict__ mean3, float* __restrict__ size3) {
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int b = threadIdx.x; b < nblk; b += kWave) {
#pragma unroll
        for (int k = 0; k < 4; ++k) s[k] += partials[b * 4 + k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = wave_sum(s[k]);
    if (threadIdx.x != 0 || s[3] <= 0.f) return;  // no finished episode: meters unchanged
    // torch_ext.AverageMeter.update: size = min(count, max_size), old = min(max_size - size, current)
    const float size = fminf(s[3], max_size);
    for (int k = 0; k < 3; ++k) {
        const float new_mean = s[k] / s[3];
        const float old = fminf(max_size - size, size3[k]);
        const float tot = old + size;
        mean3[k] = (mean3[k] * old + new_mean * size) / tot;
        size3[k] = tot;
    }
}

// ------------------------------------------------------------------------------ partial-row reductions

// ppo_opt_snap_t: Adam's step inputs as this launch found them (ppo_adam_step reads them instead of the
// originals its first block rewrites)
__device__ __forceinline__ void write_snap(ppo_opt_snap_t* snap, const double* lr, const double* step,
                                           const float* scaler) {
    ppo_opt_snap_t s{};
    s.lr = *lr;
    s.step = *step;
    s.scale = scaler ? scaler[0] : 1.f;
    *snap = s;
}

struct JobTable {
    ppo_reduce_job_t j[PPO_MAX_JOBS];
    int32_t count[PPO_MAX_JOBS];          // threads of each job
    int32_t blk_start[PPO_MAX_JOBS + 1];  // first block of each job (blocks never straddle two jobs)
    int vec[PPO_MAX_JOBS];                // columns per thread: 4 (float4 path) or 1
    int n;
    // ppo_reduce_rows_norm: k_sqnorm's partials of the values written (+ one block for the extra arrays)
    float* norm;                          // [nblk sums of (v / scale)^2 | nblk non-finite counts], or NULL
    const float* scaler;
    const float* extra[2];
    int32_t extra_n[2];
    const double* lr;  // the optimizer snapshot (NULL: none), written by the extra block
    const double* step;
    ppo_opt_snap_t* snap;
};

// The splits of one output are summed by kRedT threads -- the block's threads t + kRedOut * i take the
// i-th part of q -- and combined through LDS in part order, a fixed order: more loads in flight per CU than
// one thread per output, which left the chip at ~1.3 waves per SIMD and latency-bound (2 TB/s; two threads
// per output measured 13.8 -> 10.3 us in the trainer).
constexpr int kRedT = 4;                  // threads per output (2 / 8 measured no better in the trainer)
constexpr int kRedOut = 256 / kRedT;      // outputs (or float4 columns) per block

template <int V>
__device__ __forceinline__ void reduce_cols(const ppo_reduce_job_t& jb, int o, bool active, float inv_scale, float& sq,
                                            float& bad) {
    typedef float fv __attribute__((ext_vector_type(V)));
    __shared__ float part_s[kRedT - 1][kRedOut * 4];
    const int part = threadIdx.x / kRedOut, lo = threadIdx.x % kRedOut;
    const int cols = jb.dst_cols / V;
    const int r = o / cols, c = (o - r * cols) * V;
    const float* src = jb.src + int64_t(r) * jb.src_cols + c;
    const int per = (jb.S + kRedT - 1) / kRedT;
    const int q0 = min(jb.S, part * per), q1 = min(jb.S, q0 + per);
    fv s = {};
    if (active) {
        // up to 8 loads in flight per chunk, the chunk predicated, added in q order
        for (int q = q0; q < q1; q += 8) {
            fv v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = q + u < q1 ? *reinterpret_cast<const fv*>(src + int64_t(q + u) * jb.src_n) : fv{};
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (q + u < q1) s += v[u];
        }
    }
    if (part) {
#pragma unroll
        for (int e = 0; e < V; ++e) part_s[part - 1][lo * V + e] = s[e];
    }
    __syncthreads();
    if (part || !active) return;
#pragma unroll
    for (int i = 0; i < kRedT - 1; ++i)
#pragma unroll
        for (int e = 0; e < V; ++e) s[e] += part_s[i][lo * V + e];
    *reinterpret_cast<fv*>(jb.dst + int64_t(r) * jb.dst_stride + c) = s;
#pragma unroll
    for (int e = 0; e < V; ++e) {
        const float x = s[e] * inv_scale;
        sq += x * x;
        bad += __builtin_isfinite(s[e]) ? 0.f : 1.f;
    }
}

// dst[r][c] = sum_q src[q][r][c]; one output element per kRedT threads, or 4 consecutive elements when the
// job's strides and pointers allow 16-B accesses (the same per-element sums).  Each block belongs to one
// job, found by a block-uniform (scalar) search: a per-thread search over the job table was a chain of
// dependent vector loads ahead of every thread's first partial load.  With t.norm the blocks also leave
// k_sqnorm's partials of what they wrote (one gradient pass fewer; a last block covers the extra arrays --
// the gradients other kernels wrote)
__global__ void __launch_bounds__(256) k_reduce_rows(JobTable t) {
    const int b = blockIdx.x;
    const int nb = t.blk_start[t.n];
    const float inv_scale = t.norm && t.scaler ? 1.f / t.scaler[0] : 1.f;
    float sq = 0.f, bad = 0.f;
    if (b < nb) {
        int k = 0;
        while (b >= t.blk_start[k + 1]) ++k;
        const int o = (b - t.blk_start[k]) * kRedOut + threadIdx.x % kRedOut;
        const bool active = o < t.count[k];
        if (t.vec[k] == 4)
            reduce_cols<4>(t.j[k], o, active, inv_scale, sq, bad);
        else
            reduce_cols<1>(t.j[k], o, active, inv_scale, sq, bad);
    } else {
        if (t.snap && threadIdx.x == 0) write_snap(t.snap, t.lr, t.step, t.scaler);
        for (int a = 0; a < 2; ++a)
            for (int i = threadIdx.x; i < t.extra_n[a]; i += 256) {
                const float v = t.extra[a][i];
                const float x = v * inv_scale;
                sq += x * x;
                bad += __builtin_isfinite(v) ? 0.f : 1.f;
            }
    }
    if (!t.norm) return;  // uniform
    __shared__ float red[2][256 / kWave];
    sq = wave_sum(sq);
    bad = wave_sum(bad);
    if (threadIdx.x % kWave == 0) {
        red[0][threadIdx.x / kWave] = sq;
        red[1][threadIdx.x / kWave] = bad;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, c = 0.f;
        for (int w = 0; w < 256 / kWave; ++w) {
            a += red[0][w];
            c += red[1][w];
        }
        t.norm[b] = a;
        t.norm[gridDim.x + b] = c;
    }
}

// ------------------------------------------------------------------------------ clip + Adam

constexpr int kNormBlocks = 256;
constexpr int kAdamThreads = 256;

// block partials of ||g / scale||^2 (partials[b]; NaN / inf propagate as in torch's vector_norm) and
// of the non-finite element count (partials[gridDim.x + b]: GradScaler's found_inf, an OR over
// isfinite(g[i]) -- kept apart from the norm so a finite gradient whose square sum overflows is
// clipped, not skipped).  The scale is a power of two, so g / scale is exact.
__global__ void __launch_bounds__(256) k_sqnorm(const float* __restrict__ g, int64_t n, const float* __restrict__ scaler,
                                                float* __restrict__ partials, const double* lr, const double* step,
                                                ppo_opt_snap_t* snap) {
    __shared__ float red[2][256 / kWave];
    if (snap && blockIdx.x == 0 && threadIdx.x == 0) write_snap(snap, lr, step, scaler);
    const float inv_scale = scaler ? 1.f / scaler[0] : 1.f;
    float s = 0.f, bad = 0.f;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
        const float x = g[i] * inv_scale;
        s += x * x;
        bad += __builtin_isfinite(g[i]) ? 0.f : 1.f;
    }
    s = wave_sum(s);
    bad = wave_sum(bad);
    if (threadIdx.x % kWave == 0) {
        red[0][threadIdx.x / kWave] = s;
        red[1][threadIdx.x / kWave] = bad;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f, b = 0.f;
        for (int w = 0; w < 256 / kWave; ++w) {
            t += red[0][w];
            b += red[1][w];
        }
        partials[blockIdx.x] = t;
        partials[gridDim.x + blockIdx.x] = b;
    }
}

struct SegTable {
    ppo_seg_t s[PPO_MAX_SEG];
    int n;
};

// the end of a minibatch step (ppo_tail): GradScaler.update, the adaptive LR from the KL, Adam's step
// count, the device minibatch / statistics counters -- one thread.  The inputs are read in one go (every
// load issued before the first use: one memory round trip, not one per field)
// ppo_tail's arguments
struct ppo_tail_args_t {
    double* lr;
    const float* kl;
    float kl_threshold;
    double min_lr, max_lr;
    double* step;
    int32_t* mb_idx;
    int32_t n_minibatches;
    int32_t* stat_idx;
    float* scaler;
    int32_t growth_interval;
};

struct TailVals {
    double lr, step;
    float kl, scale, tracker;
    int mb, st;
};

__device__ __forceinline__ TailVals tail_load(const ppo_tail_args_t& t) {
    TailVals v;
    v.lr = *t.lr;
    v.step = *t.step;
    v.kl = t.kl_threshold > 0.f ? *t.kl : 0.f;
    v.scale = t.scaler ? t.scaler[0] : 1.f;
    v.tracker = t.scaler ? t.scaler[1] : 0.f;
    v.mb = *t.mb_idx;
    v.st = *t.stat_idx;
    return v;
}

__device__ void tail_store(const ppo_tail_args_t& t, const TailVals& v, bool skipped) {
    if (t.scaler) {  // GradScaler.update: backoff 0.5 on a skipped step, growth 2 after growth_interval good ones
        if (skipped) {
            t.scaler[0] = v.scale * 0.5f;
            t.scaler[1] = 0.f;
        } else if (v.tracker + 1.f >= float(t.growth_interval)) {
            t.scaler[0] = v.scale * 2.f;
            t.scaler[1] = 0.f;
        } else {
            t.scaler[1] = v.tracker + 1.f;
        }
    }
    if (t.kl_threshold > 0.f) {
        const double k = double(v.kl);
        double nxt = v.lr;
        if (k > 2.0 * double(t.kl_threshold)) nxt = fmax(v.lr / 1.5, t.min_lr);
        if (k < 0.5 * double(t.kl_threshold)) nxt = fmin(v.lr * 1.5, t.max_lr);
        *t.lr = nxt;
    }
    if (!skipped) *t.step = v.step + 1.0;  // a skipped optimizer.step() leaves Adam's step count
    *t.mb_idx = (v.mb + 1) % t.n_minibatches;
    *t.stat_idx = v.st + 1;
}

struct AdamArgs {
    float* p;
    const float* g;
    float* m;
    float* v;
    int64_t n;
    const float* np;  // norm partials [nnp sums | nnp non-finite counts]
    int nnp;
    float max_norm;
    const double* lr_p;  // !TAIL: Adam's lr / step / the scaler read here
    const double* step_p;
    const float* scaler;  // the scaler (NULL: none; with TAIL only tested for NULL, the scale is in snap)
    float b1, b2, eps;
    SegTable segs;
    uint16_t* mirror;
    int mirror_dtype;
    const ppo_opt_snap_t* snap;  // TAIL: lr / step / scale from the norm launch's snapshot
    ppo_tail_args_t tail;        // TAIL: run by block 0 on the originals
};

// clip + Adam (ppo_adam); with TAIL also ppo_tail's work, by block 0 (ppo_adam_step): the other blocks read
// lr / step / scale from the snapshot, never the originals the tail rewrites, so no block waits for another
template <bool TAIL>
__global__ void __launch_bounds__(kAdamThreads) k_adam(AdamArgs a) {
    float* __restrict__ p = a.p;
    const float* __restrict__ g = a.g;
    float* __restrict__ m = a.m;
    float* __restrict__ v = a.v;
    const float* __restrict__ np = a.np;
    const int64_t n = a.n;
    const int nnp = a.nnp;
    const float b1 = a.b1, b2 = a.b2, eps = a.eps;
    __shared__ float red[2][kAdamThreads / kWave];
    __shared__ float coef_s, step_size_s, bc2_sqrt_s, inv_scale_s;
    __shared__ int skip_s;
    // one element per thread (the grid covers n; a grid-stride form with one prologue per resident block
    // measured slower in the trainer, 9.7 -> 12.0 us: fewer waves in flight for the streaming part).  The
    // element's four operands and thread 0's scalars are loaded before the prologue's reductions, so their
    // memory round trip overlaps the norm partials' instead of following it
    const int64_t i = int64_t(blockIdx.x) * kAdamThreads + threadIdx.x;
    float g0 = 0.f, m0 = 0.f, v0 = 0.f, p0 = 0.f;
    if (i < n) {
        g0 = g[i];
        m0 = m[i];
        v0 = v[i];
        p0 = p[i];
    }
    // the norm partials (k_reduce_rows leaves one pair per block, ~1.2 k at the trainer's size) in chunks
    // of 8 loads per thread, all in flight together: the plain loop waited one round trip per iteration
    // (the partials come from other XCDs' writes, so every round trip reaches past L2).  Added in k order,
    // the same sums as the plain loop
    constexpr int kU = 8;
    float s = 0.f, bad = 0.f;
    float ps[kU], pb[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {  // clamped, unpredicated loads (nnp >= 1): no branch to wait inside
        const int k = min(int(threadIdx.x) + u * kAdamThreads, nnp - 1);
        ps[u] = np[k];
        pb[u] = np[nnp + k];
    }
    // thread 0: the bias corrections (fp64 pow / sqrt are long instruction sequences) while those loads
    // are in flight
    float scale0 = 1.f, step_size0 = 0.f, bc2_sqrt0 = 0.f;
    TailVals tv{};
    if (threadIdx.x == 0) {
        double lr, st;
        if constexpr (TAIL) {
            if (blockIdx.x == 0) tv = tail_load(a.tail);  // in flight with the partials
            lr = a.snap->lr;
            st = a.snap->step;
            scale0 = a.snap->scale;
        } else {
            lr = *a.lr_p;
            st = *a.step_p;
            if (a.scaler) scale0 = a.scaler[0];
        }
        const double ts = st + 1.0;
        step_size0 = float(lr / (1.0 - pow(double(b1), ts)));
        bc2_sqrt0 = float(sqrt(1.0 - pow(double(b2), ts)));
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const bool in = int(threadIdx.x) + u * kAdamThreads < nnp;
        s += in ? ps[u] : 0.f;
        bad += in ? pb[u] : 0.f;
    }
    for (int k0 = threadIdx.x + kU * kAdamThreads; k0 < nnp; k0 += kU * kAdamThreads) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int k = min(k0 + u * kAdamThreads, nnp - 1);
            ps[u] = np[k];
            pb[u] = np[nnp + k];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const bool in = k0 + u * kAdamThreads < nnp;
            s += in ? ps[u] : 0.f;
            bad += in ? pb[u] : 0.f;
        }
    }
    s = wave_sum(s);
    bad = wave_sum(bad);
    if (threadIdx.x % kWave == 0) {
        red[0][threadIdx.x / kWave] = s;
        red[1][threadIdx.x / kWave] = bad;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f, b = 0.f;
        for (int w = 0; w < kAdamThreads / kWave; ++w) {
            t += red[0][w];
            b += red[1][w];
        }
        // GradScaler: grads carry the loss scale (a power of two); a non-finite element skips the step
        // (scaler.step's found_inf), otherwise they are unscaled exactly before the clip (unscale_)
        inv_scale_s = 1.f / scale0;
        const bool skip = a.scaler && b > 0.f;
        skip_s = skip;
        // torch.nn.utils.clip_grad_norm_: coef = clamp(max_norm / (total_norm + 1e-6), max=1); the
        // norm is of the unscaled grads (k_sqnorm); a NaN norm makes coef NaN (clamp keeps NaN)
        const float c = a.max_norm / (sqrtf(t) + 1e-6f);
        coef_s = a.max_norm > 0.f ? (c < 1.f || c != c ? c : 1.f) : 1.f;
        step_size_s = step_size0;
        bc2_sqrt_s = bc2_sqrt0;
        if constexpr (TAIL) {
            if (blockIdx.x == 0) tail_store(a.tail, tv, skip);  // the same decision k_tail makes
        }
    }
    __syncthreads();
    const float coef = coef_s;
    const float step_size = step_size_s;
    const float bc2_sqrt = bc2_sqrt_s;
    const float inv_scale = inv_scale_s;
    const bool skip = skip_s;
    if (!skip && i < n) {
        const float gi = (g0 * inv_scale) * coef;
        const float mi = m0 + (1.f - b1) * (gi - m0);  // exp_avg.lerp_(grad, 1 - beta1)
        const float vi = v0 * b2 + (1.f - b2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        const float pi = p0 - step_size * (mi / denom);
        p[i] = pi;
        if (a.mirror) {
            for (int k = 0; k < a.segs.n; ++k) {
                const ppo_seg_t& sg = a.segs.s[k];
                if (i >= sg.off && i < sg.off + sg.len) {
                    // 32-bit division: seg_table holds every segment below 2^31 elements
                    const uint32_t j = uint32_t(i - sg.off), cols = uint32_t(sg.cols);
                    const int64_t r = j / cols, c = j % cols;
                    a.mirror[sg.moff + (sg.trans ? c * sg.mstride + r : r * sg.mstride + c)] =
                        a.mirror_dtype == PPO_DT_F16 ? f32_to_f16(pi) : f32_to_bf16(pi);
                }
            }
        }
    }
}

constexpr int kTailThreads = 256;

__global__ void __launch_bounds__(kTailThreads) k_tail(ppo_tail_args_t t, const float* np, int nnp) {
    // the norm partials' non-finite counts, 8 clamped loads per thread all in flight at once, issued with
    // thread 0's tail_load (one thread walking the partials serially was a chain of dependent global loads,
    // 6 us of every minibatch; one wave with a plain loop still waited one round trip per 64 partials)
    constexpr int kU = 8;
    __shared__ float red[kTailThreads / kWave];
    TailVals v{};
    if (threadIdx.x == 0) v = tail_load(t);
    float b = 0.f;
    if (t.scaler) {  // uniform
        for (int k0 = threadIdx.x; k0 < nnp; k0 += kU * kTailThreads) {
            float x[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) x[u] = np[nnp + min(k0 + u * kTailThreads, nnp - 1)];
#pragma unroll
            for (int u = 0; u < kU; ++u) b += k0 + u * kTailThreads < nnp ? x[u] : 0.f;
        }
        b = wave_sum(b);
        if (threadIdx.x % kWave == 0) red[threadIdx.x / kWave] = b;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 1; w < kTailThreads / kWave; ++w) b += red[w];
    }
    if (threadIdx.x == 0) tail_store(t, v, t.scaler && b > 0.f);
}

inline hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

}  // namespace

extern "C" {

int ppo_abi_version(void) { return PPO_ABI_VERSION; }

#ifndef PPO_BUILD_ID
#define PPO_BUILD_ID "unversioned"
#endif
const char* ppo_build_id(void) { return PPO_BUILD_ID; }
const char* ppo_last_error(void) { return g_err; }

int ppo_obs_stats_blocks(int32_t mb_rows) { return (mb_rows + kStatRows - 1) / kStatRows; }

int ppo_obs_stats(const float* x, const int32_t* mb_idx, int32_t mb_rows, int32_t cols, double* partials,
                  void* stream) {
    if (cols <= 0 || cols > 64 || mb_rows < 2) return fail(-1, "ppo_obs_stats: need 1 <= cols <= 64, mb_rows >= 2");
    hipLaunchKernelGGL(k_obs_stats, dim3(ppo_obs_stats_blocks(mb_rows)), dim3(64 * kStatPhases), 0, S(stream), x,
                       mb_idx, mb_rows,
                       cols, partials);
    return launched("k_obs_stats");
}

int ppo_obs_stats_update(const double* partials, int32_t nblk, int32_t cols, int32_t mb_rows, double* running_mean,
                         double* running_var, double* count, void* stream) {
    if (cols <= 0 || cols > 64) return fail(-1, "ppo_obs_stats_update: cols must be in [1, 64]");
    hipLaunchKernelGGL(k_obs_stats_update, dim3(1), dim3(256), 0, S(stream), partials, nblk, cols, mb_rows, running_mean,
                       running_var, count);
    return launched("k_obs_stats_update");
}

int ppo_obs_normalize(const float* x, const int32_t* mb_idx, int32_t mb_rows, int32_t cols, const double* running_mean,
                      const double* running_var, float eps, void* out, int32_t out_cols, int32_t out_stride,
                      int32_t out_dtype, void* stream) {
    if (out_cols < cols || out_stride < out_cols) return fail(-1, "ppo_obs_normalize: need cols <= out_cols <= out_stride");
    if (out_dtype < PPO_DT_F32 || out_dtype > PPO_DT_F16) return fail(-1, "ppo_obs_normalize: bad out_dtype");
    hipLaunchKernelGGL(k_obs_normalize, dim3(unsigned((mb_rows + kNormTileRows - 1) / kNormTileRows)),
                       dim3(kNormCols, kNormRowThreads), 0, S(stream), x, mb_idx, mb_rows,
                       cols, running_mean, running_var, eps, out, out_cols, out_stride, out_dtype);
    return launched("k_obs_normalize");
}

int ppo_loss_blocks(int32_t mb_rows) { return (mb_rows + ppo_detail::kLossRows - 1) / ppo_detail::kLossRows; }

static int launch_loss(const float* head, const float* logstd, int32_t A, int32_t mb_rows, const int32_t* mb_idx,
                       const float* actions, float* ds_mu, float* ds_sigma, const float* old_neglogp,
                       const float* advantages, const float* old_values, const float* returns, ppo_loss_cfg_t cfg,
                       const float* grad_scale, float* dhead, float* partials, uint16_t* dhead_lp, int32_t lp_dtype,
                       void* stream) {
    if (dhead_lp && lp_dtype != PPO_DT_BF16 && lp_dtype != PPO_DT_F16)
        return fail(-1, "ppo_loss_grad: dhead_lp needs lp_dtype PPO_DT_BF16 or PPO_DT_F16");
    const dim3 grid(ppo_loss_blocks(mb_rows)), block(ppo_detail::kLossThreads);
    ppo_detail::LossRowArgs p{};
    p.head = head;
    p.head_stride = A + 1;
    p.head_block_rows = true;
    p.logstd = logstd;
    p.mb_rows = mb_rows;
    p.mb_idx = mb_idx;
    p.actions = actions;
    p.ds_mu = ds_mu;
    p.ds_sigma = ds_sigma;
    p.old_nlp = old_neglogp;
    p.adv = advantages;
    p.old_v = old_values;
    p.ret = returns;
    p.cfg = cfg;
    p.grad_scale = grad_scale;
    p.dhead = dhead;
    p.dhead_lp = dhead_lp;
    p.lp_dtype = lp_dtype;
    p.partials = partials;
#define PPO_LOSS_CASE(AA)                                                                          \
    case AA:                                                                                       \
        hipLaunchKernelGGL(k_loss_grad<AA>, grid, block, 0, S(stream), p);                         \
        break;
    switch (A) {
        PPO_LOSS_CASE(2)
        PPO_LOSS_CASE(12)
        PPO_LOSS_CASE(21)
        default:
            return fail(-1, "ppo_loss_grad: action dims 2, 12 and 21 are instantiated");
    }
#undef PPO_LOSS_CASE
    return launched("k_loss_grad");
}

int ppo_loss_grad(const float* head, const float* logstd, int32_t A, int32_t mb_rows, const int32_t* mb_idx,
                  const float* actions, float* ds_mu, float* ds_sigma, const float* old_neglogp,
                  const float* advantages, const float* old_values, const float* returns, ppo_loss_cfg_t cfg,
                  const float* grad_scale, float* dhead, float* partials, uint16_t* dhead_lp, int32_t lp_dtype,
                  void* stream) {
    return launch_loss(head, logstd, A, mb_rows, mb_idx, actions, ds_mu, ds_sigma, old_neglogp, advantages, old_values,
                       returns, cfg, grad_scale, dhead, partials, dhead_lp, lp_dtype, stream);
}


int ppo_loss_finalize(const float* partials, int32_t nblk, int32_t A, int32_t mb_rows, float entropy_coef,
                      const float* grad_scale, float* grad_head_bias, float* grad_logstd, float* stats,
                      const int32_t* stat_idx, float* kl_out, void* stream) {
    if (A <= 0 || A > PPO_MAX_ACT) return fail(-1, "ppo_loss_finalize: bad action dim");
    hipLaunchKernelGGL(k_loss_finalize, dim3(2 * A + 1 + PPO_LOSS_NSTAT), dim3(kWave), 0, S(stream), partials, nblk, A,
                       mb_rows, entropy_coef, grad_scale, grad_head_bias, grad_logstd, stats, stat_idx, kl_out);
    return launched("k_loss_finalize");
}

int ppo_elu_bwd_blocks(int32_t rows) { return (rows + kEluRows - 1) / kEluRows; }

int ppo_elu_bwd(const void* dh, int32_t dh_dtype, const void* h, int32_t h_dtype, void* dz, int32_t dz_dtype,
                int32_t rows, int32_t cols, float* partials, void* stream) {
    if (cols % 64 || cols > 4 * kEluThreads) return fail(-1, "ppo_elu_bwd: cols must be a multiple of 64, <= 4096");
    const dim3 grid(ppo_elu_bwd_blocks(rows)), block(kEluThreads);
    const int code = dh_dtype * 9 + h_dtype * 3 + dz_dtype;
#define PPO_ELU_CASE(A, B, C)                                                                                          \
    case A * 9 + B * 3 + C:                                                                                            \
        hipLaunchKernelGGL((k_elu_bwd<A, B, C>), grid, block, 0, S(stream), dh, h, dz, rows, cols, partials);         \
        break;
    switch (code) {
        PPO_ELU_CASE(0, 0, 0)
        PPO_ELU_CASE(0, 0, 1)
        PPO_ELU_CASE(0, 1, 1)
        PPO_ELU_CASE(1, 1, 1)
        PPO_ELU_CASE(0, 0, 2)
        PPO_ELU_CASE(0, 2, 2)
        PPO_ELU_CASE(2, 2, 2)
        default:
            return fail(-1, "ppo_elu_bwd: dtype combination (dh, h, dz) must be (f32,f32,f32), (f32,f32,lp), "
                            "(f32,lp,lp) or (lp,lp,lp) with lp bf16 or fp16");
    }
#undef PPO_ELU_CASE
    return launched("k_elu_bwd");
}

static int reduce_table(const ppo_reduce_job_t* jobs_host, int32_t njobs, JobTable& t) {
    if (njobs <= 0 || njobs > PPO_MAX_JOBS) return fail(-1, "ppo_reduce_rows: 1..16 jobs");
    t = JobTable{};
    t.n = njobs;
    t.blk_start[0] = 0;
    for (int k = 0; k < njobs; ++k) {
        const ppo_reduce_job_t& j = jobs_host[k];
        if (j.S <= 0 || j.dst_cols <= 0 || j.src_cols < j.dst_cols || j.dst_stride < j.dst_cols || !j.src || !j.dst)
            return fail(-1, "ppo_reduce_rows: bad job");
        t.j[k] = j;
        const bool v4 = j.dst_cols % 4 == 0 && j.src_cols % 4 == 0 && j.dst_stride % 4 == 0 && j.src_n % 4 == 0 &&
                        (reinterpret_cast<uintptr_t>(j.src) | reinterpret_cast<uintptr_t>(j.dst)) % 16 == 0;
        t.vec[k] = v4 ? 4 : 1;
        const int64_t cnt = int64_t(j.out_rows) * j.dst_cols / t.vec[k];
        if (cnt > (int64_t(1) << 30)) return fail(-1, "ppo_reduce_rows: job too large");
        t.count[k] = int32_t(cnt);
        t.blk_start[k + 1] = t.blk_start[k] + int32_t((cnt + kRedOut - 1) / kRedOut);
    }
    for (int k = njobs; k < PPO_MAX_JOBS; ++k) t.blk_start[k + 1] = t.blk_start[njobs];
    return 0;
}

int ppo_reduce_rows(const ppo_reduce_job_t* jobs_host, int32_t njobs, void* stream) {
    JobTable t;
    if (const int rc = reduce_table(jobs_host, njobs, t)) return rc;
    hipLaunchKernelGGL(k_reduce_rows, dim3(unsigned(t.blk_start[njobs])), dim3(256), 0, S(stream), t);
    return launched("k_reduce_rows");
}

int ppo_reduce_rows_norm(const ppo_reduce_job_t* jobs_host, int32_t njobs, const float* scaler, const float* extra0,
                         int32_t extra0_n, const float* extra1, int32_t extra1_n, float* norm_partials,
                         int32_t max_blocks, int32_t* nblk_out, const double* lr, const double* step,
                         ppo_opt_snap_t* snap, void* stream) {
    JobTable t;
    if (const int rc = reduce_table(jobs_host, njobs, t)) return rc;
    const int nblk = t.blk_start[njobs] + 1;
    if (!norm_partials || !nblk_out || nblk > max_blocks || extra0_n < 0 || extra1_n < 0 ||
        (extra0_n && !extra0) || (extra1_n && !extra1))
        return fail(-1, "ppo_reduce_rows_norm: bad norm arguments");
    if (snap && (!lr || !step)) return fail(-1, "ppo_reduce_rows_norm: the snapshot needs lr and step");
    t.lr = lr;
    t.step = step;
    t.snap = snap;
    t.norm = norm_partials;
    t.scaler = scaler;
    t.extra[0] = extra0;
    t.extra[1] = extra1;
    t.extra_n[0] = extra0_n;
    t.extra_n[1] = extra1_n;
    *nblk_out = nblk;
    hipLaunchKernelGGL(k_reduce_rows, dim3(unsigned(nblk)), dim3(256), 0, S(stream), t);
    return launched("k_reduce_rows");
}

int ppo_policy_sample(const float* head, const float* logstd, int32_t A, int32_t rows, uint64_t seed,
                      const int64_t* step_ctr, const double* vms_mean, const double* vms_var, float vms_eps,
                      float* actions, float* neglogp, float* values, float* mus, float* sigmas, void* stream) {
    const dim3 grid((rows + 255) / 256), block(256);
#define PPO_SAMPLE_CASE(AA)                                                                                          \
    case AA:                                                                                                         \
        hipLaunchKernelGGL(k_policy_sample<AA>, grid, block, 0, S(stream), head, logstd, rows, seed, step_ctr,     \
                           vms_mean, vms_var, vms_eps, actions, neglogp, values, mus, sigmas);                      \
        break;
    switch (A) {
        PPO_SAMPLE_CASE(2)
        PPO_SAMPLE_CASE(12)
        PPO_SAMPLE_CASE(21)
        default:
            return fail(-1, "ppo_policy_sample: action dims 2, 12 and 21 are instantiated");
    }
#undef PPO_SAMPLE_CASE
    return launched("k_policy_sample");
}

int ppo_counter_add(int64_t* ctr, int64_t inc, void* stream) {
    hipLaunchKernelGGL(k_counter_add, dim3(1), dim3(64), 0, S(stream), ctr, inc);
    return launched("k_counter_add");
}

int ppo_rollout_post_blocks(int32_t n) { return (n + kPostThreads - 1) / kPostThreads; }

int ppo_rollout_post(const float* reward, const uint8_t* done, const uint8_t* time_out, const float* value,
                     int32_t n, float scale, float shift, float gamma, int32_t bootstrap, float* shaped_out,
                     float* cur_r, float* cur_s, float* cur_l, float* partials, void* stream) {
    if (n <= 0 || (bootstrap && (!time_out || !value))) return fail(-1, "ppo_rollout_post: bad arguments");
    hipLaunchKernelGGL(k_rollout_post, dim3(ppo_rollout_post_blocks(n)), dim3(kPostThreads), 0, S(stream), reward,
                       done, time_out, value, n, scale, shift, gamma, bootstrap, shaped_out, cur_r, cur_s, cur_l,
                       partials);
    return launched("k_rollout_post");
}

int ppo_meter_update(const float* partials, int32_t nblk, float max_size, float* mean3, float* size3, void* stream) {
    hipLaunchKernelGGL(k_meter_update, dim3(1), dim3(kWave), 0, S(stream), partials, nblk, max_size, mean3, size3);
    return launched("k_meter_update");
}

int ppo_sqnorm_blocks(void) { return kNormBlocks; }

int ppo_sqnorm(const float* g, int64_t n, const float* scaler, float* partials, const double* lr, const double* step,
               ppo_opt_snap_t* snap, void* stream) {
    if (snap && (!lr || !step)) return fail(-1, "ppo_sqnorm: the snapshot needs lr and step");
    hipLaunchKernelGGL(k_sqnorm, dim3(kNormBlocks), dim3(256), 0, S(stream), g, n, scaler, partials, lr, step, snap);
    return launched("k_sqnorm");
}

static int seg_table(const ppo_seg_t* segs_host, int32_t nseg, void* mirror, int32_t mirror_dtype, SegTable& t) {
    if (nseg < 0 || nseg > PPO_MAX_SEG) return fail(-1, "ppo_adam: too many mirror segments");
    if (mirror && mirror_dtype != PPO_DT_BF16 && mirror_dtype != PPO_DT_F16)
        return fail(-1, "ppo_adam: mirror_dtype must be bf16 or fp16");
    t = SegTable{};
    t.n = mirror ? nseg : 0;
    for (int k = 0; k < t.n; ++k) {
        t.s[k] = segs_host[k];
        const int64_t rows = t.s[k].cols > 0 ? t.s[k].len / t.s[k].cols : 0;
        if (t.s[k].cols <= 0 || t.s[k].len < 0 || t.s[k].len > INT32_MAX ||
            t.s[k].mstride < (t.s[k].trans ? rows : t.s[k].cols))
            return fail(-1, "ppo_adam: bad segment");
    }
    return 0;
}

int ppo_adam(float* p, const float* g, float* m, float* v, int64_t n, const float* sqnorm_partials, int32_t nblk_norm,
             float max_norm, const double* lr, double* step, float beta1, float beta2, float eps,
             const ppo_seg_t* segs_host, int32_t nseg, void* mirror, int32_t mirror_dtype, const float* scaler,
             void* stream) {
    AdamArgs a{};
    if (const int rc = seg_table(segs_host, nseg, mirror, mirror_dtype, a.segs)) return rc;
    if (nblk_norm < 1) return fail(-1, "ppo_adam: need nblk_norm >= 1");
    if (n < 0 || !lr || !step) return fail(-1, "ppo_adam: bad arguments");
    a.p = p;
    a.g = g;
    a.m = m;
    a.v = v;
    a.n = n;
    a.np = sqnorm_partials;
    a.nnp = nblk_norm;
    a.max_norm = max_norm;
    a.lr_p = lr;
    a.step_p = step;
    a.scaler = scaler;
    a.b1 = beta1;
    a.b2 = beta2;
    a.eps = eps;
    a.mirror = static_cast<uint16_t*>(mirror);
    a.mirror_dtype = mirror_dtype;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_adam<false>, dim3(unsigned((n + kAdamThreads - 1) / kAdamThreads)), dim3(kAdamThreads), 0,
                       S(stream), a);
    return launched("k_adam");
}

static int check_tail(const ppo_tail_args_t& t, const float* sqnorm_partials, int32_t nblk_norm) {
    if (!t.lr || !t.step || !t.mb_idx || !t.stat_idx || (t.kl_threshold > 0.f && !t.kl))
        return fail(-1, "ppo_tail: null pointer");
    if (t.n_minibatches <= 0) return fail(-1, "ppo_tail: n_minibatches must be positive");
    if (t.scaler && (!sqnorm_partials || nblk_norm < 1 || t.growth_interval <= 0)) return fail(-1, "ppo_tail: the scaler needs the norm partials");
    return 0;
}

int ppo_tail(double* lr, const float* kl, float kl_threshold, double min_lr, double max_lr, double* step,
             int32_t* mb_idx, int32_t n_minibatches, int32_t* stat_idx, float* scaler, const float* sqnorm_partials,
             int32_t nblk_norm, int32_t growth_interval, void* stream) {
    const ppo_tail_args_t t{lr, kl, kl_threshold, min_lr, max_lr, step, mb_idx, n_minibatches, stat_idx, scaler,
                            growth_interval};
    if (const int rc = check_tail(t, sqnorm_partials, nblk_norm)) return rc;
    hipLaunchKernelGGL(k_tail, dim3(1), dim3(kTailThreads), 0, S(stream), t, sqnorm_partials, nblk_norm);
    return launched("k_tail");
}

int ppo_adam_step(const ppo_adam_step_t* s, void* stream) {
    if (!s) return fail(-1, "ppo_adam_step: null arguments");
    AdamArgs a{};
    if (const int rc = seg_table(s->segs_host, s->nseg, s->mirror, s->mirror_dtype, a.segs)) return rc;
    if (s->nblk_norm < 1 || !s->norm_partials) return fail(-1, "ppo_adam_step: need the norm partials (nblk_norm >= 1)");
    if (s->n <= 0 || !s->snap) return fail(-1, "ppo_adam_step: need n > 0 and the snapshot");
    a.tail = ppo_tail_args_t{s->lr, s->kl, s->kl_threshold, s->min_lr, s->max_lr, s->step, s->mb_idx,
                             s->n_minibatches, s->stat_idx, s->scaler, s->growth_interval};
    if (const int rc = check_tail(a.tail, s->norm_partials, s->nblk_norm)) return rc;
    a.p = s->p;
    a.g = s->g;
    a.m = s->m;
    a.v = s->v;
    a.n = s->n;
    a.np = s->norm_partials;
    a.nnp = s->nblk_norm;
    a.max_norm = s->max_norm;
    a.scaler = s->scaler;
    a.b1 = s->beta1;
    a.b2 = s->beta2;
    a.eps = s->eps;
    a.mirror = static_cast<uint16_t*>(s->mirror);
    a.mirror_dtype = s->mirror_dtype;
    a.snap = s->snap;
    hipLaunchKernelGGL(k_adam<true>, dim3(unsigned((s->n + kAdamThreads - 1) / kAdamThreads)), dim3(kAdamThreads), 0,
                       S(stream), a);
    return launched("k_adam_step");
}

}  // extern "C"

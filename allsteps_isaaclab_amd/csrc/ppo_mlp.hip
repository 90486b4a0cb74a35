// ppo_mlp.hip -- fused MFMA forward of the Allsteps actor-critic trunk (include/ppo.h ppo_mlp_forward).
//
// rl_games' ModelA2CContinuousLogStd runs the trunk as 5 x (Linear -> ELU) plus two heads, i.e. 12
// library launches with every activation round-tripping HBM twice (GEMM out, ELU in/out).  Here one
// wave owns 32 batch rows end to end: with Y = W X (X = activations, features x batch), the
// 32x32x16 bf16 / fp16 MFMA accumulator of one layer has the batch on the lane and the features in its
// 16 registers, which is exactly the B-operand layout of the next layer's MFMA (k order permuted:
// element e of k-step s in lane half h is feature 16s + 8(e>>2) + 4h + (e&3) of the tile), so the
// activations never leave registers; the A operand (weights) is read from LDS in the same permuted
// order.  Bias + ELU are applied on the fp32 accumulators, then rounded to the trunk's element type
// once (bf16, or fp16 -- rl_games' mixed_precision autocast type -- on v_mfma_f32_32x32x16_f16 at the
// same rate).  The heads (mu | value) run as exact-f32 32x32x2 MFMAs on the fp32 layer-5 activations.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "ppo.h"

namespace ppo_detail {
void set_error(const char* msg);
}

#ifndef PPO_MLP_DBG
#define PPO_MLP_DBG 0
#endif

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// the trunk's 16-bit element type: PPO_DT_BF16 or PPO_DT_F16 (same fragment layout, same MFMA shape)
template <int DT>
struct Lp;
template <>
struct Lp<PPO_DT_BF16> {
    typedef __bf16 e;
    typedef __bf16 v8 __attribute__((ext_vector_type(8)));
    static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};
template <>
struct Lp<PPO_DT_F16> {
    typedef _Float16 e;
    typedef _Float16 v8 __attribute__((ext_vector_type(8)));
    static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};

constexpr int kHid = 256;
constexpr int kK0 = 64;
constexpr int kTiles = kHid / 32;    // output / input tiles of 32 features
constexpr int kWaves = 4;
constexpr int kRowsPerBlock = 32 * kWaves;
constexpr int kPad = 8;              // bf16 elements of padding per LDS row (16 B)
constexpr int kWBytes = kHid * (kHid + kPad) * 2;  // 135168 B: one 256 x 256 layer
constexpr int kLdsBytes = kWBytes + 5 * kHid * 4;   // + the five bias vectors (fp32)

char g_err[256];  // formatted here, published through ppo_last_error() (ppo_kernels.hip)

template <int DT>
union Frag {
    typename Lp<DT>::v8 v;
    uint2 q[2];
    uint16_t s[8];
};

// LDS image of a layer's weights: row o = output feature, row stride K + kPad; inside every 16-element
// block of a row the four 4-element quads are stored in the order [0-3, 8-11, 4-7, 12-15], so the A
// fragment of either lane half (quads {0, 2} for h = 0, {1, 3} for h = 1 of the k-step's block, the
// permuted k order above) is ONE 16-B read: ds_read_b128, conflict-free (row stride 132 dwords puts
// the 16 rows of a lane group on distinct 4-bank slots).
template <int DT>
__device__ __forceinline__ typename Lp<DT>::v8 load_a(const uint16_t* lds, int stride, int row, int kt, int s, int h) {
    return *reinterpret_cast<const typename Lp<DT>::v8*>(lds + row * stride + kt * 32 + 16 * s + 8 * h);
}

// stage a 256 x K 16-bit matrix (row stride K) into the LDS image above.  A thread copies whole 16-element
// blocks (two 16-B loads, quads re-paired in registers, two 16-B stores); addresses are one per-thread
// base plus compile-time offsets, so the PPO_STAGE_DEPTH blocks of a round are all in flight at once.
#ifndef PPO_STAGE_DEPTH
#define PPO_STAGE_DEPTH 4
#endif
template <int K>
__device__ __forceinline__ void stage_w(uint16_t* lds, const uint16_t* __restrict__ w) {
    constexpr int kBlk = K / 16;                           // blocks per row
    constexpr int kRowsPerU = 64 * kWaves / kBlk;          // rows advanced per block of a thread
    constexpr int per = kHid / kRowsPerU;                  // blocks per thread
    constexpr int D = per < PPO_STAGE_DEPTH ? per : PPO_STAGE_DEPTH;
    static_assert(64 * kWaves % kBlk == 0 && per % D == 0, "staging split");
    const int t = threadIdx.x;
    const uint16_t* __restrict__ src = w + (t / kBlk) * K + (t % kBlk) * 16;
    uint16_t* dst = lds + (t / kBlk) * (K + kPad) + (t % kBlk) * 16;
#pragma unroll
    for (int u0 = 0; u0 < per; u0 += D) {
        uint4 lo[D], hi[D];
#pragma unroll
        for (int u = 0; u < D; ++u) {
            lo[u] = *reinterpret_cast<const uint4*>(src + (u0 + u) * kRowsPerU * K);
            hi[u] = *reinterpret_cast<const uint4*>(src + (u0 + u) * kRowsPerU * K + 8);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the round's loads together (the scheduler sinks them)
#pragma unroll
        for (int u = 0; u < D; ++u) {
            uint16_t* d = dst + (u0 + u) * kRowsPerU * (K + kPad);
            *reinterpret_cast<uint4*>(d) = make_uint4(lo[u].x, lo[u].y, hi[u].x, hi[u].y);      // e0-3, e8-11
            *reinterpret_cast<uint4*>(d + 8) = make_uint4(lo[u].z, lo[u].w, hi[u].z, hi[u].w);  // e4-7, e12-15
        }
    }
}

// acc[ot] = W (256 x K, in LDS) . X (K x 32); xb[kt][s] are the B fragments of X.  k-steps outer,
// output tiles inner: eight independent accumulator chains; the A fragments of k-step n + 1 are read
// while the MFMAs of k-step n run (two fragment sets).
template <int K, int DT>
__device__ __forceinline__ void layer_mma(const uint16_t* lds, const typename Lp<DT>::v8 (&xb)[kTiles][2],
                                          f32x16 (&acc)[kTiles], int lane) {
    constexpr int NS = K / 16;
    const int i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int ot = 0; ot < kTiles; ++ot) acc[ot] = f32x16{};
    typename Lp<DT>::v8 af[2][kTiles];
#pragma unroll
    for (int ot = 0; ot < kTiles; ++ot) af[0][ot] = load_a<DT>(lds, K + kPad, ot * 32 + i, 0, 0, h);
#pragma unroll
    for (int n = 0; n < NS; ++n) {
        if (n + 1 < NS) {
#pragma unroll
            for (int ot = 0; ot < kTiles; ++ot)
                af[(n + 1) & 1][ot] = load_a<DT>(lds, K + kPad, ot * 32 + i, (n + 1) >> 1, (n + 1) & 1, h);
        }
        __builtin_amdgcn_sched_barrier(0);  // next k-step's reads stay ahead of this k-step's MFMAs
#pragma unroll
        for (int ot = 0; ot < kTiles; ++ot)
            acc[ot] = Lp<DT>::mma(af[n & 1][ot], xb[n >> 1][n & 1], acc[ot]);
    }
}

// Row stores of a tile's 16-bit chunks.  Lane (j, h) holds chunk g = features 8g + 4h + 0..3 of row j;
// one v_permlane32_swap per dword gives the lower lanes features 8g + 0..7 and the upper lanes
// 8(g + 1) + 0..7, so a lane writes 16 contiguous bytes at feature 8(g + h) (32-B runs per row per
// store instead of 16-B ones).  Every lane must execute it (cross-lane), live or not.
__device__ __forceinline__ uint4 pair_chunks(uint2 ga, uint2 gb) {
    const auto x = __builtin_amdgcn_permlane32_swap(ga.x, gb.x, false, false);
    const auto y = __builtin_amdgcn_permlane32_swap(ga.y, gb.y, false, false);
    return make_uint4(x[0], y[0], x[1], y[1]);
}

// feature of register r of a tile for lane half h
__device__ __forceinline__ int feat(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <int DT>
__global__ void __launch_bounds__(64 * kWaves, 1) k_mlp_fwd(ppo_mlp_fwd_t a) {
    typedef typename Lp<DT>::e E;
    typedef typename Lp<DT>::v8 V8;
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int j = lane & 31, h = lane >> 5;
    const int row = blockIdx.x * kRowsPerBlock + wave * 32 + j;  // this lane's batch row
    const bool live = row < a.rows;
    float* lbias = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + kWBytes);
    {  // the five bias vectors: one independent load per layer per thread (blockDim == kHid)
        float bl[5];
#pragma unroll
        for (int l = 0; l < 5; ++l) bl[l] = a.b[l][threadIdx.x];
#pragma unroll
        for (int l = 0; l < 5; ++l) lbias[l * kHid + threadIdx.x] = bl[l];
    }

    // layer-0 input fragments (k order permuted as for a chained accumulator)
    V8 xb[kTiles][2];
#pragma unroll
    for (int kt = 0; kt < kTiles; ++kt) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            Frag<DT> f;
            f.q[0] = make_uint2(0, 0);
            f.q[1] = make_uint2(0, 0);
            if (kt < kK0 / 32 && live) {
                const uint16_t* p = a.x + int64_t(row) * a.x_stride + kt * 32 + 16 * s + 4 * h;
                f.q[0] = *reinterpret_cast<const uint2*>(p);
                f.q[1] = *reinterpret_cast<const uint2*>(p + 8);
            }
            xb[kt][s] = f.v;
        }
    }
    f32x16 acc[kTiles];
    for (int l = 0; l < 5; ++l) {
        __syncthreads();  // previous layer's LDS reads are done
        if (!(PPO_MLP_DBG & 1)) {
            if (l == 0)
                stage_w<kK0>(lds, a.w[0]);
            else
                stage_w<kHid>(lds, a.w[l]);
        }
        __syncthreads();
        if (!(PPO_MLP_DBG & 2)) {
            if (l == 0)
                layer_mma<kK0, DT>(lds, xb, acc, lane);
            else
                layer_mma<kHid, DT>(lds, xb, acc, lane);
        }
        // epilogue: bias + ELU in fp32, store, and the next layer's B fragments
        const float* bias = lbias + l * kHid;
        // per-lane row bases: every store below is base + a compile-time offset (no per-store address)
        uint16_t* __restrict__ hrow = l < 4 && a.h[l] ? a.h[l] + int64_t(row) * a.h_stride + 8 * h : nullptr;
        float* __restrict__ h5row = l == 4 && a.h5 ? a.h5 + int64_t(row) * kHid + 4 * h : nullptr;
#pragma unroll
        for (int ot = 0; ot < kTiles; ++ot) {
            Frag<DT> f[2];
            float bv[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {  // features ot*32 + 8g + 4h + 0..3 of registers 4g..4g+3
                const float4 q = *reinterpret_cast<const float4*>(bias + ot * 32 + 8 * g + 4 * h);
                bv[4 * g] = q.x;
                bv[4 * g + 1] = q.y;
                bv[4 * g + 2] = q.z;
                bv[4 * g + 3] = q.w;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float z = acc[ot][r] + bv[r];
                // ELU (alpha 1): exp(z) - 1 on the hardware exp; |error| ~1e-7, far below the bf16 step
                const float y = (PPO_MLP_DBG & 4) ? z : (z > 0.f ? z : __expf(z) - 1.f);
                acc[ot][r] = y;
                f[r >> 3].v[r & 7] = (E)y;  // v_cvt_pk_bf16_f32 / v_cvt_f16_f32 (round to nearest even)
            }
            xb[ot][0] = f[0].v;
            xb[ot][1] = f[1].v;
            if (hrow) {
                const uint4 c01 = pair_chunks(f[0].q[0], f[0].q[1]), c23 = pair_chunks(f[1].q[0], f[1].q[1]);
                if (live) {
                    *reinterpret_cast<uint4*>(hrow + ot * 32) = c01;
                    *reinterpret_cast<uint4*>(hrow + ot * 32 + 16) = c23;
                }
            }
            if (live) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (h5row)
                        *reinterpret_cast<float4*>(h5row + ot * 32 + 8 * g) =
                            make_float4(acc[ot][4 * g], acc[ot][4 * g + 1], acc[ot][4 * g + 2], acc[ot][4 * g + 3]);
                }
            }
        }
    }
    // heads in exact f32: head[row][o] = sum_f wh[o][f] h5[f] + bh[o]
    if (PPO_MLP_DBG & 8) return;
    __syncthreads();
    float* wl = reinterpret_cast<float*>(lds);
    constexpr int kHs = kHid + 4;
    {  // 32 x 256 fp32 head weights (rows >= nh zero): 8 independent 16-B loads per thread
        constexpr int per = 32 * kHid / 4 / (64 * kWaves);
        float4 v[per];
#pragma unroll
        for (int u = 0; u < per; ++u) {
            const int c = u * (64 * kWaves) + threadIdx.x;
            const int o = c / (kHid / 4), col = (c % (kHid / 4)) * 4;
            v[u] = o < a.nh ? *reinterpret_cast<const float4*>(a.wh + o * kHid + col) : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < per; ++u) {
            const int c = u * (64 * kWaves) + threadIdx.x;
            *reinterpret_cast<float4*>(wl + (c / (kHid / 4)) * kHs + (c % (kHid / 4)) * 4) = v[u];
        }
    }
    __syncthreads();
    f32x16 hq[4] = {};  // four independent chains (the f32 MFMA result latency is not exposed)
#pragma unroll
    for (int ot = 0; ot < kTiles; ++ot) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float wv = wl[j * kHs + ot * 32 + feat(r, h)];
            hq[r & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv, acc[ot][r], hq[r & 3], 0, 0, 0);
        }
    }
    const f32x16 hacc = (hq[0] + hq[1]) + (hq[2] + hq[3]);
    if (live && a.head) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = feat(r, h);
            if (o < a.nh) a.head[int64_t(row) * a.nh + o] = hacc[r] + a.bh[o];
        }
    }
}

// ------------------------------------------------------------------------------ backward chain

template <int DT>
__global__ void __launch_bounds__(64 * kWaves, 1) k_mlp_bwd(ppo_mlp_bwd_t a) {
    typedef typename Lp<DT>::e E;
    typedef typename Lp<DT>::v8 V8;
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int j = lane & 31, h = lane >> 5, i = lane & 31;
    const int row = blockIdx.x * kRowsPerBlock + wave * 32 + j;
    const bool live = row < a.rows;
    constexpr int kHs = kHid + 4;
    // dh5 = Wh^T dhead: A[feature i][k] = wh[k][feature], B[k][batch j] = dhead[j][k]; k = 2t + h
    float* wl = reinterpret_cast<float*>(lds);
    {
        constexpr int per = 32 * kHid / 4 / (64 * kWaves);
        float4 v[per];
#pragma unroll
        for (int u = 0; u < per; ++u) {
            const int c = u * (64 * kWaves) + threadIdx.x;
            const int o = c / (kHid / 4), col = (c % (kHid / 4)) * 4;
            v[u] = o < a.nh ? *reinterpret_cast<const float4*>(a.wh + o * kHid + col) : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < per; ++u) {
            const int c = u * (64 * kWaves) + threadIdx.x;
            *reinterpret_cast<float4*>(wl + (c / (kHid / 4)) * kHs + (c % (kHid / 4)) * 4) = v[u];
        }
    }
    float bq[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const int k = 2 * t + h;
        bq[t] = (live && k < a.nh) ? a.dhead[int64_t(row) * a.nh + k] : 0.f;
    }
    __syncthreads();
    f32x16 acc[kTiles];
#pragma unroll
    for (int ot = 0; ot < kTiles; ++ot) acc[ot] = f32x16{};
    const int nsteps = (a.nh + 1) / 2;
    for (int t = 0; t < nsteps; ++t) {
        const int k = 2 * t + h;
#pragma unroll
        for (int ot = 0; ot < kTiles; ++ot)
            acc[ot] = __builtin_amdgcn_mfma_f32_32x32x2f32(wl[k * kHs + ot * 32 + i], bq[t], acc[ot], 0, 0, 0);
    }
    V8 xb[kTiles][2];
    uint2 yb[kTiles][4];  // 16-bit activations of layer l - 1, loaded while layer l's MFMAs run
    for (int l = 4; l >= 0; --l) {
        // dz_l = dh * elu'(y_l), y_l = layer-l activations (layer 5 in fp32, the others 16-bit)
        uint16_t* __restrict__ dzo = a.dz[l];
#pragma unroll
        for (int ot = 0; ot < kTiles; ++ot) {
            float y[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int c = ot * 32 + 8 * g + 4 * h;
                if (!live) {
                    y[4 * g] = y[4 * g + 1] = y[4 * g + 2] = y[4 * g + 3] = 0.f;
                } else if (l == 4) {
                    const float4 q = *reinterpret_cast<const float4*>(a.h5 + int64_t(row) * kHid + c);
                    y[4 * g] = q.x;
                    y[4 * g + 1] = q.y;
                    y[4 * g + 2] = q.z;
                    y[4 * g + 3] = q.w;
                } else {
                    Frag<DT> ff;
                    ff.q[0] = yb[ot][g];
#pragma unroll
                    for (int e = 0; e < 4; ++e) y[4 * g + e] = float(ff.v[e]);
                }
            }
            Frag<DT> f[2];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float dz = y[r] > 0.f ? acc[ot][r] : acc[ot][r] * (y[r] + 1.f);
                f[r >> 3].v[r & 7] = (E)dz;
            }
            xb[ot][0] = f[0].v;
            xb[ot][1] = f[1].v;
            const uint4 c01 = pair_chunks(f[0].q[0], f[0].q[1]), c23 = pair_chunks(f[1].q[0], f[1].q[1]);
            if (live) {
                uint16_t* d = dzo + int64_t(row) * kHid + ot * 32 + 8 * h;
                *reinterpret_cast<uint4*>(d) = c01;
                *reinterpret_cast<uint4*>(d + 16) = c23;
            }
        }
        if (l == 0) break;
        // dh of layer l's input = W_l^T dz_l
        __syncthreads();
        stage_w<kHid>(lds, a.wt[l - 1]);
        __syncthreads();
        // issued after the staging loads have been waited for, so only the MFMAs below cover them
        if (live) {
            const uint16_t* __restrict__ yrow = a.h[l - 1] + int64_t(row) * a.h_stride + 4 * h;
#pragma unroll
            for (int ot = 0; ot < kTiles; ++ot)
#pragma unroll
                for (int g = 0; g < 4; ++g) yb[ot][g] = *reinterpret_cast<const uint2*>(yrow + ot * 32 + 8 * g);
        }
        layer_mma<kHid, DT>(lds, xb, acc, lane);
    }
}

}  // namespace

// the kernel of a dtype, with its dynamic-LDS reservation made once
template <typename F>
static int reserve_lds(F kernel, int bytes, bool& done, const char* what) {
    if (done) return 0;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            bytes) != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "%s: cannot reserve %d B of LDS", what, bytes);
        ppo_detail::set_error(g_err);
        return -2;
    }
    done = true;
    return 0;
}

extern "C" int ppo_mlp_backward(const ppo_mlp_bwd_t* args_host, void* stream) {
    if (!args_host || !args_host->dhead || args_host->nh <= 0 || args_host->nh > 32 || args_host->rows <= 0 ||
        args_host->h_stride < kHid || (args_host->dtype != PPO_DT_BF16 && args_host->dtype != PPO_DT_F16)) {
        snprintf(g_err, sizeof(g_err), "ppo_mlp_backward: bad arguments");
        ppo_detail::set_error(g_err);
        return -1;
    }
    static bool attr[2] = {false, false};
    const bool f16 = args_host->dtype == PPO_DT_F16;
    const int rc = f16 ? reserve_lds(k_mlp_bwd<PPO_DT_F16>, kWBytes, attr[1], "ppo_mlp_backward")
                       : reserve_lds(k_mlp_bwd<PPO_DT_BF16>, kWBytes, attr[0], "ppo_mlp_backward");
    if (rc) return rc;
    const int blocks = (args_host->rows + kRowsPerBlock - 1) / kRowsPerBlock;
    if (f16)
        hipLaunchKernelGGL(k_mlp_bwd<PPO_DT_F16>, dim3(blocks), dim3(64 * kWaves), kWBytes,
                           static_cast<hipStream_t>(stream), *args_host);
    else
        hipLaunchKernelGGL(k_mlp_bwd<PPO_DT_BF16>, dim3(blocks), dim3(64 * kWaves), kWBytes,
                           static_cast<hipStream_t>(stream), *args_host);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "k_mlp_bwd: %s", hipGetErrorString(e));
        ppo_detail::set_error(g_err);
        return -2;
    }
    return 0;
}

extern "C" int ppo_mlp_forward(const ppo_mlp_fwd_t* args_host, void* stream) {
    if (!args_host || !args_host->x || args_host->nh <= 0 || args_host->nh > 32 || args_host->rows <= 0 ||
        args_host->x_stride < kK0 || args_host->h_stride < kHid || (args_host->x_stride % 4) || (args_host->h_stride % 8) ||
        (args_host->dtype != PPO_DT_BF16 && args_host->dtype != PPO_DT_F16)) {
        snprintf(g_err, sizeof(g_err), "ppo_mlp_forward: bad arguments");
        ppo_detail::set_error(g_err);
        return -1;
    }
    static bool attr[2] = {false, false};
    const bool f16 = args_host->dtype == PPO_DT_F16;
    const int rc = f16 ? reserve_lds(k_mlp_fwd<PPO_DT_F16>, kLdsBytes, attr[1], "ppo_mlp_forward")
                       : reserve_lds(k_mlp_fwd<PPO_DT_BF16>, kLdsBytes, attr[0], "ppo_mlp_forward");
    if (rc) return rc;
    const int blocks = (args_host->rows + kRowsPerBlock - 1) / kRowsPerBlock;
    if (f16)
        hipLaunchKernelGGL(k_mlp_fwd<PPO_DT_F16>, dim3(blocks), dim3(64 * kWaves), kLdsBytes,
                           static_cast<hipStream_t>(stream), *args_host);
    else
        hipLaunchKernelGGL(k_mlp_fwd<PPO_DT_BF16>, dim3(blocks), dim3(64 * kWaves), kLdsBytes,
                           static_cast<hipStream_t>(stream), *args_host);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "k_mlp_fwd: %s", hipGetErrorString(e));
        ppo_detail::set_error(g_err);
        return -2;
    }
    return 0;
}

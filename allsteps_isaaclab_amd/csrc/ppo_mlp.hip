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
#include "ppo_loss.h"

namespace ppo_detail {
void set_error(const char* msg);
}

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

// ------------------------------------------------------------------------------ forward (weight-stationary)
//
// One workgroup of 8 waves per CU (two waves per SIMD) owns 128 batch rows (4 N-tiles of 32).  Wave w
// owns output features [32w, 32w + 32) of every layer and keeps ITS slice of the layer's weights in
// registers (the A fragments: 32 features x K, 16 B per lane per k-step), loaded straight from L2 while
// the previous layer's epilogue runs -- no weight staging through LDS.  The activations live in LDS
// (two [128][264] buffers, the B fragments: one ds_read_b128 per MFMA, 1 KB per 32-cycle MFMA per SIMD,
// half the LDS array's rate): layer l reads one buffer, its epilogue (bias + ELU in fp32, one rounding
// to the trunk's type) writes the other, one barrier per layer.  The two waves of a SIMD interleave one
// wave's epilogue with the other's MFMAs.  The heads (mu | value, nh <= 32 outputs) run on the 16-bit
// layer-5 activations with fp16 / bf16 weights and fp32 accumulation, as rl_games' autocast does
// (Linear under autocast: 16-bit inputs, fp32 accumulate, 16-bit output + bias), on waves 0..3 (one
// N-tile each).  The hidden layers are the previous (register-chained) form's arithmetic: the same
// ascending 16-wide k-steps accumulated in fp32 and the same epilogue; only the position of each
// product inside an MFMA's 16-element step differs (natural k order instead of the permuted one).
constexpr int kFWaves = 8;
constexpr int kFThreads = 64 * kFWaves;
constexpr int kFRows = 128;               // batch rows per workgroup (4 N-tiles of 32)
constexpr int kXs = kHid + kPad;          // LDS activation row stride, elements (132 dwords: conflict-free b128)
constexpr int kXBytes = kFRows * kXs * 2; // 67584 B per activation buffer
constexpr int kFLds = 2 * kXBytes;        // 135168 B

// A fragments of k-steps [0, NS) for features F0 + i: row F0 + i of a [256][K] 16-bit matrix, k 16s + 8h..+7
template <int DT, int NS>
__device__ __forceinline__ void load_wa(const uint16_t* __restrict__ w, int K, int F0, int i, int h,
                                        typename Lp<DT>::v8 (&wa)[16]) {
    typedef typename Lp<DT>::v8 V8;
    const uint16_t* p = w + int64_t(F0 + i) * K + 8 * h;
#pragma unroll
    for (int s = 0; s < NS; ++s) wa[s] = *reinterpret_cast<const V8*>(p + 16 * s);
}

// the heads' A fragments: fp32 wh[o][256] (o < nh, zero rows above) rounded to the trunk's type
template <int DT>
__device__ __forceinline__ void load_wh(const float* __restrict__ wh, int nh, int i, int h, typename Lp<DT>::v8 (&wa)[16]) {
    typedef typename Lp<DT>::e E;
    const bool ok = i < nh;
    const float* p = wh + (ok ? i : 0) * kHid + 8 * h;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const float4 u = ok ? *reinterpret_cast<const float4*>(p + 16 * s) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 v = ok ? *reinterpret_cast<const float4*>(p + 16 * s + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        wa[s][0] = (E)u.x; wa[s][1] = (E)u.y; wa[s][2] = (E)u.z; wa[s][3] = (E)u.w;
        wa[s][4] = (E)v.x; wa[s][5] = (E)v.y; wa[s][6] = (E)v.z; wa[s][7] = (E)v.w;
    }
}

// bias of features F0 + feat(r, h) (16 per lane)
__device__ __forceinline__ void load_bias(const float* __restrict__ b, int F0, int h, float (&bv)[16]) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 q = *reinterpret_cast<const float4*>(b + F0 + 8 * g + 4 * h);
        bv[4 * g] = q.x; bv[4 * g + 1] = q.y; bv[4 * g + 2] = q.z; bv[4 * g + 3] = q.w;
    }
}

// acc[t] = W_slice (32 x 16 NS) . X[rows 32 (T0 + t) + 0..31] for t < NT; B fragments read from the LDS
// activation image one k-step ahead of their MFMAs
template <int DT, int NS, int NT>
__device__ __forceinline__ void mma_rows(const uint16_t* X, const typename Lp<DT>::v8 (&wa)[16], f32x16 (&acc)[4],
                                         int T0, int j, int h) {
    typedef typename Lp<DT>::v8 V8;
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
    V8 bf[2][NT];
    const uint16_t* xr = X + (32 * T0 + j) * kXs + 8 * h;
#pragma unroll
    for (int t = 0; t < NT; ++t) bf[0][t] = *reinterpret_cast<const V8*>(xr + 32 * t * kXs);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (s + 1 < NS) {
#pragma unroll
            for (int t = 0; t < NT; ++t) bf[(s + 1) & 1][t] = *reinterpret_cast<const V8*>(xr + 32 * t * kXs + 16 * (s + 1));
        }
        __builtin_amdgcn_sched_barrier(0);  // the next k-step's reads stay ahead of this k-step's MFMAs
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = Lp<DT>::mma(wa[s], bf[s & 1][t], acc[t]);
    }
}

#ifndef PPO_MLP_PRIO
// A/B knob: static s_setprio 1 for waves 4..7 of the trunk kernels (MI355X_MICROARCH.md "Two waves per
// SIMD" item 4).  Measured with each library in its own processes (scripts/mlp_ab.py, r05t): forward 46.7 /
// 46.9 us, backward 43.3 / 43.7 us without / with -- no gain, so off
#define PPO_MLP_PRIO 0
#endif
#ifndef PPO_MMA_PD
#define PPO_MMA_PD 4  // B-fragment reads issued this many k-steps ahead of their MFMA (A/B knob)
#endif
#ifndef PPO_MMA_SCHED
#define PPO_MMA_SCHED 1  // the sched_barriers that keep the reads and MFMAs in order (A/B knob)
#endif
#ifndef PPO_FWD_SINGLE_W
#define PPO_FWD_SINGLE_W 0
#endif
#ifndef PPO_FWD_COPY
// A/B knob.  1: the layers' activation stores leave through full-row copies of the LDS image (every wave
// store 1 KB contiguous: two whole rows) once a tile row block is complete, instead of each wave storing its
// own 32 features (32-B runs per row) from its epilogue -- the same bytes and values (bit-identical, r06f).
// Measured (DESIGN §7 "Round 6"): the standalone forward 44.1 -> 43.0 us, but the training forward with the
// fused losses slower (update_s 0.0513 -> 0.0520 s): off.  (A timing-only build with the stores made
// contiguous in a wrong layout, PPO_FWD_DBG 256, put the row pattern's share of the store cost at 4.4 of
// ~10 us; the copies' extra LDS reads and the tail copies give most of it back.)
#define PPO_FWD_COPY 0
#endif
#ifndef PPO_FWD_DBG
#define PPO_FWD_DBG 0  // timing-only builds (scripts/fwd_dbg.sh): 2 no exp, 4 no stores, 16 no MFMA, 32 no ELU / convert,
                       // 64 no loss block, 128 no heads, 256 the activation stores as contiguous 1-KB wave stores
                       // (wrong layout: is the 32-B-run row pattern what the stores cost?); backward: 512 dz
                       // stores contiguous, 1024 y loads contiguous, 2048 no y loads, 4096 no dz stores
#endif

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef __amdgpu_buffer_rsrc_t Rsrc;

// a range-checked buffer over `bytes` bytes from p (uniform kernel-argument inputs): stores past the
// end are dropped by the hardware, so the partial last workgroup needs no per-row branch (a branch
// would split the block the scheduler interleaves)
__device__ __forceinline__ Rsrc rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(bytes > 0x7fffffff ? 0x7fffffff : bytes),
                                             0x00020000);
}

__device__ __forceinline__ u32x4_t u4(uint4 v) { return u32x4_t{v.x, v.y, v.z, v.w}; }

// ELU (alpha 1) of one tile's fp32 values (bias already in the accumulator), one rounding to the 16-bit
// type: the next layer's LDS image and, when STORE, the layer's global activations.  Lane (j, h) holds
// row j, features F0 + feat(r, h).
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// two fp32 values -> one dword of two 16-bit values (v_cvt_pk_f16_f32 / v_cvt_pk_bf16_f32, round to
// nearest even)
template <int DT>
__device__ __forceinline__ uint32_t pack2(f32x2_t v) {
    typedef typename Lp<DT>::e E;
    typedef E e2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, e2));
}

template <int DT, bool STORE>
__device__ __forceinline__ void tile_epi(const f32x16& acc, uint16_t* Xn, int rl, int row, Rsrc rh, int h_stride, int F0,
                                         int h) {
    // ELU(z) = med3(exp(z) - 1, z, 0): for z > 0 the three sort as 0 < z < e^z - 1, for z <= 0 as
    // z <= e^z - 1 <= 0, so the median is z or e^z - 1 -- one v_med3_f32 instead of a compare + select
    // (and its VCC hazard).  exp(z) - 1 = exp2(z log2 e) - 1 as __expf (|error| ~1e-7, far below the 16-bit
    // step).  Scalar f32 ops only: packed f32 VALU costs extra issue cycles beside the MFMAs.
    uint32_t dw[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float y[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float z = acc[2 * k + e];
            y[e] = __builtin_amdgcn_fmed3f(__builtin_amdgcn_exp2f(z * 1.44269502f) - 1.f, z, 0.f);
        }
        dw[k] = pack2<DT>(f32x2_t{y[0], y[1]});
    }
#if PPO_FWD_DBG & 2
#pragma unroll
    for (int k = 0; k < 8; ++k) dw[k] = pack2<DT>(f32x2_t{acc[2 * k], acc[2 * k + 1]});
#endif
#if PPO_FWD_DBG & 32
#pragma unroll
    for (int k = 0; k < 8; ++k) dw[k] = __builtin_bit_cast(uint32_t, acc[2 * k]) ^ __builtin_bit_cast(uint32_t, acc[2 * k + 1]);
#endif
    // dwords 2g, 2g + 1 = features 8g + 4h + 0..3 (register r = 4g + e)
    const uint4 c01 = pair_chunks(make_uint2(dw[0], dw[1]), make_uint2(dw[2], dw[3]));
    const uint4 c23 = pair_chunks(make_uint2(dw[4], dw[5]), make_uint2(dw[6], dw[7]));
    uint16_t* xn = Xn + rl * kXs + F0 + 8 * h;
    *reinterpret_cast<uint4*>(xn) = c01;
    *reinterpret_cast<uint4*>(xn + 16) = c23;
    if (STORE && !PPO_FWD_COPY) {
#if PPO_FWD_DBG & 256
        // timing-only: the same bytes as fully contiguous 1-KB wave stores (wrong layout)
        const int tb = (row - (threadIdx.x & 31)) * h_stride * 2 + (F0 / 32) * 2 * 2048 + 16 * int(threadIdx.x & 63);
        __builtin_amdgcn_raw_buffer_store_b128(u4(c01), rh, tb, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(u4(c23), rh, tb + 1024, 0, 0);
#else
        const int off = (row * h_stride + F0 + 8 * h) * 2;
        __builtin_amdgcn_raw_buffer_store_b128(u4(c01), rh, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(u4(c23), rh, off + 32, 0, 0);
#endif
    }
}

// Rows [r0, r0 + NR) of the LDS activation image X (features 0..255) to global rows row0 + r0.. of rh (range-
// checked): 16-B chunks, 32 per row, consecutive threads on consecutive chunks, so every wave store covers two
// whole 512-B rows.  The constant ones column (256) of the global rows is left alone.
template <int NR>
__device__ __forceinline__ void copy_rows(const uint16_t* X, int r0, Rsrc rh, int h_stride, int row0) {
    constexpr int kChunks = NR * (kHid / 8);
    static_assert(kChunks % kFThreads == 0, "whole chunks per thread");
#pragma unroll
    for (int u = 0; u < kChunks / kFThreads; ++u) {
        const int c = u * kFThreads + int(threadIdx.x), r = r0 + c / (kHid / 8), q = c % (kHid / 8);
        const uint4 v = *reinterpret_cast<const uint4*>(X + r * kXs + 8 * q);
        __builtin_amdgcn_raw_buffer_store_b128(u4(v), rh, ((row0 + r) * h_stride + 8 * q) * 2, 0, 0);
    }
}

// The MFMAs of one N-tile (32 rows) for the wave's 32 features: NS k-steps accumulated onto `c` (the
// bias), B fragments PD k-steps ahead of their MFMA (an LDS read's latency is ~4 MFMA issue slots);
// the reads and MFMAs keep their order (sched_barrier), the VALU, LDS writes and stores of an epilogue
// placed beside them in the source may move across (mask: ALU | VALU | SALU | VMEM write | DS write).
template <int DT, int NS>
__device__ __forceinline__ f32x16 mfma_tile(const uint16_t* X, const typename Lp<DT>::v8 (&wa)[16], f32x16 c, int t,
                                            int j, int h) {
    typedef typename Lp<DT>::v8 V8;
    constexpr int PD = NS < PPO_MMA_PD ? NS : PPO_MMA_PD;
    constexpr int kFloat = 0x1 | 0x2 | 0x4 | 0x40 | 0x200;
    const uint16_t* xr = X + (32 * t + j) * kXs + 8 * h;
    V8 b[NS];
#pragma unroll
    for (int s = 0; s < PD; ++s) b[s] = *reinterpret_cast<const V8*>(xr + 16 * s);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (s + PD < NS) b[s + PD] = *reinterpret_cast<const V8*>(xr + 16 * (s + PD));
#if PPO_MMA_SCHED
        __builtin_amdgcn_sched_barrier(kFloat);
#endif
#if PPO_FWD_DBG & 16
        c[s & 15] += __builtin_bit_cast(float, uint32_t(b[s][0] != b[s][1]));
#else
        c = Lp<DT>::mma(wa[s], b[s], c);
#endif
#if PPO_MMA_SCHED
        __builtin_amdgcn_sched_barrier(kFloat);
#endif
    }
    return c;
}

// One layer of the wave's 32 output features over the workgroup's 4 N-tiles, software-pipelined by
// tile so that every phase carries matrix work AND epilogue work (exp / convert / stores): phase 0 runs
// this layer's tile-0 MFMAs beside the PREVIOUS layer's tile-3 epilogue (`pend`, written into rows
// 96..127 of this layer's input), phase t (1..3) tile t's MFMAs beside tile t - 1's epilogue; tile 3's
// accumulator is handed on to the next layer (or the last layer's own tail).  Two barriers per layer:
// before phase 3 (rows 96..127 of the input, which phase 0 completed, are read there) and at the end
// (rows 0..95 of the output complete; every read of the input done before the layer after the next
// overwrites it).
template <int DT, int NS, bool STORE, bool HAS_PREV>
__device__ __forceinline__ void layer(const uint16_t* Xin, uint16_t* Xout, const typename Lp<DT>::v8 (&wa)[16],
                                      const float (&bv)[16], f32x16& pend, Rsrc rh_prev, Rsrc rh, int h_stride, int row0,
                                      int F0, int j, int h) {
    f32x16 binit;
#pragma unroll
    for (int r = 0; r < 16; ++r) binit[r] = bv[r];
    const f32x16 c0 = mfma_tile<DT, NS>(Xin, wa, binit, 0, j, h);
    if (HAS_PREV)
        tile_epi<DT, STORE>(pend, const_cast<uint16_t*>(Xin), 96 + j, row0 + 96 + j, rh_prev, h_stride, F0, h);
    // the previous layer's output (this layer's input image) leaves by row copies: rows 0..95 (complete since
    // the previous layer's last barrier) beside tiles 1 and 2, rows 96..127 beside tile 3
    if (STORE && PPO_FWD_COPY && HAS_PREV) copy_rows<48>(Xin, 0, rh_prev, h_stride, row0);
    const f32x16 c1 = mfma_tile<DT, NS>(Xin, wa, binit, 1, j, h);
    tile_epi<DT, STORE>(c0, Xout, j, row0 + j, rh, h_stride, F0, h);
    if (STORE && PPO_FWD_COPY && HAS_PREV) copy_rows<48>(Xin, 48, rh_prev, h_stride, row0);
    const f32x16 c2 = mfma_tile<DT, NS>(Xin, wa, binit, 2, j, h);
    tile_epi<DT, STORE>(c1, Xout, 32 + j, row0 + 32 + j, rh, h_stride, F0, h);
    __syncthreads();
    if (STORE && PPO_FWD_COPY && HAS_PREV) copy_rows<32>(Xin, 96, rh_prev, h_stride, row0);
    const f32x16 c3 = mfma_tile<DT, NS>(Xin, wa, binit, 3, j, h);
    tile_epi<DT, STORE>(c2, Xout, 64 + j, row0 + 64 + j, rh, h_stride, F0, h);
    pend = c3;
    __syncthreads();
}

template <int DT, bool STORE, int LA>
__device__ __forceinline__ void mlp_fwd_body(const ppo_mlp_fwd_t& a) {
    typedef typename Lp<DT>::e E;
    typedef typename Lp<DT>::v8 V8;
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    uint16_t* X0 = lds;
    uint16_t* X1 = lds + kFRows * kXs;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
#if PPO_MLP_PRIO
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half wins VALU arbitration
#endif
    const int j = lane & 31, h = lane >> 5, i = lane & 31;
    const int F0 = 32 * wave;                 // this wave's output features
    const int row0 = blockIdx.x * kFRows;
    const int rows = a.rows;
    if (a.obs) {
        // the input normalisation fused in (ppo_obs_normalize's formula): the column constants (float(mean),
        // sqrtf(float(var) + eps)) formed once per workgroup into scratch at the head of X1 (layer 0 writes
        // X1 only after the barriers below), then thread -> row tid / 4, 16 columns, its 16 loads issued
        // together (after the barrier: held across it they pushed the kernel past 256 VGPRs)
        static_assert(kFRows * kK0 == 16 * kFThreads, "16 input columns per thread");
        float* nm = reinterpret_cast<float*>(X1);
        float* nd = nm + kK0;
        if (threadIdx.x < kK0) {
            const int c = threadIdx.x;
            const bool in = c < a.obs_dim;
            nm[c] = in ? float(a.mean[c]) : 0.f;
            nd[c] = in ? sqrtf(float(a.var[c]) + a.eps) : 1.f;
        }
        __syncthreads();
        const int r = threadIdx.x >> 2, c0 = 16 * (threadIdx.x & 3), row = row0 + r;
        const float* src = a.obs + (int64_t(*a.mb_idx) * rows + row) * a.obs_dim;
        float x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = c0 + k < a.obs_dim && row < rows ? src[c0 + k] : 0.f;
        uint32_t dw[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float v[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int c = c0 + 2 * k + e;
                v[e] = c < a.obs_dim && row < rows ? fminf(fmaxf((x[2 * k + e] - nm[c]) / nd[c], -5.f), 5.f) : 0.f;
            }
            dw[k] = pack2<DT>(f32x2_t{v[0], v[1]});
        }
        const uint4 lo = make_uint4(dw[0], dw[1], dw[2], dw[3]), hi = make_uint4(dw[4], dw[5], dw[6], dw[7]);
        *reinterpret_cast<uint4*>(X0 + r * kXs + c0) = lo;
        *reinterpret_cast<uint4*>(X0 + r * kXs + c0 + 8) = hi;
        if (a.x_out && row < rows) {
            uint16_t* d = a.x_out + int64_t(row) * a.x_stride + c0;
            *reinterpret_cast<uint4*>(d) = lo;
            *reinterpret_cast<uint4*>(d + 8) = hi;
        }
    } else {
        // layer-0 input rows -> X0 (16-B chunks, zero past `rows`)
#pragma unroll
        for (int u = 0; u < kFRows * (kK0 / 8) / kFThreads; ++u) {
            const int c = u * kFThreads + threadIdx.x, r = c / (kK0 / 8), q = c % (kK0 / 8);
            uint4 v = make_uint4(0, 0, 0, 0);
            if (row0 + r < rows) v = *reinterpret_cast<const uint4*>(a.x + int64_t(row0 + r) * a.x_stride + 8 * q);
            *reinterpret_cast<uint4*>(X0 + r * kXs + 8 * q) = v;
        }
    }
    const int hs = a.h_stride;
    Rsrc rh[5];
#pragma unroll
    for (int l = 0; l < 5; ++l) rh[l] = rsrc(STORE ? a.h[l] : nullptr, STORE ? int64_t(rows) * hs * 2 : 0);
    f32x16 pend = {};
    float bhv[16];
#if PPO_FWD_SINGLE_W
    // timing variant: ONE register set of weights, each layer's slice loaded after the previous layer's
    // MFMAs (64 VGPRs freed for the B-fragment prefetch; the load latency exposed once per layer).
    // Measured (r05t): 48.0 -> 55.4 us -- the compiler fills the freed registers and spills
    V8 wa[16];
    float ba[16];
    load_wa<DT, kK0 / 16>(a.w[0], kK0, F0, i, h, wa);
    load_bias(a.b[0], F0, h, ba);
    __syncthreads();
    layer<DT, kK0 / 16, STORE, false>(X0, X1, wa, ba, pend, rh[0], rh[0], hs, row0, F0, j, h);
    load_wa<DT, 16>(a.w[1], kHid, F0, i, h, wa);
    load_bias(a.b[1], F0, h, ba);
    layer<DT, 16, STORE, true>(X1, X0, wa, ba, pend, rh[0], rh[1], hs, row0, F0, j, h);
    load_wa<DT, 16>(a.w[2], kHid, F0, i, h, wa);
    load_bias(a.b[2], F0, h, ba);
    layer<DT, 16, STORE, true>(X0, X1, wa, ba, pend, rh[1], rh[2], hs, row0, F0, j, h);
    load_wa<DT, 16>(a.w[3], kHid, F0, i, h, wa);
    load_bias(a.b[3], F0, h, ba);
    layer<DT, 16, STORE, true>(X1, X0, wa, ba, pend, rh[2], rh[3], hs, row0, F0, j, h);
    load_wa<DT, 16>(a.w[4], kHid, F0, i, h, wa);
    load_bias(a.b[4], F0, h, ba);
#pragma unroll
    for (int r = 0; r < 16; ++r) bhv[r] = feat(r, h) < a.nh ? a.bh[feat(r, h)] : 0.f;
    layer<DT, 16, STORE, true>(X0, X1, wa, ba, pend, rh[3], rh[4], hs, row0, F0, j, h);
    tile_epi<DT, STORE>(pend, X1, 96 + j, row0 + 96 + j, rh[4], hs, F0, h);
    if (wave < 4) load_wh<DT>(a.wh, a.nh, i, h, wa);
    V8 (&whf)[16] = wa;
#else
    // Weight slices double-buffered in registers (wa / wb): layer l + 1's slice is requested at the start
    // of layer l, ahead of layer l's activation stores (a load waited for with vmcnt also waits for every
    // older store of the wave).  Bias vectors likewise one layer ahead.
    V8 wa[16], wb[16];
    float ba[16], bb[16];
    load_wa<DT, kK0 / 16>(a.w[0], kK0, F0, i, h, wa);
    load_bias(a.b[0], F0, h, ba);
    __syncthreads();
    load_wa<DT, 16>(a.w[1], kHid, F0, i, h, wb);
    load_bias(a.b[1], F0, h, bb);
    layer<DT, kK0 / 16, STORE, false>(X0, X1, wa, ba, pend, rh[0], rh[0], hs, row0, F0, j, h);
    load_wa<DT, 16>(a.w[2], kHid, F0, i, h, wa);
    load_bias(a.b[2], F0, h, ba);
    layer<DT, 16, STORE, true>(X1, X0, wb, bb, pend, rh[0], rh[1], hs, row0, F0, j, h);
    load_wa<DT, 16>(a.w[3], kHid, F0, i, h, wb);
    load_bias(a.b[3], F0, h, bb);
    layer<DT, 16, STORE, true>(X0, X1, wa, ba, pend, rh[1], rh[2], hs, row0, F0, j, h);
    load_wa<DT, 16>(a.w[4], kHid, F0, i, h, wa);
    load_bias(a.b[4], F0, h, ba);
    layer<DT, 16, STORE, true>(X1, X0, wb, bb, pend, rh[2], rh[3], hs, row0, F0, j, h);
    // the fifth layer; the heads' weights and biases fly under it
    if (wave < 4) load_wh<DT>(a.wh, a.nh, i, h, wb);
#pragma unroll
    for (int r = 0; r < 16; ++r) bhv[r] = feat(r, h) < a.nh ? a.bh[feat(r, h)] : 0.f;
    layer<DT, 16, STORE, true>(X0, X1, wa, ba, pend, rh[3], rh[4], hs, row0, F0, j, h);
    tile_epi<DT, STORE>(pend, X1, 96 + j, row0 + 96 + j, rh[4], hs, F0, h);
    if (STORE && PPO_FWD_COPY) copy_rows<96>(X1, 0, rh[4], hs, row0);  // layer 5's rows 0..95 (complete)
    V8 (&whf)[16] = wb;
#endif
    // ---- fused losses (LA > 0): ppo_loss_grad's work for the block's rows (ppo_loss.h), eight lanes per row
    // in two passes.  Their dataset loads are issued here, ahead of the heads, so the round trip overlaps the
    // heads' MFMAs and the two barriers (layer 5's weights are dead: the registers are free)
    constexpr int kHS = (LA + 1) | 1;
    float* sh = reinterpret_cast<float*>(X0);
    ppo_detail::LossRowArgs p{};
    ppo_detail::LossIn<LA> lin[LA > 0 ? ppo_detail::loss_passes<kFThreads>() : 1];
    if constexpr (LA > 0) {
        p.head = sh;
        p.head_stride = kHS;
        p.head_block_rows = false;
        p.logstd = a.loss.logstd;
        p.mb_rows = rows;
        p.mb_idx = a.mb_idx;
        p.actions = a.loss.actions;
        p.ds_mu = a.loss.ds_mu;
        p.ds_sigma = a.loss.ds_sigma;
        p.old_nlp = a.loss.old_neglogp;
        p.adv = a.loss.advantages;
        p.old_v = a.loss.old_values;
        p.ret = a.loss.returns;
        p.cfg = a.loss.cfg;
        p.grad_scale = a.loss.grad_scale;
        p.dhead = nullptr;
        p.dhead_lp = a.loss.dhead_lp;
        p.lp_dtype = DT;
        p.partials = a.loss.partials;
        static_assert(kFRows == ppo_detail::kLossRows, "one loss block per workgroup");
        static_assert(ppo_detail::loss_lds_floats(LA) * 4 <= kXBytes, "the loss tables fit the free image");
        ppo_detail::loss_prefetch<LA, kFThreads>(p, blockIdx.x, lin);
    }
    __syncthreads();
    if (STORE && PPO_FWD_COPY) copy_rows<32>(X1, 96, rh[4], hs, row0);  // layer 5's rows 96..127
    // ---- heads: wave w < 4 takes N-tile w; out = 16-bit(acc + 16-bit(bh)) as under autocast.  With the
    // fused losses (LA > 0) the values also go to a table of the block's rows at the head of X0 (free: layer
    // 5 has read it), the losses' input
    if (wave < 4 && a.head && !(PPO_FWD_DBG & 128)) {
        f32x16 hacc[4];
        mma_rows<DT, 16, 1>(X1, whf, hacc, wave, j, h);
        const int rl = 32 * wave + j, row = row0 + rl;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = feat(r, h);
            const float v = float((E)(hacc[0][r] + float((E)bhv[r])));
            if (o < a.nh && row < rows) a.head[int64_t(row) * a.nh + o] = v;
            if (LA > 0 && o <= LA) sh[rl * kHS + o] = v;
        }
    }
    if constexpr (LA > 0) {
        // the losses' per-row table in X1 (the heads' MFMAs have read it)
        __syncthreads();
        if (!(PPO_FWD_DBG & 64)) ppo_detail::loss_block<LA, kFThreads>(p, blockIdx.x, reinterpret_cast<float*>(X1), lin);
    }
}

template <int DT, int LA>
__global__ void __launch_bounds__(kFThreads, 1) k_mlp_fwd(ppo_mlp_fwd_t a) {
    // training stores layers 1..5 for the backward (all five pointers set); the rollout form stores none
    if constexpr (LA > 0) {
        mlp_fwd_body<DT, !(PPO_FWD_DBG & 4), LA>(a);
    } else {
        if (a.h[0] && !(PPO_FWD_DBG & 4))
            mlp_fwd_body<DT, true, 0>(a);
        else
            mlp_fwd_body<DT, false, 0>(a);
    }
}

// ------------------------------------------------------------------------------ backward chain
//
// The forward's layout run backwards (weight-stationary, 8 waves, 128 rows, two LDS images): stage H
// forms dh5 = Wh^T dhead for the wave's 32 features of layer 5 (lp MFMAs with fp32 accumulation on the
// 16-bit dhead and lp(Wh), as autocast runs the heads' Linear backward), then each stage l = 4..1 forms
// dh = W_l^T dz_l for the wave's 32 INPUT features of layer l (the A fragments: rows of the 16-bit W_l^T
// mirror, in registers, loaded one stage ahead; the B fragments: dz_l from LDS), and every epilogue turns
// dh into dz = dh * elu'(y) (y > 0 ? 1 : y + 1, the output form) with y the layer's stored 16-bit
// activations, rounds it once, writes it to the next stage's LDS image and to dz[l] for the weight
// gradients.  Same tile pipelining and barriers as the forward.

// y of tile rows for the wave's features F0 + feat(r, h): 16-bit activations, 8 dwords
struct YT {
    u32x2_t v[4];
};

__device__ __forceinline__ YT load_y(Rsrc ry, int row, int stride, int F0, int h) {
    YT y;
#pragma unroll
#if PPO_FWD_DBG & 2048
    for (int g = 0; g < 4; ++g) y.v[g] = u32x2_t{0u, 0u};  // timing-only: no y loads
#elif PPO_FWD_DBG & 1024
    // timing-only: the same bytes as contiguous 512-B wave loads (wrong values)
    for (int g = 0; g < 4; ++g)
        y.v[g] = __builtin_amdgcn_raw_buffer_load_b64(ry, (row - int(threadIdx.x & 31)) * stride * 2 + F0 * 64 + 512 * g +
                                                               8 * int(threadIdx.x & 63), 0, 0);
#else
    for (int g = 0; g < 4; ++g) y.v[g] = __builtin_amdgcn_raw_buffer_load_b64(ry, (row * stride + F0 + 8 * g + 4 * h) * 2, 0, 0);
#endif
    return y;
}

template <int DT>
__device__ __forceinline__ float y_at(const YT& y, int r) {
    typedef typename Lp<DT>::e E;
    const uint32_t d = y.v[r >> 2][(r & 3) >> 1];
    const uint16_t u = (r & 1) ? uint16_t(d >> 16) : uint16_t(d & 0xffff);
    return float(__builtin_bit_cast(E, u));
}

// dz of one tile: dh * elu'(y) in fp32, one rounding; into the next stage's LDS image and dz (global,
// rows x 256, range-checked)
template <int DT>
__device__ __forceinline__ void tile_bepi(const f32x16& dh, const YT& y, uint16_t* Xn, int rl, int row, Rsrc rdz, int F0,
                                          int h) {
    uint32_t dw[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float v[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int r = 2 * k + e;
            // elu'(y) = y > 0 ? 1 : y + 1 = min(y + 1, 1) = clamp(y + 1, 0, 1) for ELU outputs (y >= -1):
            // one v_add_f32 with the clamp modifier; dh * 1 is dh, so the value is the select's exactly
            v[e] = dh[r] * __builtin_amdgcn_fmed3f(y_at<DT>(y, r) + 1.f, 0.f, 1.f);
        }
        dw[k] = pack2<DT>(f32x2_t{v[0], v[1]});
    }
    const uint4 c01 = pair_chunks(make_uint2(dw[0], dw[1]), make_uint2(dw[2], dw[3]));
    const uint4 c23 = pair_chunks(make_uint2(dw[4], dw[5]), make_uint2(dw[6], dw[7]));
    uint16_t* xn = Xn + rl * kXs + F0 + 8 * h;
    *reinterpret_cast<uint4*>(xn) = c01;
    *reinterpret_cast<uint4*>(xn + 16) = c23;
#if PPO_FWD_DBG & 4096
    (void)row; (void)rdz;  // timing-only: no dz stores
#elif PPO_FWD_DBG & 512
    // timing-only: the same bytes as contiguous 1-KB wave stores (wrong layout)
    const int tb = (row - int(threadIdx.x & 31)) * kHid * 2 + F0 * 128 + 16 * int(threadIdx.x & 63);
    __builtin_amdgcn_raw_buffer_store_b128(u4(c01), rdz, tb, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(u4(c23), rdz, tb + 1024, 0, 0);
#else
    const int off = (row * kHid + F0 + 8 * h) * 2;
    __builtin_amdgcn_raw_buffer_store_b128(u4(c01), rdz, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(u4(c23), rdz, off + 32, 0, 0);
#endif
}

// stage l = 4..1: dh = W_l^T dz_l (Xin) for the wave's input features, epilogue against y (layer l - 1's
// activations, ry) into Xout and dz[l - 1]; phase 0 also finishes the previous stage's tile 3 (pend,
// against ypend, into Xin rows 96..127 and dz[l]); HAS_PREV = false for the first stage (stage H
// completed all four of its tiles)
template <int DT, bool HAS_PREV>
__device__ __forceinline__ void bstage(const uint16_t* Xin, uint16_t* Xout, const typename Lp<DT>::v8 (&wa)[16],
                                       f32x16& pend, YT& yp, Rsrc rdz_prev, Rsrc ry, int y_stride, Rsrc rdz, int row0,
                                       int F0, int j, int h) {
    const f32x16 zero = {};
    YT y0 = load_y(ry, row0 + j, y_stride, F0, h);
    const f32x16 c0 = mfma_tile<DT, 16>(Xin, wa, zero, 0, j, h);
    if (HAS_PREV) tile_bepi<DT>(pend, yp, const_cast<uint16_t*>(Xin), 96 + j, row0 + 96 + j, rdz_prev, F0, h);
    YT y1 = load_y(ry, row0 + 32 + j, y_stride, F0, h);
    const f32x16 c1 = mfma_tile<DT, 16>(Xin, wa, zero, 1, j, h);
    tile_bepi<DT>(c0, y0, Xout, j, row0 + j, rdz, F0, h);
    YT y2 = load_y(ry, row0 + 64 + j, y_stride, F0, h);
    const f32x16 c2 = mfma_tile<DT, 16>(Xin, wa, zero, 2, j, h);
    tile_bepi<DT>(c1, y1, Xout, 32 + j, row0 + 32 + j, rdz, F0, h);
    if (HAS_PREV) __syncthreads();
    yp = load_y(ry, row0 + 96 + j, y_stride, F0, h);
    const f32x16 c3 = mfma_tile<DT, 16>(Xin, wa, zero, 3, j, h);
    tile_bepi<DT>(c2, y2, Xout, 64 + j, row0 + 64 + j, rdz, F0, h);
    pend = c3;
    __syncthreads();
}

template <int DT>
__global__ void __launch_bounds__(kFThreads, 1) k_mlp_bwd(ppo_mlp_bwd_t a) {
    typedef typename Lp<DT>::v8 V8;
    typedef typename Lp<DT>::e E;
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    uint16_t* X0 = lds;
    uint16_t* X1 = lds + kFRows * kXs;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
#if PPO_MLP_PRIO
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half wins VALU arbitration
#endif
    const int j = lane & 31, h = lane >> 5, i = lane & 31;
    const int F0 = 32 * wave;
    const int row0 = blockIdx.x * kFRows;
    const int rows = a.rows, nh = a.nh, hs = a.h_stride;
    Rsrc rdz[5], rh[5];
#pragma unroll
    for (int l = 0; l < 5; ++l) rdz[l] = rsrc(a.dz[l], int64_t(rows) * kHid * 2);
#pragma unroll
    for (int l = 0; l < 5; ++l) rh[l] = rsrc(a.h[l], int64_t(rows) * hs * 2);
    const Rsrc rdh = rsrc(a.dhead, int64_t(rows) * 32 * 2);
    // ---- stage H: dh5 = Wh^T dhead (A[i][k] = lp(wh[k][F0 + i]), k = 16s + 8h + e; B[k][n] = dhead[n][k])
    V8 ah[2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = 16 * s + 8 * h + e;
            ah[s][e] = (E)(k < nh ? a.wh[k * kHid + F0 + i] : 0.f);
        }
    V8 wa[16], wb[16];
    load_wa<DT, 16>(a.wt[3], kHid, F0, i, h, wa);  // W_4^T, the first hidden stage's slice
    YT y5[4];
    f32x16 dh5[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int row = row0 + 32 * t + j;
        y5[t] = load_y(rh[4], row, hs, F0, h);
        f32x16 c = {};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if (16 * s < nh) {  // uniform
                const u32x4_t q = __builtin_amdgcn_raw_buffer_load_b128(rdh, (row * 32 + 16 * s + 8 * h) * 2, 0, 0);
                c = Lp<DT>::mma(ah[s], __builtin_bit_cast(V8, q), c);
            }
        }
        dh5[t] = c;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) tile_bepi<DT>(dh5[t], y5[t], X0, 32 * t + j, row0 + 32 * t + j, rdz[4], F0, h);
    __syncthreads();
    // ---- stages 4..1 (dz_l in the LDS image -> dz_{l-1}); the next stage's W^T slice flies under each
    f32x16 pend = {};
    YT yp;
    load_wa<DT, 16>(a.wt[2], kHid, F0, i, h, wb);
    bstage<DT, false>(X0, X1, wa, pend, yp, rdz[4], rh[3], hs, rdz[3], row0, F0, j, h);
    load_wa<DT, 16>(a.wt[1], kHid, F0, i, h, wa);
    bstage<DT, true>(X1, X0, wb, pend, yp, rdz[3], rh[2], hs, rdz[2], row0, F0, j, h);
    load_wa<DT, 16>(a.wt[0], kHid, F0, i, h, wb);
    bstage<DT, true>(X0, X1, wa, pend, yp, rdz[2], rh[1], hs, rdz[1], row0, F0, j, h);
    bstage<DT, true>(X1, X0, wb, pend, yp, rdz[1], rh[0], hs, rdz[0], row0, F0, j, h);
    tile_bepi<DT>(pend, yp, X0, 96 + j, row0 + 96 + j, rdz[0], F0, h);
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
    bool ok = args_host && args_host->dhead && args_host->wh && args_host->nh > 0 && args_host->nh <= 32 &&
              args_host->rows > 0 && args_host->h_stride >= kHid && args_host->h_stride % 8 == 0 &&
              (args_host->dtype == PPO_DT_BF16 || args_host->dtype == PPO_DT_F16);
    for (int l = 0; ok && l < 5; ++l) ok = args_host->h[l] && args_host->dz[l] && (l == 4 || args_host->wt[l]);
    if (!ok) {
        snprintf(g_err, sizeof(g_err), "ppo_mlp_backward: bad arguments");
        ppo_detail::set_error(g_err);
        return -1;
    }
    static bool attr[2] = {false, false};
    const bool f16 = args_host->dtype == PPO_DT_F16;
    const int rc = f16 ? reserve_lds(k_mlp_bwd<PPO_DT_F16>, kFLds, attr[1], "ppo_mlp_backward")
                       : reserve_lds(k_mlp_bwd<PPO_DT_BF16>, kFLds, attr[0], "ppo_mlp_backward");
    if (rc) return rc;
    const int blocks = (args_host->rows + kFRows - 1) / kFRows;
    if (f16)
        hipLaunchKernelGGL(k_mlp_bwd<PPO_DT_F16>, dim3(blocks), dim3(kFThreads), kFLds,
                           static_cast<hipStream_t>(stream), *args_host);
    else
        hipLaunchKernelGGL(k_mlp_bwd<PPO_DT_BF16>, dim3(blocks), dim3(kFThreads), kFLds,
                           static_cast<hipStream_t>(stream), *args_host);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "k_mlp_bwd: %s", hipGetErrorString(e));
        ppo_detail::set_error(g_err);
        return -2;
    }
    return 0;
}

template <int DT, int LA>
static int launch_fwd(const ppo_mlp_fwd_t* a, void* stream) {
    static bool attr = false;
    if (const int rc = reserve_lds(k_mlp_fwd<DT, LA>, kFLds, attr, "ppo_mlp_forward")) return rc;
    const int blocks = (a->rows + kFRows - 1) / kFRows;
    hipLaunchKernelGGL((k_mlp_fwd<DT, LA>), dim3(blocks), dim3(kFThreads), kFLds, static_cast<hipStream_t>(stream), *a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "k_mlp_fwd: %s", hipGetErrorString(e));
        ppo_detail::set_error(g_err);
        return -2;
    }
    return 0;
}

extern "C" int ppo_mlp_forward(const ppo_mlp_fwd_t* args_host, void* stream) {
    const ppo_mlp_fwd_t* a = args_host;
    bool ok = a && (a->x || a->obs) && a->nh > 0 && a->nh <= 32 && a->rows > 0 &&
              !(a->obs && (!a->mb_idx || !a->mean || !a->var || a->obs_dim <= 0 || a->obs_dim > kK0)) &&
              a->x_stride >= kK0 && a->h_stride >= kHid && !(a->x_stride % 8) && !(a->h_stride % 8) &&
              (a->dtype == PPO_DT_BF16 || a->dtype == PPO_DT_F16) &&
              // the activations are stored all five or not at all (the rollout form)
              !(a->h[0] && !(a->h[1] && a->h[2] && a->h[3] && a->h[4]));
    const int LA = ok ? a->loss.A : 0;
    if (ok && LA)  // the fused losses: training form, every dataset pointer, the heads' width A + 1
        ok = (LA == 12 || LA == 21) && a->nh == LA + 1 && a->h[0] && a->head && a->mb_idx && a->loss.logstd &&
             a->loss.actions && a->loss.ds_mu && a->loss.ds_sigma && a->loss.old_neglogp && a->loss.advantages &&
             a->loss.old_values && a->loss.returns && a->loss.dhead_lp && a->loss.partials;
    if (!ok) {
        snprintf(g_err, sizeof(g_err), "ppo_mlp_forward: bad arguments");
        ppo_detail::set_error(g_err);
        return -1;
    }
    const bool f16 = a->dtype == PPO_DT_F16;
    if (LA == 21) return f16 ? launch_fwd<PPO_DT_F16, 21>(a, stream) : launch_fwd<PPO_DT_BF16, 21>(a, stream);
    if (LA == 12) return f16 ? launch_fwd<PPO_DT_F16, 12>(a, stream) : launch_fwd<PPO_DT_BF16, 12>(a, stream);
    return f16 ? launch_fwd<PPO_DT_F16, 0>(a, stream) : launch_fwd<PPO_DT_BF16, 0>(a, stream);
}

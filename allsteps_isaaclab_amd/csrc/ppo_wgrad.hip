// ppo_wgrad.hip -- split-K weight and bias gradients of the five trunk layers in one MFMA launch
// (include/ppo.h ppo_weight_grads).
//
// For layer l, split s:  part[s][o][c] = sum_{b in rows of s} dz[b][o] * hin[b][c]   (c < kin)
//                        part[s][o][kin] = sum_{b in rows of s} dz[b][o]             (bias column)
// which is the (S, 256, stride) fp32 block the five torch.bmm calls produced before, so the single
// deterministic reduce launch (ppo_reduce_rows) that sums the S partials stays as it was.
//
// Both operands are batch-major ([row][feature], as the forward / backward kernels write them) while
// the MFMA wants 8 consecutive k (= batch rows) per lane: a workgroup stages 64 rows of dz and of the
// layer input into LDS in that same row-major form and reads the operands with ds_read_b64_tr_b16,
// which hands every lane one feature column of a 4-row block.  Rows are padded to a pitch whose
// 4-row blocks fall on disjoint banks, so the transposed reads are conflict-free.  One workgroup
// (8 waves) owns the whole 256 x kin output of its row range, so every input byte is read once;
// the register prefetch of the next 64 rows overlaps the MFMAs of the current ones (LDS double
// buffer, one barrier per stage).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "ppo.h"

namespace ppo_detail {
void set_error(const char* msg);
}

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kOut = 256;                // output features of every trunk layer
constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kKT = 64;                  // batch rows per stage
constexpr int kPitchDz = kOut * 2 + 64;  // bytes: 576 = 144 dwords, +16 banks per row (mod 64)
constexpr int kPitchH256 = 256 * 2 + 64;
constexpr int kPitchH64 = 64 * 2 + 64;   // 192 B = 48 dwords: rows on banks 0, 48, 32, 16 (+16 each)
constexpr int kStageDz = kKT * kPitchDz;
constexpr int kStageH = kKT * kPitchH256;
constexpr int kStage = kStageDz + kStageH;
constexpr int kLdsBytes = 2 * kStage;    // 147456 B (one workgroup per CU)

char g_err[256];

// the 16-bit element type (PPO_DT_BF16 / PPO_DT_F16): fragment vector, MFMA, the all-ones operand
template <int DT>
struct Lp;
template <>
struct Lp<PPO_DT_BF16> {
    typedef bf16x8 v8;
    static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ v8 one() {
        v8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (__bf16)1.0f;
        return o;
    }
};
template <>
struct Lp<PPO_DT_F16> {
    typedef f16x8 v8;
    static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ v8 one() {
        v8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (_Float16)1.0f;
        return o;
    }
};

template <int DT>
union Frag {
    typename Lp<DT>::v8 v;
    s16x4 h[2];
};

// 32x32x16 operand from a row-major [k][col] LDS image: lane l gets column col0 + (l & 31) at rows
// kb + 8 (l >> 5) + 0..7 (two 4-row transposed reads; the same k order for both operands)
template <int DT>
__device__ __forceinline__ typename Lp<DT>::v8 tr_frag(const char* img, int pitch, int col0, int kb, int lane) {
    const int g = (lane >> 4) & 3, i = lane & 15, q = i >> 2, p = i & 3;
    const int row = kb + 8 * (g >> 1) + q;
    const int col = col0 + 16 * (g & 1) + 4 * p;
    const char* a = img + row * pitch + col * 2;
    Frag<DT> f;
    f.h[0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
    f.h[1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * pitch));
    return f.v;
}

// stage loads: rows [r0, r0 + kKT) of a [rows][stride] 16-bit matrix, columns [0, cols); rows past
// `rend` are zero (the pad rows then add nothing to the MFMA sums)
template <int COLS>
struct Stager {
    static constexpr int kChunksPerRow = COLS * 2 / 16;
    static constexpr int kPer = kKT * kChunksPerRow / kThreads;
    static_assert(kPer >= 1 && kKT * kChunksPerRow % kThreads == 0, "stage split");
    uint4 v[kPer];
    __device__ __forceinline__ void load(const uint16_t* __restrict__ src, int stride, int r0, int rend) {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int c = u * kThreads + threadIdx.x;
            const int r = r0 + c / kChunksPerRow;
            v[u] = r < rend ? *reinterpret_cast<const uint4*>(src + int64_t(r) * stride + (c % kChunksPerRow) * 8)
                            : make_uint4(0, 0, 0, 0);
        }
    }
    __device__ __forceinline__ void store(char* img, int pitch) const {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int c = u * kThreads + threadIdx.x;
            *reinterpret_cast<uint4*>(img + (c / kChunksPerRow) * pitch + (c % kChunksPerRow) * 16) = v[u];
        }
    }
};

// KIN input features: 256 (trunk layers, 8 column tiles: wave = 2 o-blocks of 4 tiles x 4 c-blocks
// of 2 tiles) or 64 (layer 0: 2 column tiles, wave = one o-tile x both c-tiles).  The bias sums of
// o-tile obase + cblock ride along as one MFMA against an all-ones B operand.
template <int KIN, int DT>
__device__ __forceinline__ void wgrad_layer(const ppo_wgrad_t& a, int l, char* lds) {
    typedef typename Lp<DT>::v8 V8;
    constexpr int NCT = KIN / 32;
    constexpr int CBLK = NCT / 2;            // c-blocks of 2 tiles
    constexpr int OTW = CBLK;                // o-tiles per wave (8 waves cover 8 o-tiles x NCT)
    static_assert(OTW * (kWaves / CBLK) == kOut / 32, "wave tiling");
    constexpr int PH = KIN == 256 ? kPitchH256 : kPitchH64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int cb = wave % CBLK, obase = (wave / CBLK) * OTW;
    const int S = a.splits, s = blockIdx.x;
    const int64_t rows = a.rows;
    const int r_begin = int(rows * s / S), r_end = int(rows * (s + 1) / S);
    const uint16_t* __restrict__ dz = a.dz[l];
    const uint16_t* __restrict__ hin = a.hin[l];
    const int hs = a.hin_stride[l];

    f32x16 acc[OTW][2], accb = {};
#pragma unroll
    for (int t = 0; t < OTW; ++t) acc[t][0] = acc[t][1] = f32x16{};
    const V8 ones = Lp<DT>::one();

    Stager<kOut> sd;
    Stager<KIN> sh;
    sd.load(dz, kOut, r_begin, r_end);
    sh.load(hin, hs, r_begin, r_end);
    const int nst = (r_end - r_begin + kKT - 1) / kKT;
    for (int it = 0; it < nst; ++it) {
        char* img = lds + (it & 1) * kStage;
        sd.store(img, kPitchDz);
        sh.store(img + kStageDz, PH);
        if (it + 1 < nst) {
            const int r0 = r_begin + (it + 1) * kKT;
            sd.load(dz, kOut, r0, r_end);
            sh.load(hin, hs, r0, r_end);
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < kKT / 16; ++ks) {
            V8 af[OTW], bfr[2];
#pragma unroll
            for (int t = 0; t < OTW; ++t) af[t] = tr_frag<DT>(img, kPitchDz, (obase + t) * 32, ks * 16, lane);
#pragma unroll
            for (int u = 0; u < 2; ++u) bfr[u] = tr_frag<DT>(img + kStageDz, PH, (2 * cb + u) * 32, ks * 16, lane);
#pragma unroll
            for (int t = 0; t < OTW; ++t)
#pragma unroll
                for (int u = 0; u < 2; ++u) acc[t][u] = Lp<DT>::mma(af[t], bfr[u], acc[t][u]);
            V8 ab = af[0];  // af[cb] without a dynamically indexed register array
#pragma unroll
            for (int t = 1; t < OTW; ++t) ab = cb == t ? af[t] : ab;
            accb = Lp<DT>::mma(ab, ones, accb);
        }
    }
    // D[o][c]: c = lane & 31 on the lane, o = 8 (r >> 2) + 4 (lane >> 5) + (r & 3) in register r
    float* __restrict__ part = a.part[l] + int64_t(s) * kOut * hs;
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int t = 0; t < OTW; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = (obase + t) * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                part[int64_t(o) * hs + (2 * cb + u) * 32 + j] = acc[t][u][r];
            }
    if (j == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = (obase + cb) * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
            part[int64_t(o) * hs + KIN] = accb[r];
        }
    }
}

template <int DT>
__global__ void __launch_bounds__(kThreads, 1) k_wgrad(ppo_wgrad_t a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int l = blockIdx.y;
    if (a.kin[l] == 64)
        wgrad_layer<64, DT>(a, l, lds);
    else
        wgrad_layer<256, DT>(a, l, lds);
}

}  // namespace

extern "C" int ppo_weight_grads(const ppo_wgrad_t* args_host, void* stream) {
    const ppo_wgrad_t* a = args_host;
    bool ok = a && a->rows > 0 && a->splits > 0 && a->splits <= a->rows && a->layers > 0 && a->layers <= 5 &&
              (a->dtype == PPO_DT_BF16 || a->dtype == PPO_DT_F16);
    for (int l = 0; ok && l < a->layers; ++l)
        ok = a->dz[l] && a->hin[l] && a->part[l] && (a->kin[l] == 64 || a->kin[l] == 256) &&
             a->hin_stride[l] >= a->kin[l] + 1 && a->hin_stride[l] % 8 == 0 &&
             (reinterpret_cast<uintptr_t>(a->dz[l]) | reinterpret_cast<uintptr_t>(a->hin[l])) % 16 == 0;
    if (!ok) {
        snprintf(g_err, sizeof(g_err), "ppo_weight_grads: bad arguments");
        ppo_detail::set_error(g_err);
        return -1;
    }
    const bool f16 = a->dtype == PPO_DT_F16;
    static bool attr[2] = {false, false};
    if (!attr[f16]) {
        const void* k = f16 ? reinterpret_cast<const void*>(k_wgrad<PPO_DT_F16>)
                            : reinterpret_cast<const void*>(k_wgrad<PPO_DT_BF16>);
        if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes) != hipSuccess) {
            snprintf(g_err, sizeof(g_err), "ppo_weight_grads: cannot reserve %d B of LDS", kLdsBytes);
            ppo_detail::set_error(g_err);
            return -2;
        }
        attr[f16] = true;
    }
    if (f16)
        hipLaunchKernelGGL(k_wgrad<PPO_DT_F16>, dim3(a->splits, a->layers), dim3(kThreads), kLdsBytes,
                           static_cast<hipStream_t>(stream), *a);
    else
        hipLaunchKernelGGL(k_wgrad<PPO_DT_BF16>, dim3(a->splits, a->layers), dim3(kThreads), kLdsBytes,
                           static_cast<hipStream_t>(stream), *a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "k_wgrad: %s", hipGetErrorString(e));
        ppo_detail::set_error(g_err);
        return -2;
    }
    return 0;
}

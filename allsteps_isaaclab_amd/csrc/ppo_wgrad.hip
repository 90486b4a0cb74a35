// ppo_wgrad.hip -- split-K weight and bias gradients of the five trunk layers and the head weights in
// one MFMA launch (include/ppo.h ppo_weight_grads).
//
// For job l, split s:  part[s][o][c]   = sum_{b in rows of s} dz[b][o] * hin[b][c]   (c < kin)
//                      part[s][o][kin] = sum_{b in rows of s} dz[b][o]             (bias column, trunk)
// the (S, nout, stride) fp32 blocks that ONE deterministic reduce launch (ppo_reduce_rows) sums.
//
// Both operands are batch-major ([row][feature], as the forward / backward kernels write them) while
// the MFMA wants 8 consecutive k (= batch rows) per lane: a workgroup stages 64 rows of dz and of the
// layer input into LDS in that same row-major form and reads the operands with ds_read_b64_tr_b16,
// which hands every lane one feature column of a 4-row block.  Rows are padded to a pitch whose
// 4-row blocks fall on disjoint banks, so the transposed reads are conflict-free.  The register
// prefetch of the next 64 rows overlaps the MFMAs of the current ones (LDS double buffer, one barrier
// per stage).
//
// Work split (round 5).  The kernel streams ~170 MB per 32768-row minibatch (dz of five layers, their
// inputs, the head gradient and layer 5), so it is bound by HBM / Infinity-Cache bandwidth, which a
// chip-wide stream only reaches with every CU pulling its share (~24-33 GB/s per CU): the workgroups
// must cover all 256 CUs.  Splitting K (rows) finer costs partials (each split writes a full 256 x 264
// fp32 block, which the reduce reads back); so a trunk split is instead TWO workgroups, output
// features 0..127 and 128..255, each reading its half of dz and the whole layer input -- placed 8 block
// indices apart so that both land on the same XCD at the same time (blocks are dealt to the XCDs
// round-robin) and the input they both stream is fetched from memory once into that XCD's L2.  The
// head gradient (dhead, 32 columns, against layer 5) is one more job of single workgroups.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "ppo.h"
#include "ppo_loss.h"

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
constexpr int kHeadOut = 32;             // the head job's output rows (dhead columns, nh <= 32)
constexpr int kOG = 128;                 // output features of one trunk workgroup
constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kKT = 64;                  // batch rows per stage
// row pitches in bytes: +16 banks per row (mod 64), so the four rows of a transposed read are disjoint
constexpr int kPitchD128 = kOG * 2 + 64;       // 320 B = 80 dwords
constexpr int kPitchD32 = kHeadOut * 2;        // 64 B = 16 dwords
constexpr int kPitchH256 = 256 * 2 + 64;       // 576 B = 144 dwords
constexpr int kPitchH64 = 64 * 2 + 64;         // 192 B = 48 dwords: rows on banks 0, 48, 32, 16 (+16 each)
constexpr int kStageD = kKT * kPitchD128;
constexpr int kStageH = kKT * kPitchH256;
constexpr int kStage = kStageD + kStageH;
constexpr int kLdsBytes = 2 * kStage;    // 114688 B (one workgroup per CU)

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

// stage loads: rows [r0, r0 + kKT) of a [rows][stride] 16-bit matrix, columns [c0, c0 + COLS); rows past
// `rend` are zero (the pad rows then add nothing to the MFMA sums)
template <int COLS>
struct Stager {
    static constexpr int kChunksPerRow = COLS * 2 / 16;
    static constexpr int kTotal = kKT * kChunksPerRow;
    static constexpr int kPer = (kTotal + kThreads - 1) / kThreads;
    uint4 v[kPer];
    __device__ __forceinline__ void load(const uint16_t* __restrict__ src, int stride, int c0, int r0, int rend) {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int c = u * kThreads + threadIdx.x;
            const int r = r0 + c / kChunksPerRow;
            v[u] = (kTotal % kThreads == 0 || c < kTotal) && r < rend
                       ? *reinterpret_cast<const uint4*>(src + int64_t(r) * stride + c0 + (c % kChunksPerRow) * 8)
                       : make_uint4(0, 0, 0, 0);
        }
    }
    __device__ __forceinline__ void store(char* img, int pitch) const {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int c = u * kThreads + threadIdx.x;
            if (kTotal % kThreads == 0 || c < kTotal)
                *reinterpret_cast<uint4*>(img + (c / kChunksPerRow) * pitch + (c % kChunksPerRow) * 16) = v[u];
        }
    }
};

// One workgroup's output block: OG output features (o0 .. o0 + OG - 1 of the job's nout) x KIN input
// features (+ the bias column when BIAS) over rows [r_begin, r_end).  The block is OT x CT tiles of 32 x 32;
// wave w takes WO consecutive o-tiles x WC consecutive c-tiles (oi = w % (OT / WO), ci = w / (OT / WO)), and
// when BIAS the waves with ci < WO also form the bias sums of o-tile oi * WO + ci as one MFMA against an
// all-ones B operand.  Shapes: trunk 128 x 256 (2 x 2 tiles per wave), layer 0 128 x 64 (1 x 1), the
// head 32 x 256 (1 x 1, no bias).
template <int OG, int KIN, int WO, int WC, bool BIAS, int DT>
__device__ __forceinline__ void wgrad_block(const uint16_t* __restrict__ dz, int dz_stride, int o0,
                                            const uint16_t* __restrict__ hin, int hs, float* __restrict__ part,
                                            int r_begin, int r_end, char* lds) {
    typedef typename Lp<DT>::v8 V8;
    constexpr int OT = OG / 32, CT = KIN / 32;
    constexpr int NOI = OT / WO;
    static_assert(NOI * (CT / WC) == kWaves, "wave tiling");
    static_assert(!BIAS || CT / WC >= WO, "bias tiles");
    constexpr int PD = OG == 128 ? kPitchD128 : kPitchD32;
    constexpr int PH = KIN == 256 ? kPitchH256 : kPitchH64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int oi = wave % NOI, ci = wave / NOI;
    const bool bias_wave = BIAS && ci < WO;

    f32x16 acc[WO][WC], accb = {};
#pragma unroll
    for (int t = 0; t < WO; ++t)
#pragma unroll
        for (int u = 0; u < WC; ++u) acc[t][u] = f32x16{};
    const V8 ones = Lp<DT>::one();

    Stager<OG> sd;
    Stager<KIN> sh;
    sd.load(dz, dz_stride, o0, r_begin, r_end);
    sh.load(hin, hs, 0, r_begin, r_end);
    const int nst = (r_end - r_begin + kKT - 1) / kKT;
    for (int it = 0; it < nst; ++it) {
        char* img = lds + (it & 1) * kStage;
        sd.store(img, PD);
        sh.store(img + kStageD, PH);
        if (it + 1 < nst) {
            const int r0 = r_begin + (it + 1) * kKT;
            sd.load(dz, dz_stride, o0, r0, r_end);
            sh.load(hin, hs, 0, r0, r_end);
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < kKT / 16; ++ks) {
            V8 af[WO], bfr[WC];
#pragma unroll
            for (int t = 0; t < WO; ++t) af[t] = tr_frag<DT>(img, PD, (oi * WO + t) * 32, ks * 16, lane);
#pragma unroll
            for (int u = 0; u < WC; ++u) bfr[u] = tr_frag<DT>(img + kStageD, PH, (ci * WC + u) * 32, ks * 16, lane);
#pragma unroll
            for (int t = 0; t < WO; ++t)
#pragma unroll
                for (int u = 0; u < WC; ++u) acc[t][u] = Lp<DT>::mma(af[t], bfr[u], acc[t][u]);
            if (bias_wave) {  // uniform per wave
                V8 ab = af[0];  // af[ci] without a dynamically indexed register array
#pragma unroll
                for (int t = 1; t < WO; ++t) ab = ci == t ? af[t] : ab;
                accb = Lp<DT>::mma(ab, ones, accb);
            }
        }
    }
    // D[o][c]: c = lane & 31 on the lane, o = 8 (r >> 2) + 4 (lane >> 5) + (r & 3) in register r
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int t = 0; t < WO; ++t)
#pragma unroll
        for (int u = 0; u < WC; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = o0 + (oi * WO + t) * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                part[int64_t(o) * hs + (ci * WC + u) * 32 + j] = acc[t][u][r];
            }
    if (bias_wave && j == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = o0 + (oi * WO + ci) * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
            part[int64_t(o) * hs + KIN] = accb[r];
        }
    }
}

// ppo_loss_finalize's work (include/ppo.h ppo_wgrad_t.loss): value k of the loss kernel's block partials
// summed over the blocks in block order, the partials staged through LDS by all threads in passes
__device__ void loss_finalize_side(const ppo_loss_side_t& f, float* sm) {
    const int NV = 2 * f.A + 1 + PPO_LOSS_NSTAT;
    const int chunk = (kLdsBytes / 4) / NV;
    float acc = 0.f;
    for (int b0 = 0; b0 < f.nblk; b0 += chunk) {
        const int nb = min(chunk, f.nblk - b0);
        __syncthreads();
        for (int e = threadIdx.x; e < nb * NV; e += kThreads) sm[e] = f.partials[int64_t(b0) * NV + e];
        __syncthreads();
        if (int(threadIdx.x) < NV) {
            float c4[4] = {0.f, 0.f, 0.f, 0.f};
            int bb = 0;
            for (; bb + 4 <= nb; bb += 4)
#pragma unroll
                for (int u = 0; u < 4; ++u) c4[u] += sm[(bb + u) * NV + threadIdx.x];
            for (; bb < nb; ++bb) c4[0] += sm[bb * NV + threadIdx.x];
            acc += (c4[0] + c4[1]) + (c4[2] + c4[3]);
        }
    }
    if (int(threadIdx.x) < NV)
        ppo_detail::loss_finalize_value(threadIdx.x, acc, f.A, f.mb_rows, f.entropy_coef, f.grad_scale, f.grad_head_bias,
                                        f.grad_logstd, f.stats, f.stat_idx, f.kl_out);
}

// block index -> job.  Trunk pairs (layer l < 5, split s) in layer-major order, two workgroups each
// (output halves); the pairs are dealt in groups of 8 so that the halves of a pair sit 8 block indices
// apart (same XCD, dispatched together); the last group holds the remainder.  Then the head splits.
template <int DT>
__global__ void __launch_bounds__(kThreads, 1) k_wgrad(ppo_wgrad_t a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int ntrunk = a.layers < 5 ? a.layers : 5;
    int pairs = 0;
    for (int l = 0; l < ntrunk; ++l) pairs += a.splits[l];
    const int b = blockIdx.x;
    if (b < 2 * pairs) {
        const int q = b / 16, full = (pairs - 8 * q) >= 8 ? 8 : pairs - 8 * q;
        const int r = b - 16 * q;
        const int half = r / full, pair = 8 * q + r % full;
        int l = 0, s = pair;
        while (s >= a.splits[l]) s -= a.splits[l++];
        const int S = a.splits[l];
        const int r_begin = int(int64_t(a.rows) * s / S), r_end = int(int64_t(a.rows) * (s + 1) / S);
        float* part = a.part[l] + int64_t(s) * kOut * a.hin_stride[l];
        if (a.kin[l] == 64)
            wgrad_block<kOG, 64, 1, 1, true, DT>(a.dz[l], kOut, half * kOG, a.hin[l], a.hin_stride[l], part,
                                                 r_begin, r_end, lds);
        else
            wgrad_block<kOG, 256, 2, 2, true, DT>(a.dz[l], kOut, half * kOG, a.hin[l], a.hin_stride[l], part,
                                                  r_begin, r_end, lds);
    } else {
        const int s = b - 2 * pairs, S = a.splits[5];
        const int r_begin = int(int64_t(a.rows) * s / S), r_end = int(int64_t(a.rows) * (s + 1) / S);
        float* part = a.part[5] + int64_t(s) * kHeadOut * a.hin_stride[5];
        wgrad_block<kHeadOut, 256, 1, 1, false, DT>(a.dz[5], kHeadOut, 0, a.hin[5], a.hin_stride[5], part,
                                                     r_begin, r_end, lds);
        // the side job on the last head workgroup (a head split streams ~0.6 of a trunk split's bytes, so
        // this one finishes early even with the finalize added)
        if (s == S - 1 && a.loss.partials) {
            __syncthreads();  // the block's LDS stages are done with
            loss_finalize_side(a.loss, reinterpret_cast<float*>(lds));
        }
    }
}

}  // namespace

extern "C" int ppo_weight_grads(const ppo_wgrad_t* args_host, void* stream) {
    const ppo_wgrad_t* a = args_host;
    bool ok = a && a->rows > 0 && a->layers > 0 && a->layers <= 6 && (a->dtype == PPO_DT_BF16 || a->dtype == PPO_DT_F16);
    int blocks = 0;
    for (int l = 0; ok && l < a->layers; ++l) {
        const bool head = l == 5;
        const int kin = head ? 256 : a->kin[l];
        ok = a->dz[l] && a->hin[l] && a->part[l] && a->splits[l] > 0 && a->splits[l] <= a->rows &&
             (head ? a->kin[l] == 256 : (kin == 64 || kin == 256) && (l == 0 || kin == 256)) &&
             a->hin_stride[l] >= kin + (head ? 0 : 1) && a->hin_stride[l] % 8 == 0 &&
             (reinterpret_cast<uintptr_t>(a->dz[l]) | reinterpret_cast<uintptr_t>(a->hin[l])) % 16 == 0;
        blocks += head ? a->splits[l] : 2 * a->splits[l];
    }
    if (ok && a->loss.partials)  // the side job runs on the head job's last workgroup
        ok = a->layers == 6 && a->loss.nblk > 0 && a->loss.A > 0 && a->loss.A <= PPO_MAX_ACT && a->loss.mb_rows > 0 &&
             a->loss.grad_head_bias && a->loss.grad_logstd && a->loss.stats && a->loss.stat_idx && a->loss.kl_out;
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
        hipLaunchKernelGGL(k_wgrad<PPO_DT_F16>, dim3(blocks), dim3(kThreads), kLdsBytes,
                           static_cast<hipStream_t>(stream), *a);
    else
        hipLaunchKernelGGL(k_wgrad<PPO_DT_BF16>, dim3(blocks), dim3(kThreads), kLdsBytes,
                           static_cast<hipStream_t>(stream), *a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "k_wgrad: %s", hipGetErrorString(e));
        ppo_detail::set_error(g_err);
        return -2;
    }
    return 0;
}

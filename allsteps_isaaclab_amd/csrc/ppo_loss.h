// ppo_loss.h -- the PPO loss block (ppo_loss_grad's per-row losses and head gradients for 128 minibatch
// rows) and the per-value output rule of the loss finalize (ppo_loss_finalize), shared by the standalone
// kernels (ppo_kernels.hip), the trunk forward that runs the loss block in its epilogue (ppo_mlp.hip) and
// the weight-gradient launch that runs the finalize as a side job (ppo_wgrad.hip).  Value k of the loss-kernel block partials, summed over the blocks (s):
//   k <= A: head-bias gradient; A < k <= 2A: log-sigma gradient minus entropy_coef (times the loss scale);
//   k > 2A: statistic k - 2A - 1, as its mean over the minibatch (the KL also into kl_out).
#pragma once
#include <stdint.h>

#include "ppo.h"

namespace ppo_detail {

__device__ __forceinline__ void loss_finalize_value(int k, float s, int A, int mb_rows, float entropy_coef,
                                                    const float* __restrict__ grad_scale, float* __restrict__ g_hb,
                                                    float* __restrict__ g_ls, float* __restrict__ stats,
                                                    const int32_t* __restrict__ stat_idx, float* __restrict__ kl_out) {
    if (k <= A) {
        g_hb[k] = s;
    } else if (k <= 2 * A) {
        // - entropy_coef * mean(entropy): d/d logstd_j = -entropy_coef (times the loss scale)
        g_ls[k - A - 1] = s - entropy_coef * (grad_scale ? *grad_scale : 1.f);
    } else {
        const int st = k - 2 * A - 1;
        const float mean = s / float(mb_rows);
        stats[int64_t(*stat_idx) * PPO_LOSS_NSTAT + st] = mean;
        if (st == 4) *kl_out = mean;
    }
}


// one block's worth of ppo_loss_grad (include/ppo.h): rows [blk * kLossRows, +kLossRows) of the minibatch
struct LossRowArgs {
    const float* head;     // rows x head_stride fp32 ([mu | value]); global, or an LDS table of the block's rows
    int head_stride;
    bool head_block_rows;  // true: head row = minibatch row r; false: row r - blk * kLossRows (a block table)
    const float* logstd;
    int mb_rows;
    const int32_t* mb_idx;
    const float* actions;
    float* ds_mu;
    float* ds_sigma;
    const float* old_nlp;
    const float* adv;
    const float* old_v;
    const float* ret;
    ppo_loss_cfg_t cfg;
    const float* grad_scale;
    float* dhead;          // rows x (A + 1) fp32, or NULL
    uint16_t* dhead_lp;    // rows x 32 lp, or NULL
    int lp_dtype;
    float* partials;       // nblk x (2A + 1 + PPO_LOSS_NSTAT)
};

__device__ __forceinline__ uint16_t loss_bf16(float f) {  // round to nearest even
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7f800000u) == 0x7f800000u) return uint16_t((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
    u += 0x7fffu + ((u >> 16) & 1u);
    return uint16_t(u >> 16);
}
__device__ __forceinline__ uint16_t loss_f16(float f) { return __builtin_bit_cast(uint16_t, static_cast<_Float16>(f)); }

// gradient of max(u1, u2) (torch.maximum: ties split the gradient in half)
__device__ __forceinline__ float loss_max_grad(float u1, float u2, float g1, float g2) {
    return u1 > u2 ? g1 : (u2 > u1 ? g2 : 0.5f * (g1 + g2));
}

// Eight lanes per row (round 5; the round-4 form spread a row over a 32-lane group -- 10 of 32 lanes idle,
// the row sums as chains of LDS-routed permutes; a one-row-per-lane form ran out of parallelism, 512
// waves for a 32768-row minibatch).  Lane g of a row owns head columns NJ*g .. NJ*g + NJ - 1 (the
// actions, then the value column A; NJ = ceil((A + 1) / 8)), so a row's loads are one contiguous run
// across its eight lanes; the row sums (sum d^2, the KL, the bound loss) are three DPP steps inside the
// eight lanes (bit-identical on every lane); the per-row scalar work (ratio, clipping) runs on all eight.
// The per-row contributions to the column sums land in an LDS table that NV threads sum down in row order
// (deterministic), one partial row per block.
constexpr int kLossLanes = 8;
constexpr int kLossRows = 128;                         // rows per block
constexpr int kLossThreads = kLossRows * kLossLanes;   // 1024 (the standalone kernel: one pass)
constexpr float kLog2PiL = 1.8378770664093453f;
__host__ __device__ constexpr int loss_rp(int A) { return (2 * A + 1 + PPO_LOSS_NSTAT) | 1; }  // LDS row pitch
constexpr int kLossColGroups = 8;  // the column sums: 8 row groups of 16, then the 8 group sums in order
// LDS floats loss_block needs: the per-row table + the group sums
__host__ __device__ constexpr int loss_lds_floats(int A) {
    return kLossRows * loss_rp(A) + kLossColGroups * (2 * A + 1 + PPO_LOSS_NSTAT);
}

// sum over the eight lanes of a row (xor 1, xor 2 by quad permutes, then the mirrored half-row): the same
// two operands meet on every lane, so all eight hold the bit-identical sum
__device__ __forceinline__ float sum8(float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
    x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x141, 0xF, 0xF, false));
    return x;
}


template <int A>
constexpr int loss_nj() { return (A + 1 + kLossLanes - 1) / kLossLanes; }
template <int NT>
constexpr int loss_passes() { return kLossRows / (NT / kLossLanes); }

// a lane's minibatch inputs for one pass (its row's dataset values; the head values come later)
template <int A>
struct LossIn {
    float av[loss_nj<A>()], m1[loss_nj<A>()], s1[loss_nj<A>()];
    float onlp, adv, vp, Rt;
};

// the dataset loads of every pass, issued together (no dependence on the head values: the trunk forward
// issues them before its heads, so their round trip overlaps the heads' MFMAs and barriers)
template <int A, int NT>
__device__ __forceinline__ void loss_prefetch(const LossRowArgs& p, int blk, LossIn<A> (&in)[loss_passes<NT>()]) {
    constexpr int NJ = loss_nj<A>();
    const int tid = threadIdx.x, g = tid % kLossLanes;
    const int64_t base = int64_t(*p.mb_idx) * p.mb_rows;
#pragma unroll
    for (int pass = 0; pass < loss_passes<NT>(); ++pass) {
        const int r = blk * kLossRows + pass * (NT / kLossLanes) + tid / kLossLanes;
        const bool ok = r < p.mb_rows;
        const int64_t row = base + (ok ? r : 0);
#pragma unroll
        for (int k = 0; k < NJ; ++k) {
            const bool act = ok && NJ * g + k < A;
            in[pass].av[k] = act ? p.actions[row * A + NJ * g + k] : 0.f;
            in[pass].m1[k] = act ? p.ds_mu[row * A + NJ * g + k] : 0.f;
            in[pass].s1[k] = act ? p.ds_sigma[row * A + NJ * g + k] : 1.f;
        }
        in[pass].onlp = ok ? p.old_nlp[row] : 0.f;
        in[pass].adv = ok ? p.adv[row] : 0.f;
        in[pass].vp = ok ? p.old_v[row] : 0.f;
        in[pass].Rt = ok ? p.ret[row] : 0.f;
    }
}

// NT threads (a multiple of 8) cover the block's 128 rows in 128 / (NT / 8) passes; s_red: kLossRows x
// loss_rp(A) floats of LDS; `in`: loss_prefetch's loads (this thread's own rows: ds_mu / ds_sigma are read
// there before this thread rewrites them here)
template <int A, int NT>
__device__ void loss_block(const LossRowArgs& p, int blk, float* __restrict__ s_red,
                           const LossIn<A> (&in)[loss_passes<NT>()]) {
    static_assert(A + 1 <= 32, "heads of at most 32 outputs");
    static_assert(NT % kLossLanes == 0 && kLossRows % (NT / kLossLanes) == 0, "whole passes of rows");
    constexpr int NV = 2 * A + 1 + PPO_LOSS_NSTAT, RP = loss_rp(A);
    constexpr int NJ = loss_nj<A>();
    const ppo_loss_cfg_t cfg = p.cfg;
    const int mb_rows = p.mb_rows;
    const int tid = threadIdx.x, g = tid % kLossLanes;
    // the loss scale (a power of two, GradScaler) enters every gradient through the 1/B factor: exact
    const float inv_b = (p.grad_scale ? *p.grad_scale : 1.f) * (1.f / float(mb_rows));
    float sum_ls = 0.f;
#pragma unroll
    for (int j = 0; j < A; ++j) sum_ls += p.logstd[j];
    const float entropy = float(A) * (0.5f + 0.5f * kLog2PiL) + sum_ls;
    const int64_t base = int64_t(*p.mb_idx) * mb_rows;
    // a lane's columns are the same in every pass: sigma_j = exp(logstd_j) and its reciprocal once per
    // lane; the divisions by sigma below are products with the correctly rounded 1 / sigma (round 5:
    // within an ulp of torch's quotients, ~80 fewer VALU instructions per pass)
    float sgc[NJ], rsg[NJ];
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
        const int j = NJ * g + k;
        sgc[k] = j < A ? expf(p.logstd[j]) : 1.f;
        rsg[k] = 1.f / sgc[k];
    }
#pragma unroll
    for (int pass = 0; pass < loss_passes<NT>(); ++pass) {
    const int rl = pass * (NT / kLossLanes) + tid / kLossLanes;
    const int r = blk * kLossRows + rl;  // minibatch row
    const bool ok = r < mb_rows;
    const int64_t row = base + (ok ? r : 0);
    const float* hrow = p.head + int64_t(p.head_block_rows ? r : rl) * p.head_stride;
    float hj[NJ], sg[NJ];
    const float* av = in[pass].av;
    const float* m1 = in[pass].m1;
    const float* s1 = in[pass].s1;
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
        const int j = NJ * g + k;
        hj[k] = ok && j <= A ? hrow[j] : 0.f;
        sg[k] = sgc[k];
    }
    const float onlp = in[pass].onlp, adv = in[pass].adv;
    const float vp = in[pass].vp, Rt = in[pass].Rt;
    // policy: d_j = (a_j - mu_j) / sigma_j; nlp = 0.5 sum d^2 + 0.5 log(2 pi) A + sum logstd;
    // policy_kl(p0 = current, p1 = dataset); the bound loss
    float d[NJ];
    float q = 0.f, kl = 0.f, bl = 0.f;
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
        d[k] = 0.f;
        if (NJ * g + k < A) {
            d[k] = (av[k] - hj[k]) * rsg[k];
            q += d[k] * d[k];
            const float dm = m1[k] - hj[k];
            kl += logf(s1[k] * rsg[k] + 1e-5f) + (sg[k] * sg[k] + dm * dm) / (2.f * (s1[k] * s1[k] + 1e-5f)) - 0.5f;
            if (cfg.bound_loss == 1) {
                const float lo = fminf(hj[k] + cfg.soft_bound, 0.f), hi = fmaxf(hj[k] - cfg.soft_bound, 0.f);
                bl += lo * lo + hi * hi;
            } else if (cfg.bound_loss == 2) {
                bl += hj[k] * hj[k];
            }
        }
    }
    q = sum8(q);
    kl = sum8(kl);
    bl = sum8(bl);
    const float nlp = 0.5f * q + 0.5f * kLog2PiL * float(A) + sum_ls;
    float a_loss, g_nlp;
    if (cfg.ppo) {
        const float ratio = expf(onlp - nlp);
        const float rc = fminf(fmaxf(ratio, 1.f - cfg.e_clip), 1.f + cfg.e_clip);
        const float u1 = -adv * ratio, u2 = -adv * rc;
        const bool inside = ratio >= 1.f - cfg.e_clip && ratio <= 1.f + cfg.e_clip;
        // d(-adv * ratio)/d nlp = adv * ratio (d ratio / d nlp = -ratio); torch.maximum ties split
        g_nlp = loss_max_grad(u1, u2, adv * ratio, inside ? adv * ratio : 0.f);
        a_loss = fmaxf(u1, u2);
    } else {
        a_loss = nlp * adv;
        g_nlp = adv;
    }
    g_nlp *= inv_b;
    float* red = s_red + rl * RP;
    float gh[NJ];  // d loss / d head for this lane's columns (0 past the value column)
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
        const int j = NJ * g + k;
        gh[k] = 0.f;
        if (j < A) {
            float dbj = 0.f;
            if (cfg.bound_loss == 1) {
                const float lo = fminf(hj[k] + cfg.soft_bound, 0.f), hi = fmaxf(hj[k] - cfg.soft_bound, 0.f);
                dbj = 2.f * (lo + hi);
            } else if (cfg.bound_loss == 2) {
                dbj = 2.f * hj[k];
            }
            // d nlp / d mu = -d / sigma ; d nlp / d logstd = 1 - d^2
            gh[k] = -g_nlp * d[k] * rsg[k] + cfg.bounds_coef * inv_b * dbj;
            red[j] = ok ? gh[k] : 0.f;
            red[A + 1 + j] = ok ? g_nlp * (1.f - d[k] * d[k]) : 0.f;
            if (ok) {
                p.ds_mu[row * A + j] = hj[k];  // dataset.update_mu_sigma
                p.ds_sigma[row * A + j] = sg[k];
            }
        } else if (j == A) {  // critic
            const float v = hj[k];
            float c_loss, g_v;
            if (cfg.clip_value) {
                const float dv = v - vp;
                const float vc = vp + fminf(fmaxf(dv, -cfg.e_clip), cfg.e_clip);
                const float l1 = (v - Rt) * (v - Rt), l2 = (vc - Rt) * (vc - Rt);
                const bool inside = dv >= -cfg.e_clip && dv <= cfg.e_clip;
                g_v = loss_max_grad(l1, l2, 2.f * (v - Rt), inside ? 2.f * (vc - Rt) : 0.f);
                c_loss = fmaxf(l1, l2);
            } else {
                c_loss = (Rt - v) * (Rt - v);
                g_v = 2.f * (v - Rt);
            }
            g_v *= 0.5f * cfg.critic_coef * inv_b;
            gh[k] = g_v;
            red[A] = ok ? g_v : 0.f;
            red[2 * A + 1 + 1] = ok ? c_loss : 0.f;
        }
    }
    if (g == 0) {
        red[2 * A + 1 + 0] = ok ? a_loss : 0.f;
        red[2 * A + 1 + 2] = ok ? bl : 0.f;
        red[2 * A + 1 + 3] = ok ? entropy : 0.f;
        red[2 * A + 1 + 4] = ok ? kl : 0.f;
    }
    if (ok) {
        if (p.dhead) {
#pragma unroll
            for (int k = 0; k < NJ; ++k)
                if (NJ * g + k <= A) p.dhead[int64_t(r) * (A + 1) + NJ * g + k] = gh[k];
        }
        // the 16-bit copy (autocast: the gradient reaching the heads' fp16 Linear is fp16), rows x 32, zero
        // past the value column
        if (p.dhead_lp) {
            uint16_t* dl = p.dhead_lp + int64_t(r) * 32;
#pragma unroll
            for (int k = 0; k < NJ; ++k)
                if (NJ * g + k < 32) dl[NJ * g + k] = p.lp_dtype == PPO_DT_F16 ? loss_f16(gh[k]) : loss_bf16(gh[k]);
            for (int c = NJ * kLossLanes + g; c < 32; c += kLossLanes) dl[c] = 0;
        }
    }
    }  // pass
    __syncthreads();
    // block partials: value k summed over the block's rows in a fixed order -- eight groups of 16 rows on
    // 8 x NV threads (two chains each), then the eight group sums in group order (one 48-thread pass over
    // all 128 rows left seven of the forward's eight waves idle); ppo_loss_finalize sums them over the
    // blocks.  (Round 5 measured the finalize folded into this kernel's last block -- sc1 hand-off, relaxed
    // agent counter -- at 16.9 us against 11.5 us for the two launches: each block's store drain and
    // counter round trip sit on the kernel's tail, scripts/loss_bench.py.)
    constexpr int kRG = kLossRows / kLossColGroups;
    static_assert(NT >= kLossColGroups * NV, "one thread per (group, value)");
    float* s_grp = s_red + kLossRows * RP;
    if (tid < kLossColGroups * NV) {
        const int c = tid % NV, gi = tid / NV;
        const float* col = s_red + gi * kRG * RP + c;
        float t0 = 0.f, t1 = 0.f;
#pragma unroll
        for (int rr = 0; rr < kRG; rr += 2) {
            t0 += col[rr * RP];
            t1 += col[(rr + 1) * RP];
        }
        s_grp[gi * NV + c] = t0 + t1;
    }
    __syncthreads();
    if (tid < NV) {
        float t = 0.f;
#pragma unroll
        for (int gi = 0; gi < kLossColGroups; ++gi) t += s_grp[gi * NV + tid];
        p.partials[int64_t(blk) * NV + tid] = t;
    }
}

template <int A, int NT>
__device__ __forceinline__ void loss_block(const LossRowArgs& p, int blk, float* __restrict__ s_red) {
    LossIn<A> in[loss_passes<NT>()];
    loss_prefetch<A, NT>(p, blk, in);
    loss_block<A, NT>(p, blk, s_red, in);
}


}  // namespace ppo_detail

// ppo_loss.h -- the per-value output rule of the PPO loss finalize (ppo_loss_finalize), shared by the
// finalize kernel (ppo_kernels.hip) and the same work run as a side job of the weight-gradient launch
// (ppo_wgrad.hip).  Value k of the loss-kernel block partials, summed over the blocks (s):
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

}  // namespace ppo_detail

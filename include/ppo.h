/*
 * ppo.h -- C ABI of the MI355X PPO-update kernels (libppo_hip.so) used by the rl_games-semantics
 * trainer (allsteps_isaaclab_amd/learning/fused.py).
 *
 * The reference trains with rl_games 1.6.1 (third-party, absent offline): every minibatch it runs
 * autograd over ModelA2CContinuousLogStd + the PPO losses (a2c_continuous.py calc_gradients), clips
 * the gradient norm and steps torch.optim.Adam, then adapts the learning rate from the KL
 * (a2c_common.py train_epoch, schedule_type 'legacy').  These kernels are the non-GEMM half of that
 * minibatch step, written for a HIP-graph replay with NO host round trip:
 *   ppo_obs_stats / ppo_obs_stats_update  RunningMeanStd train-mode update (running_mean_std.py)
 *   ppo_obs_normalize                     (x - mean) / sqrt(var + eps), clamp +-5 -> trunk input
 *   ppo_loss_grad / ppo_loss_finalize     actor (clipped ratio) + critic (clipped value) + bound +
 *                                         entropy losses, KL(policy_kl), and their analytic
 *                                         gradients w.r.t. the heads (mu, value) and log-sigma;
 *                                         writes mu / sigma back into the dataset (update_mu_sigma)
 *   ppo_elu_bwd                           ELU backward (output form) + per-block bias-grad partials
 *   ppo_sqnorm / ppo_adam                 clip_grad_norm_ + Adam over the flat parameter buffer, and
 *                                         the bf16 / fp16 mirror of the trunk weights for the next
 *                                         forward; with a loss scaler (rl_games mixed_precision:
 *                                         torch.cuda.amp.GradScaler) the unscale, the skip of a step
 *                                         with non-finite gradients and the scale update
 *   ppo_tail                              adaptive LR from the (rank-averaged) KL; minibatch counter
 *   ppo_adam_step                         ppo_adam + ppo_tail in ONE launch (round 5): Adam reads its
 *                                         lr / step / scale from the snapshot the norm launch took
 *                                         (ppo_opt_snap_t), so the first block may run the tail on the
 *                                         originals while the others still read
 *   ppo_mlp_forward / ppo_mlp_backward    the whole trunk forward / input-gradient chain (MFMA)
 *   ppo_weight_grads                      split-K weight + bias gradients of all trunk layers and the
 *                                         head weights (MFMA, one launch)
 *
 * Minibatch rows are selected on the device: row r of minibatch i is dataset row i*mb_rows + r with i
 * read from `mb_idx` (int32, device), so one captured graph serves every minibatch.
 * All pointers are DEVICE pointers; `stream` is a hipStream_t.  Every function returns 0 or a
 * negative error code (ppo_last_error()).
 */
#ifndef PPO_H
#define PPO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPO_ABI_VERSION 5
/* element types of the low-precision (trunk) buffers */
#define PPO_DT_F32 0
#define PPO_DT_BF16 1
#define PPO_DT_F16 2
#define PPO_MAX_ACT 32
#define PPO_MAX_SEG 16
#define PPO_LOSS_NSTAT 5 /* a_loss, c_loss, b_loss, entropy, kl */

typedef struct {
    float e_clip, critic_coef, entropy_coef, bounds_coef, soft_bound;
    int32_t ppo, clip_value, bound_loss; /* bound_loss: 0 none, 1 'bound', 2 'regularisation' */
} ppo_loss_cfg_t;

/* one contiguous run of the flat parameter buffer that has a low-precision mirror (trunk layers):
 * flat[off + r*cols + c] -> mirror[moff + r*mstride + c]  (mstride >= cols; the pad stays zero), or
 * with trans != 0 the transpose: mirror[moff + c*mstride + r] (mstride >= rows = len / cols) */
typedef struct {
    int64_t off, len, moff;
    int32_t cols, mstride, trans;
} ppo_seg_t;

int ppo_abi_version(void);
const char* ppo_last_error(void);
/* Provenance digest (-DPPO_BUILD_ID; see as_build_id in allsteps.h). */
const char* ppo_build_id(void);

/* column sum / sum of squares (fp64) of rows [i*mb_rows, (i+1)*mb_rows) of x (row stride `cols`),
 * one partial per block into partials[nblk][2][64]; nblk = ppo_obs_stats_blocks(mb_rows). */
int ppo_obs_stats_blocks(int32_t mb_rows);
int ppo_obs_stats(const float* x, const int32_t* mb_idx, int32_t mb_rows, int32_t cols, double* partials,
                  void* stream);
/* fold the partials into running_mean / running_var / count (fp64, rl_games formula, unbiased batch var) */
int ppo_obs_stats_update(const double* partials, int32_t nblk, int32_t cols, int32_t mb_rows, double* running_mean,
                         double* running_var, double* count, void* stream);
/* out[r*out_stride + c] = clamp((x[row][c] - mean[c]) / sqrt(var[c] + eps), -5, 5) for c < cols, 0 for
 * cols <= c < out_cols (columns out_cols .. out_stride-1 are left untouched, e.g. a constant ones column);
 * out_dtype: PPO_DT_F32, PPO_DT_BF16 or PPO_DT_F16 */
int ppo_obs_normalize(const float* x, const int32_t* mb_idx, int32_t mb_rows, int32_t cols, const double* running_mean,
                      const double* running_var, float eps, void* out, int32_t out_cols, int32_t out_stride,
                      int32_t out_dtype, void* stream);

/* Per-row PPO losses and head gradients.  head = [mu(0..A-1) | value(A)] (mb_rows x (A+1), fp32);
 * logstd (A); dataset rows (selected by mb_idx): actions / mu / sigma (A each), old_neglogp,
 * advantages, old_values, returns (1 each).  Writes dhead (mb_rows x (A+1)) = d loss / d head,
 * new mu / sigma into the dataset rows, and per-block partials[nblk][2A+1+PPO_LOSS_NSTAT]
 * (sum over rows of dhead columns, d loss / d logstd, the five statistics); nblk = ppo_loss_blocks().
 * grad_scale (device fp32, a power of two; NULL = 1): every gradient is of scale * loss (GradScaler).
 * dhead may be NULL; dhead_lp (NULL = skip) receives the same gradient rounded to lp_dtype (PPO_DT_BF16 /
 * PPO_DT_F16) as mb_rows x 32 (columns A+1..31 zero): the 16-bit gradient autocast hands to the heads'
 * Linear backward, read by ppo_mlp_backward and ppo_weight_grads. */
int ppo_loss_blocks(int32_t mb_rows);
int ppo_loss_grad(const float* head, const float* logstd, int32_t A, int32_t mb_rows, const int32_t* mb_idx,
                  const float* actions, float* ds_mu, float* ds_sigma, const float* old_neglogp,
                  const float* advantages, const float* old_values, const float* returns, ppo_loss_cfg_t cfg,
                  const float* grad_scale, float* dhead, float* partials, uint16_t* dhead_lp, int32_t lp_dtype,
                  void* stream);
/* sum the partials: bias grads of the heads -> grad_head_bias (A+1), logstd grads (+ -entropy_coef) ->
 * grad_logstd (A); the statistics (means) -> stats[stat_idx][PPO_LOSS_NSTAT] (stat_idx from device);
 * the KL also -> kl_out (the slot that rides in the gradient all-reduce); grad_scale as ppo_loss_grad */
int ppo_loss_finalize(const float* partials, int32_t nblk, int32_t A, int32_t mb_rows, float entropy_coef,
                      const float* grad_scale, float* grad_head_bias, float* grad_logstd, float* stats,
                      const int32_t* stat_idx, float* kl_out, void* stream);

/* dz = dh * (h > 0 ? 1 : h + 1) (ELU alpha 1, output form), rows x cols (cols multiple of 64);
 * dtype of dh / h / dz: PPO_DT_* (fp32, or one low-precision type lp in bf16 / fp16: (f32,f32,f32),
 * (f32,f32,lp), (f32,lp,lp), (lp,lp,lp)); per-block column partial sums
 * of dz into partials[nblk][cols] (nblk = ppo_elu_bwd_blocks(rows)) */
int ppo_elu_bwd_blocks(int32_t rows);
int ppo_elu_bwd(const void* dh, int32_t dh_dtype, const void* h, int32_t h_dtype, void* dz, int32_t dz_dtype,
                int32_t rows, int32_t cols, float* partials, void* stream);

/* Sum S partial rows into the flat gradient, several independent jobs in ONE launch (split-K GEMM
 * partials, ELU bias partials): dst[r*dst_stride + c] = sum_s src[s*src_n + r*src_cols + c] for
 * r < out_rows, c < dst_cols (fixed summation order). */
typedef struct {
    const float* src;
    float* dst;
    int32_t S, out_rows, src_cols, dst_cols, dst_stride;
    int64_t src_n;
} ppo_reduce_job_t;
#define PPO_MAX_JOBS 16
int ppo_reduce_rows(const ppo_reduce_job_t* jobs_host, int32_t njobs, void* stream);
/* ppo_reduce_rows + ppo_sqnorm's work over the values it writes (round 5, one gradient pass fewer when no
 * all-reduce sits between the two): norm_partials receives [nblk sums of (v / scale)^2 | nblk non-finite
 * counts] (scaler: as ppo_sqnorm) over every dst element written plus the extra arrays (the gradients
 * other kernels wrote: head biases, log-sigma); *nblk_out = nblk (<= max_blocks) is the count to pass to
 * ppo_adam / ppo_tail as nblk_norm. */
/* Adam's step inputs as a launch ahead of the optimizer found them: lr, step (the count before this step),
 * scale (the loss scale; 1 without a scaler).  Written by ppo_sqnorm / ppo_reduce_rows_norm when given a
 * snapshot pointer (one thread, after nothing of theirs depends on it), read by ppo_adam_step. */
typedef struct {
    double lr;
    double step;
    float scale;
    float pad_;
} ppo_opt_snap_t;

/* ... + snap (NULL = none): the snapshot of *lr, *step and the scale (lr / step non-NULL with it) */
int ppo_reduce_rows_norm(const ppo_reduce_job_t* jobs_host, int32_t njobs, const float* scaler, const float* extra0,
                         int32_t extra0_n, const float* extra1, int32_t extra1_n, float* norm_partials,
                         int32_t max_blocks, int32_t* nblk_out, const double* lr, const double* step,
                         ppo_opt_snap_t* snap, void* stream);

/* Rollout policy head (graph-safe sampling): head = [mu | value] (rows x (A+1), fp32), logstd (A).
 * actions = mu + exp(logstd) * N(0, 1) with the normals from Philox4x32-10 keyed by `seed` and
 * countered by (row, chunk, *step_ctr) -- the same draw for the same (seed, step, row) on any replay;
 * neglogp as ModelA2CContinuousLogStd.neglogp; values denormalised by the value normaliser
 * (sqrt(var + eps) * clamp(v, -5, 5) + mean) when vms_mean != NULL.  Outputs are row-major
 * (rows x A for actions / mus / sigmas, rows for neglogp / values). */
int ppo_policy_sample(const float* head, const float* logstd, int32_t A, int32_t rows, uint64_t seed,
                      const int64_t* step_ctr, const double* vms_mean, const double* vms_var, float vms_eps,
                      float* actions, float* neglogp, float* values, float* mus, float* sigmas, void* stream);
/* *ctr += inc (one thread; orders after the kernels that read it) */
int ppo_counter_add(int64_t* ctr, int64_t inc, void* stream);

/* Fused actor-critic trunk forward on MFMA (lp in, fp32 accumulate; lp = dtype: PPO_DT_BF16 on
 * v_mfma_f32_32x32x16_bf16, PPO_DT_F16 on v_mfma_f32_32x32x16_f16 -- rl_games' fp16 autocast): 5 layers
 * x 256, ELU, then the fp32 heads.  x: rows x 64 lp (normalised obs, zero-padded 59 -> 64; row stride
 * x_stride >= 64); w[0]: 256 x 64 lp, w[1..4]: 256 x 256 lp (the trunk mirror); b[l]: 256 fp32; wh: nh x 256 fp32
 * ([mu.w | value.w]), bh: nh fp32 (nh <= 32).  Outputs (row-major, NULL = skip): h[0..4] = layers
 * 1..5 (lp, columns 0..255 of rows with stride h_stride >= 256, a multiple of 8; columns beyond are
 * not touched), head = rows x nh fp32 holding lp values: the heads run as
 * rl_games' autocast runs them -- lp layer-5 activations, lp(wh), lp(bh), fp32 accumulation, an lp
 * output.  x_stride is a multiple of 8.  A workgroup of 8 waves owns 128 rows; wave w keeps the weights
 * of output features [32w, 32w + 32) in registers and the activations pass through LDS. */
typedef struct {
    const uint16_t* x;
    const uint16_t* w[5];
    const float* b[5];
    const float* wh;
    const float* bh;
    uint16_t* h[5];
    float* head;
    int32_t rows, nh, x_stride, h_stride;
    int32_t dtype; /* PPO_DT_BF16 or PPO_DT_F16 */
    /* Fused input normalisation (the RunningMeanStd of the model, rl_games running_mean_std.py; replaces a
     * ppo_obs_normalize launch): when obs != NULL the layer-0 input is formed in-kernel from the fp32
     * observation rows [*mb_idx * rows, (*mb_idx + 1) * rows) of obs (row stride obs_dim <= 64):
     * clamp((obs - (float)mean) / sqrtf((float)var + eps), -5, 5), zero in columns obs_dim..63, rounded
     * to lp -- the same formula as ppo_obs_normalize -- and written to x_out (columns 0..63, row stride
     * x_stride) when x_out != NULL (the weight gradients read it); x is then unused. */
    const float* obs;
    const int32_t* mb_idx;
    const double* mean;
    const double* var;
    uint16_t* x_out;
    float eps;
    int32_t obs_dim;
    /* Fused losses (round 5): with loss.A > 0 (12 or 21; training form, every h[] set, obs set) the
     * workgroup runs ppo_loss_grad's work for its 128 rows right after the heads, from the head values
     * it holds (the minibatch is rows [*mb_idx * rows, ...) of the dataset tensors): the dataset's mu /
     * sigma rows updated, the 16-bit head gradient into loss.dhead_lp (rows x 32, the trunk's dtype), one
     * row of block partials per workgroup into loss.partials (ppo_loss_blocks(rows) rows) -- bit-identical
     * to ppo_loss_grad, one launch fewer per minibatch. */
    struct {
        int32_t A;
        const float* logstd;
        const float* actions;
        float* ds_mu;
        float* ds_sigma;
        const float* old_neglogp;
        const float* advantages;
        const float* old_values;
        const float* returns;
        ppo_loss_cfg_t cfg;
        const float* grad_scale;
        uint16_t* dhead_lp;
        float* partials;
    } loss;
} ppo_mlp_fwd_t;
int ppo_mlp_forward(const ppo_mlp_fwd_t* args_host, void* stream);

/* Fused backward of the trunk's input-gradient chain (the weight gradients are ppo_weight_grads):
 *   dh5 = Wh^T dhead (lp MFMA, fp32 accumulation: autocast's head Linear backward), dz4 = dh5 * elu'(h5),
 *   for l = 4..1: dz_{l-1} = (W_l^T dz_l) * elu'(h_l)   (lp MFMA, W_l^T from wt[l-1])
 * with elu'(y) = 1 if y > 0 else y + 1 (output form), one lp rounding per dz.  dhead: rows x 32 lp
 * (ppo_loss_grad's dhead_lp; columns nh..31 zero); wh: nh x 256 fp32 (rounded to lp in-kernel);
 * wt[k]: W_{k+1}^T (256 x 256 lp, row = input feature); h[k]: layer k+1 activations (lp, k = 0..4, row
 * stride h_stride); outputs dz[l] (l = 0..4): rows x 256 lp.  lp = dtype. */
typedef struct {
    const uint16_t* dhead;
    const float* wh;
    const uint16_t* wt[4];
    const uint16_t* h[5];
    uint16_t* dz[5];
    int32_t rows, nh, h_stride;
    int32_t dtype; /* PPO_DT_BF16 or PPO_DT_F16 */
} ppo_mlp_bwd_t;
int ppo_mlp_backward(const ppo_mlp_bwd_t* args_host, void* stream);

/* Split-K weight + bias gradients of the trunk layers and the head weights, all in one launch (the
 * Linear weight / bias gradients of loss.backward() in a2c_continuous.py calc_gradients):
 *   part[l][s][o][c]   = sum_{b in split s} dz[l][b][o] * hin[l][b][c]   (o < nout[l], c < kin[l])
 *   part[l][s][o][kin] = sum_{b in split s} dz[l][b][o]                   (bias column; trunk only)
 * Job l < 5 is trunk layer l: dz[l] rows x 256 lp, nout 256, kin 64 (l = 0) or 256.  Job 5 (when
 * layers == 6) is the heads: dz[5] = ppo_loss_grad's dhead_lp (rows x 32), nout 32, kin 256 (layer 5's
 * activations), no bias column.  hin[l]: rows x hin_stride[l] lp; part[l]: splits[l] x nout x hin_stride[l]
 * fp32 (columns past kin[l] (+1) untouched).  Split s of job l covers rows
 * [rows*s/splits[l], rows*(s+1)/splits[l]).  A trunk split is two workgroups (output features 0..127 and
 * 128..255), placed 8 block indices apart so that, in every full group of 8 pairs, the two halves run on
 * one XCD and the layer input they both stream is fetched once into its L2 (a performance placement,
 * not a requirement: a last group of fewer than 8 pairs -- any split total that is not a multiple of 8,
 * e.g. small minibatches -- is handled and only loses the co-location).  The partials are summed by
 * ppo_reduce_rows. */
/* ppo_loss_finalize's arguments, for running that work as a side job (below) */
typedef struct {
    const float* partials; /* ppo_loss_grad's block partials, nblk x (2A+1+PPO_LOSS_NSTAT); NULL = no side job */
    int32_t nblk, A, mb_rows;
    float entropy_coef;
    const float* grad_scale;
    float* grad_head_bias;
    float* grad_logstd;
    float* stats;
    const int32_t* stat_idx;
    float* kl_out;
} ppo_loss_side_t;
typedef struct {
    const uint16_t* dz[6];
    const uint16_t* hin[6];
    float* part[6];
    int32_t kin[6];
    int32_t hin_stride[6];
    int32_t splits[6];
    int32_t rows, layers;
    int32_t dtype; /* PPO_DT_BF16 or PPO_DT_F16 */
    /* Side job (round 5): with loss.partials set (and layers == 6), the head job's last workgroup also does
     * ppo_loss_finalize's work -- a head split streams about 0.6 of a trunk split's bytes, so that
     * workgroup has the slack, and the minibatch step saves a launch.  Same outputs as ppo_loss_finalize
     * (the sums over the blocks in block order: equal to its to fp32 rounding). */
    ppo_loss_side_t loss;
} ppo_wgrad_t;
int ppo_weight_grads(const ppo_wgrad_t* args_host, void* stream);

/* Rollout bookkeeping of one step (a2c_common.play_steps after env_step), per env:
 *   shaped = (reward + shift) * scale [+ gamma * value * time_out]  -> shaped_out (td rewards[n])
 *   cur_r += reward; cur_s += shaped; cur_l += 1
 *   for done envs: block partials of (cur_r, cur_s, cur_l, 1) -> partials[nblk][4], then cur_* = 0
 * then ppo_meter_update folds the finished episodes into the three AverageMeters (rl_games
 * torch_ext.AverageMeter: mean of the last max_size games) -- no host round trip, no nonzero(). */
int ppo_rollout_post_blocks(int32_t n);
int ppo_rollout_post(const float* reward, const uint8_t* done, const uint8_t* time_out, const float* value,
                     int32_t n, float scale, float shift, float gamma, int32_t bootstrap, float* shaped_out,
                     float* cur_r, float* cur_s, float* cur_l, float* partials, void* stream);
/* meters: mean[3] (reward, shaped reward, length), size[3] (current_size) */
int ppo_meter_update(const float* partials, int32_t nblk, float max_size, float* mean3, float* size3, void* stream);

/* partials[2 * nblk] (fp32, nblk = ppo_sqnorm_blocks()): [0, nblk) block sums of (g / scale)^2 (scaler
 * NULL: scale 1; NaN / inf propagate into the norm as in torch), [nblk, 2 nblk) block counts of
 * non-finite g (GradScaler's found_inf: an OR over isfinite, separate from the norm) */
int ppo_sqnorm_blocks(void);
/* snap (NULL = none): as ppo_reduce_rows_norm */
int ppo_sqnorm(const float* g, int64_t n, const float* scaler, float* partials, const double* lr, const double* step,
               ppo_opt_snap_t* snap, void* stream);
/* clip (max_norm > 0: g *= min(1, max_norm / (||g|| + 1e-6))) + Adam (torch.optim.Adam, amsgrad off,
 * weight_decay 0) with device lr / step (fp64); writes the mirror (mirror_dtype PPO_DT_BF16 / PPO_DT_F16)
 * of the listed segments.  scaler (device fp32 [scale, growth tracker], NULL = none): the gradients
 * carry the loss scale -- a non-finite element skips the whole update (GradScaler.step), otherwise
 * g / scale (exact: a power of two) is what is clipped and applied (GradScaler.unscale_).
 * nblk_norm >= 1 (the partials' pair count); segments hold fewer than 2^31 elements each */
int ppo_adam(float* p, const float* g, float* m, float* v, int64_t n, const float* sqnorm_partials, int32_t nblk_norm,
             float max_norm, const double* lr, double* step, float beta1, float beta2, float eps,
             const ppo_seg_t* segs_host, int32_t nseg, void* mirror, int32_t mirror_dtype, const float* scaler,
             void* stream);
/* adaptive LR (rl_games AdaptiveScheduler; kl_threshold <= 0: identity) from kl (device fp32), then
 * step += 1 (Adam's count; ppo_adam used step + 1) unless the scaler skipped the step,
 * mb_idx = (mb_idx + 1) % n_minibatches, stat_idx += 1; with a scaler, GradScaler.update from the same
 * norm partials (nblk_norm >= 1): scale *= 0.5 after a skipped step, *= 2 after growth_interval good ones
 * in a row */
int ppo_tail(double* lr, const float* kl, float kl_threshold, double min_lr, double max_lr, double* step,
             int32_t* mb_idx, int32_t n_minibatches, int32_t* stat_idx, float* scaler, const float* sqnorm_partials,
             int32_t nblk_norm, int32_t growth_interval, void* stream);

/* ppo_adam then ppo_tail as ONE launch: the clip + Adam of ppo_adam with lr, step and the scale read from
 * `snap` (taken this minibatch by ppo_sqnorm / ppo_reduce_rows_norm), and ppo_tail's update of the
 * originals (lr, step, mb_idx, stat_idx, scaler) run by the launch's first block -- no other block reads
 * them, so no hand-off is needed.  Same arguments and results as the two calls. */
typedef struct {
    float* p;
    const float* g;
    float* m;
    float* v;
    int64_t n;
    const float* norm_partials;
    int32_t nblk_norm;
    float max_norm, beta1, beta2, eps;
    const ppo_seg_t* segs_host;
    int32_t nseg;
    void* mirror;
    int32_t mirror_dtype;
    const ppo_opt_snap_t* snap;
    /* the tail (ppo_tail's arguments) */
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
} ppo_adam_step_t;
int ppo_adam_step(const ppo_adam_step_t* a, void* stream);


#ifdef __cplusplus
}
#endif
#endif

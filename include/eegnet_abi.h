/*
 * eegnet_abi.h -- C-ABI of libeegnet_hip.so, the MI355X (gfx950) EEGNet train/infer step.
 *
 * Drop-in boundary for the reference's hot path (PraKesEy/EEGNetReplication):
 *   EEGNet.forward            src/eegnet_repl/model.py:91-99   -> eegnet_forward_train / eegnet_forward_eval
 *   loss.backward() + hooks   src/eegnet_repl/model.py:44,84,147 -> eegnet_backward
 *   optimizer.step() (Adam)   src/eegnet_repl/train.py:94-101, model.py:148 -> eegnet_adam_step
 *   one hot-loop iteration    src/eegnet_repl/model.py:136-148 -> eegnet_train_step
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer (hipMalloc / torch CUDA tensor) unless noted.  The library never
 *     allocates or frees; the caller owns params, buffers and the workspace (eegnet_workspace_bytes).
 *   - All work is enqueued on `stream`; no host synchronisation happens inside, so every call can be
 *     captured in a hipGraph.
 *   - Return 0 on success, a negative EEGNET_E* code otherwise; eegnet_last_error() (thread-local)
 *     describes the failure.  The Python side raises RuntimeError with that text.
 *   - `params` is ONE flat fp32 buffer in nn.Module.named_parameters() order:
 *       temporal.0.weight[F1,1,1,K1]  temporal.1.weight[F1]  temporal.1.bias[F1]
 *       spatial.weight[F2,1,C,1]      aggregation.0.weight[F2] aggregation.0.bias[F2]
 *       block_2.0.weight[F2,1,1,16]   block_2.1.weight[F2,F2,1,1]
 *       block_2.2.weight[F2]          block_2.2.bias[F2]
 *       classifier.weight[4,F2*(T/32)] classifier.bias[4]          (F2 = F1*D)
 *     (1,716 floats for EEGNet-8,2 at C=22, T=256).  `grads` has the same layout.
 *   - `bn_buffers` is one flat fp32 buffer: running_mean/running_var of temporal.1 [F1,F1],
 *     aggregation.0 [F2,F2], block_2.2 [F2,F2].  The three num_batches_tracked counters are an
 *     optional separate int64[3] device buffer (the last argument of eegnet_forward_train and
 *     eegnet_train_step; NULL = not tracked), incremented in-kernel once per train-mode forward.
 *   - x is [B,C,T] fp32 row-major; labels int64 [B] in [0,4); logits fp32 [B,4].
 *   - Dropout keep-masks: uint8 [B,F2,T/4] and [B,F2,T/128] (1 = keep), nullable.  NULL means the
 *     on-device counter-based generator keyed by (seed, offset): the same (seed, offset) always
 *     produces the same masks, and forward and backward see the same ones.
 */
#ifndef EEGNET_ABI_H
#define EEGNET_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct eegnet_dims {
    int B;          /* trials in the batch                                  */
    int C;          /* EEG channels          (model.py:13 `C`)              */
    int T;          /* samples per trial     (model.py:13 `T`)              */
    int F1;         /* temporal filters      (model.py:13, default 8)       */
    int D;          /* depth multiplier      (model.py:13, default 2)       */
    int K1;         /* temporal kernel length (model.py:26: 32; 64 also supported) */
    float p_drop;   /* dropout p             (model.py:13, 50, 74)          */
    float bn_eps;   /* BatchNorm2d eps (1e-5)                               */
    float bn_momentum; /* BatchNorm2d momentum (0.1)                        */
    int x_pitch;    /* floats between consecutive channel rows of x (0: T, x is [B][C][T]); a
                       larger pitch (eegnet_x_pitch) lets the training kernels load the rows of
                       x in 16-byte units; samples [T, x_pitch) of a row are never read     */
} eegnet_dims;

enum {
    EEGNET_OK = 0,
    EEGNET_EINVAL = -1,   /* unsupported or inconsistent dims / null pointer */
    EEGNET_ELAUNCH = -2,  /* a kernel launch failed                          */
};

enum { EEGNET_TRAIN = 1, EEGNET_EVAL = 0 };

/* eegnet_backward flags */
enum {
    EEGNET_NO_CLAMP = 1,      /* leave model.py:44/84 clamps to eegnet_clamp_grads (after an all-reduce) */
    EEGNET_KEY_FROM_STEP = 2  /* eegnet_train_step: dropout key = mix(seed, offset + *step), read on the
                                 device, so a captured hipGraph draws fresh masks on every replay */
    /* 4 (round 5's opt-in one-launch persistent step) is retired: eegnet_train_step rejects any other
       bit with EEGNET_EINVAL */
};

/* Number of fp32 elements of the flat parameter buffer for these dims. */
int eegnet_param_count(const eegnet_dims* dims, int64_t* out);

/* Bytes of scratch the train-mode calls need (forward -> backward state lives here).  The workspace
 * must be zero-filled once before its first use (hipMemset / torch.zeros); the library keeps its
 * reduction tickets re-armed from then on. */
int eegnet_workspace_bytes(const eegnet_dims* dims, size_t* out);

/* Train-mode forward (BN batch statistics, dropout, running-stat momentum update).
 * Replaces model.py:141 `preds = model(signals)` in train mode.  Leaves what backward needs in `ws`.
 * num_batches_tracked (nullable): the three BatchNorm2d counters as one int64[3] device buffer,
 * incremented in-kernel. */
int eegnet_forward_train(const eegnet_dims* dims, const float* params, float* bn_buffers,
                         const float* x, const uint8_t* mask2, const uint8_t* mask3,
                         uint64_t seed, uint64_t offset, float* logits, void* ws, void* stream,
                         int64_t* num_batches_tracked);

/* Backward of the last eegnet_forward_train on the same `ws` (same x, params, masks, seed/offset).
 * Gradient source: `dlogits` [B,4] if non-NULL (autograd), else mean cross-entropy against `labels`
 * (train.py:103), in which case the scalar loss is written to `loss` (device fp32, nullable).
 * `grads` receives all 12 parameter gradients with the clamps of model.py:44 (+-1) and model.py:84
 * (+-0.25) applied, unless flags has EEGNET_NO_CLAMP. */
int eegnet_backward(const eegnet_dims* dims, const float* params, const float* x,
                    const float* dlogits, const int64_t* labels, const uint8_t* mask2,
                    const uint8_t* mask3, uint64_t seed, uint64_t offset, float* grads, float* loss,
                    void* ws, void* stream, int flags);

/* The gradient hooks of model.py:44 (spatial.weight, +-1) and model.py:84 (classifier.weight,
 * +-0.25) on a flat grad buffer -- for data-parallel runs, after the gradient all-reduce. */
int eegnet_clamp_grads(const eegnet_dims* dims, float* grads, void* stream);

/* Eval-mode forward (running statistics, no dropout): one fused kernel.  model.py:161/220, ui.py:35. */
int eegnet_forward_eval(const eegnet_dims* dims, const float* params, const float* bn_buffers,
                        const float* x, float* logits, void* stream);

/* bf16 batched eval-mode forward (BASELINE cfg5, EEGNet-16,4 at 64ch x 512):
 * the same function as eegnet_forward_eval (model.py:91-99 in .eval(), called at model.py:161/220,
 * ui.py:35) on bf16 input x [B,C,T] (16-byte aligned when T % 8 == 0), bf16 MFMA operands and fp32
 * accumulation; params / bn_buffers / logits as for eegnet_forward_eval (fp32).  Covers every
 * supported (C, T, F1, D) whose trial fits one workgroup's LDS, including the F2 > 16 shapes the
 * fp32 path runs through the wide kernels. */
int eegnet_forward_eval_bf16(const eegnet_dims* dims, const float* params, const float* bn_buffers,
                             const uint16_t* x, float* logits, void* stream);

/* torch.optim.Adam step (weight_decay 0, amsgrad off) over n elements; `step` is a device int32
 * that is incremented in-kernel (graph-capturable).  torch/optim/adam.py:457,476,531-547. */
int eegnet_adam_step(int64_t n, float* params, const float* grads, float* exp_avg,
                     float* exp_avg_sq, int32_t* step, float lr, float beta1, float beta2,
                     float eps, void* stream);

/* One fused hot-loop iteration (model.py:141-148): forward_train + CE + backward + clamps + Adam.
 * adam_state = [exp_avg | exp_avg_sq] (2 * param_count floats); step as in eegnet_adam_step.
 * adam_state == NULL stops after the gradients (data-parallel callers all-reduce them, then call
 * eegnet_clamp_grads and eegnet_adam_step); flags as for eegnet_backward, plus EEGNET_KEY_FROM_STEP
 * (needs step; the mask key then follows the device step, for hipGraph capture).  logits is nullable. */
int eegnet_train_step(const eegnet_dims* dims, float* params, float* bn_buffers, const float* x,
                      const int64_t* labels, uint64_t seed, uint64_t offset, float* grads,
                      float* adam_state, int32_t* step, float lr, float beta1, float beta2,
                      float eps, float* loss, float* logits, void* ws, void* stream, int flags,
                      int64_t* num_batches_tracked);

/* One stage of a data-parallel train step with synchronised BatchNorm (SURVEY 8(e)2's SyncBN option;
 * the reference has no multi-device path -- this is the single-device semantics of model.py:141-148
 * over the global batch, split at the five batch-global reductions so a caller can all-reduce each).
 * stage 2k (k = 0..4: passes A..E) launches pass k and leaves its fp64 sums in the workspace
 * (eegnet_stage_sums says where) instead of finalizing; stage 2k + 1 runs pass k's finalize on those
 * sums once the caller has summed them over the ranks (all_reduce SUM).  norm_batch = the global batch:
 * BatchNorm statistics, running statistics and the CE mean are normalised by it, so the gradients,
 * clamps (model.py:44/84, on the global gradient) and the fused Adam of stage 9 come out the same on
 * every rank and no separate gradient all-reduce is needed.  Other arguments as for eegnet_train_step
 * (adam_state NULL: gradients only).  F1*D <= 16 only. */
int eegnet_train_stage(const eegnet_dims* dims, int stage, int64_t norm_batch, float* params,
                       float* bn_buffers, const float* x, const int64_t* labels, uint64_t seed,
                       uint64_t offset, float* grads, float* adam_state, int32_t* step, float lr,
                       float beta1, float beta2, float eps, float* loss, void* ws, void* stream,
                       int flags, int64_t* num_batches_tracked);

/* Where stage 2k leaves pass k's sums in a workspace of eegnet_workspace_bytes(dims): byte offset and
 * number of fp64 values (the buffer a synchronised-BatchNorm caller all-reduces). */
int eegnet_stage_sums(const eegnet_dims* dims, int pass, size_t* offset_bytes, int* count);

/* One model (fold) of a fold-indexed train step: everything eegnet_train_step takes per model.
 * Every pointer is a device pointer; an array of these lives in DEVICE memory. */
typedef struct eegnet_fold {
    float* params;                  /* flat parameters (named_parameters order)                   */
    float* bn_buffers;              /* rm1 rv1 rm2 rv2 rm3 rv3                                    */
    int64_t* num_batches_tracked;   /* int64[3] or NULL                                           */
    const float* x;                 /* this fold's epoch data [N, C, T], rows already shuffled    */
    const int64_t* labels;          /* [N]                                                        */
    float* grads;                   /* flat gradients (written)                                   */
    float* adam_state;              /* [exp_avg | exp_avg_sq]                                     */
    int32_t* step;                  /* Adam step counter (device int32)                           */
    float* losses;                  /* per-batch loss slots (NULL: not written)                   */
    void* ws;                       /* workspace of eegnet_workspace_bytes(dims), zeroed once     */
    const int64_t* perm;            /* epoch permutation: batch row r is x / labels row perm[r]   */
                                    /* (NULL: row r itself, i.e. x already shuffled)              */
    uint64_t seed;                  /* dropout key seed: key = mix(seed, offset + *step)          */
    const float* xstat;             /* NULL, or eegnet_x_stats(x) of this fold's x: its rows' BN1  */
                                    /* lag sums, read instead of recomputed every epoch (ABI 5:   */
                                    /* appended after seed, so the round-3 fields keep offsets)   */
} eegnet_fold;

/* The hot-loop iteration of eegnet_train_step (forward + CE + backward + clamps + Adam) for
 * `nfolds` independent models in ONE launch per pass: the fold index is the grid's y dimension,
 * each fold keeps its own parameters, BN buffers, Adam state, workspace and reductions.  Replaces
 * the per-fold loops of train.py:50-140 (within-subject, 36 runs) and train.py:182-290
 * (cross-subject, 90 runs) at batch 64 (train.py:87,229), where one model's step cannot fill the
 * GPU.  All folds train on batch [row0, row0 + dims.B) of their own x / labels -- rows
 * perm[row0 ...] of x / labels when the fold has a perm (the epoch's shuffle without a gather of
 * the trials) -- and the loss goes to losses[slot].  Dropout keys follow each fold's device step (EEGNET_KEY_FROM_STEP semantics with
 * `offset`), so a captured graph draws fresh masks on every replay.  F1*D <= 16 only. */
int eegnet_train_step_folds(const eegnet_dims* dims, int nfolds, const eegnet_fold* folds, int64_t row0,
                            int64_t slot, uint64_t offset, float lr, float beta1, float beta2, float eps,
                            void* stream);

/* Per-trial BatchNorm-1 statistics of x that do not depend on the parameters: for each of the n
 * trials x[i] ([C][T] rows at dims->x_pitch), the lag sums of its zero-padded rows summed over the
 * channels G0[d] (d < K1), the window-0 sample sum, and the head / tail products and sums of the
 * 'same' padding's edges -- eegnet_x_stats_width(dims) floats per trial, written to out[n][width].
 * BN1's batch statistics (model.py:32) are w1-quadratic forms of their sums over the batch
 * (DESIGN.md section 3), so a fold whose training set is fixed for all epochs (train.py:87-106,
 * 225-246) computes them once and its fold-indexed steps read the batch's rows through eegnet_fold.
 * xstat instead of recomputing the lag-Gram (180 K of pass A's 423 K MAC per 22 x 256 trial).  The
 * narrow path (F1*D <= 16) only; dims->B is ignored. */
int eegnet_x_stats_width(const eegnet_dims* dims);
int eegnet_x_stats(const eegnet_dims* dims, int64_t n, const float* x, float* out, void* stream);

/* Optional per-kernel device timing for benchmarks: `on` is a bitmask of kernel ids (bit i = the
 * i-th name eegnet_profile_collect reports: k_pass_a, k_pass_b, k_pass_c, k_pass_d, k_pass_e,
 * k_adam, k_infer, memset_tickets, k_infer_bf16, k_wpass_a, k_wpass_b, k_wpass_b2, k_wpass_c,
 * k_wpass_d, k_wpass_e, k_winfer, k_coltail, k_xstats; -1 = all, 0 = off; the k_w* kernels are the F2 > 16 path).  Every selected kernel this
 * thread launches through the calls above is bracketed by hipEvents.  eegnet_profile_collect
 * synchronises them and reports, per kernel name (32-byte slots in `names`), launch count and
 * summed device ms; it returns the number of kernels in *n_out.  Not for use under hipGraph
 * capture.  Each bracketed launch costs a few microseconds of stream time, so a benchmark's timed
 * region should select only the kernel it prices. */
int eegnet_profile_enable(int on);
int eegnet_profile_collect(char* names, int* counts, double* total_ms, int cap, int* n_out);

/* Optional timeline instrumentation for kernel tuning: while `buf` (a zeroed device buffer of
 * eegnet_trace_bytes() bytes) is set, every pass kernel stamps phase boundaries into it
 * ([pass][workgroup][16] uint64: wall clock at entry / prologue / loop end / publish / tickets /
 * finalize, shader-clock sums of in-loop phases).  NULL turns it off. */
int eegnet_trace_enable(void* buf);
size_t eegnet_trace_bytes(void);

/* The x row pitch the training entry points (eegnet_train_step, _folds, _forward_train, _backward,
 * _train_stage) load fastest for `dims`: T rounded up to 4 floats when the kernels for these dims take
 * x rows in 16-byte units at such a pitch (22 x 257, the recordings' shape: a 257-float row is not
 * 16-byte aligned), else T.  Only those dims accept a pitch other than T (22 x 256 rows are 16-byte
 * units already; its kernels have the pitch T compiled in).  Every other entry point needs x_pitch = 0
 * or T.  No GPU needed. */
int eegnet_x_pitch(const eegnet_dims* dims);

/* 1 when `dims` run the wide kernels compiled for the EEGNet-16,4 64 x 512 geometry (compile-time
 * bounds and offsets), 0 when they run the generic wide / narrow kernels (for a wide K1 = 32 shape the
 * differing geometry fields are then in eegnet_last_error()), < 0 on invalid dims.  No GPU needed. */
int eegnet_wide_spec(const eegnet_dims* dims);

/* sizeof(eegnet_dims) and sizeof(eegnet_fold) as this library was compiled: a binding checks its
 * struct mirrors against them at load (a stale library with another fold layout would read every
 * fold after the first from the wrong offsets). */
size_t eegnet_dims_bytes(void);
size_t eegnet_fold_bytes(void);

/* The struct layouts above are versioned: EEGNET_ABI_VERSION changes whenever a field of eegnet_dims
 * or eegnet_fold moves (a reordering keeps the size, so eegnet_fold_bytes alone cannot catch it).
 * A caller asserts eegnet_abi_version() == the EEGNET_ABI_VERSION it was compiled against.
 *   4: eegnet_fold.xstat added before seed (round 4)
 *   5: xstat moved after seed -- the round-3 fields at their round-3 offsets again (round 5) */
#define EEGNET_ABI_VERSION 5
int eegnet_abi_version(void);

/* Thread-local description of the last error ("" if none). */
const char* eegnet_last_error(void);

/* Library/build identification string (gfx target, build flags). */
const char* eegnet_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* EEGNET_ABI_H */

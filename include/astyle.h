/*
 * astyle.h — C ABI of libastyle.so, the MI355X (gfx950) implementation of the
 * winlp4ever/audio_style_transfer optimisation loop's hot path.
 *
 * The reference has no FFI: its boundary is Python calling TensorFlow 1.x.  Each entry point
 * below replaces one reference interface (file:line into the reference):
 *
 *   ast_create / ast_destroy  <- GatysNet.build graph construction + tf.Session
 *                                (methods.py:44-77, 184-188)
 *   ast_set_weight            <- tf.train.Saver(...).restore(sess, ckpt)  (methods.py:79-84),
 *                                one variable per call, by TF name (masked.py:141-145)
 *   ast_forward /             <- cfg.build(...) + cfg.extracts (model.py:57-127) evaluated by
 *   ast_get_extract              sess.run on extracts[i]
 *   ast_embeds                <- GatysNet.get_embeds: sess.run(embeds_c | embeds_s)
 *                                (methods.py:86-95; taps and Gram methods.py:58-76)
 *   ast_set_targets           <- the phi_c / phi_s constants fed into define_loss
 *                                (methods.py:113-119, 207-213)
 *   ast_loss_grad             <- one ScipyOptimizerInterface evaluation: sess.run([loss, grad])
 *                                of define_loss + tf.gradients w.r.t. x (methods.py:113-137,167)
 *   ast_set_gamma             <- the --gamma constant of define_loss (methods.py:125)
 *   ast_lbfgs_*               <- scipy L-BFGS-B under ScipyOptimizerInterface.minimize
 *                                (methods.py:132-137,164-181), per clip on the device
 *   ast_adam_step             <- (new) fused optimiser update on the audio buffer; the
 *                                reference's optimiser is host L-BFGS-B (methods.py:133-137)
 *
 * Conventions: every function returns 0 on success and a negative AST_E* code on failure;
 * ast_last_error() returns a thread-local message.  All buffers named *_dev are device
 * pointers owned by the caller; the context owns weights and the activation workspace
 * (sized at create).  No entry point allocates after ast_create, so ast_loss_grad and
 * ast_adam_step are hipGraph-capturable.  A context is bound to one device and is not
 * re-entrant; the stream is passed per call (NULL = legacy default stream).
 */
#ifndef ASTYLE_H
#define ASTYLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AST_OK 0
#define AST_E_ARG (-1)      /* invalid argument / configuration */
#define AST_E_HIP (-2)      /* HIP runtime error */
#define AST_E_STATE (-3)    /* call order violated (e.g. loss before targets) */
#define AST_E_NAME (-4)     /* unknown weight name or wrong element count */

#define AST_MAX_TAPS 32

typedef struct ast_ctx ast_ctx;

typedef struct ast_cfg {
    int batch;                       /* clips per context (the reference: 1) */
    int T;                           /* samples per clip (--batch_size), multiple of 512 */
    int n_cont;                      /* --cont_lyrs count            (methods.py:254) */
    int cont_ids[AST_MAX_TAPS];      /* extract ids 0..31            (methods.py:58) */
    int cnt_channels;                /* --cnt_channels               (methods.py:259) */
    int n_style;                     /* resolved style layer count   (methods.py:60-66) */
    int style_ids[AST_MAX_TAPS];     /* extract ids 0..30 */
    int nb_channels;                 /* --channels                   (methods.py:75,258) */
    int gatys;                       /* --gatys                      (methods.py:68-71) */
    int precision;                   /* 0 = fp32 storage + fp32 MFMA; 1 = bf16 storage + bf16 MFMA;
                                        2 = fp32 storage, encoder GEMMs on split-fp16 MFMA (each
                                        fp32 operand as two fp16 halves, 3 products, fp32
                                        accumulation), Gram on bf16 MFMA */
    float lambd;                     /* --lambd                      (methods.py:125) */
    float gamma;                     /* --gamma, STFT regulariser    (methods.py:121-125) */
} ast_cfg;

/* Context lifetime. */
int ast_create(const ast_cfg* cfg, int hip_device, ast_ctx** out);
void ast_destroy(ast_ctx* ctx);
/* Device bytes ast_create(cfg) on the current device would allocate.  Where the Gram backward
 * puts the style-tapped tensors' direct loss gradients D: a buffer of their own (one more
 * activation set) when the workspace with it leaves max(16 GiB, 10 %) of the device free (this
 * query and ast_create decide so from the current device's free memory), else in place over the
 * activations.  Where both fit and D is >= 4 GiB, the context's first evaluation that is not
 * being captured into a graph (ast_loss_grad / _phase) times its Gram backward in both placements
 * on its own data and keeps the faster (releasing the buffer when in place wins; a capture before
 * it keeps out of place), so the query is the upper bound.  Env ASTYLE_DOOP=1 / 0 forces either.
 * Results are bit-identical in both. */
int ast_workspace_bytes(const ast_cfg* cfg, size_t* out_bytes);
/* *out = 1 when the context keeps D out of place (above), 0 when in place; tuned_ms (may be
 * NULL) [2] = the timed Gram backward in place / out of place (-1: not (yet) timed).  No
 * reference counterpart (a memory-placement report). */
int ast_d_out_of_place(const ast_ctx* ctx, int* out, float* tuned_ms);

/* Weights, HWIO float32 host arrays named as the TF variables ("ae_dilatedconv_7/W",
 * "ae_res_7/biases", "ae_startconv/W", "ae_bottleneck/W", ...). n = element count. */
int ast_set_weight(ast_ctx* ctx, const char* tf_name, const float* host, size_t n);

/* Encoder forward over x_dev [batch, T] (mu-law units, methods.py:49-54). */
int ast_forward(ast_ctx* ctx, const float* x_dev, void* stream);
/* Copy extracts[id] (after ast_forward) to out_dev as float32 [batch, T, C] (C = 16 for id 31). */
int ast_get_extract(ast_ctx* ctx, int extract_id, float* out_dev, void* stream);

/* Forward + taps: emb_c_dev [batch, T, n_cont_cols]; emb_s_dev [batch, nb, L, L] (ours) or
 * [batch, L, 128, 128] (Gatys), l2-normalised.  Either output may be NULL. */
int ast_embeds(ast_ctx* ctx, const float* x_dev, float* emb_c_dev, float* emb_s_dev, void* stream);
int ast_content_cols(ast_ctx* ctx);  /* n_cont_cols of emb_c */

/* Targets (device pointers, caller keeps them alive).  *_shared != 0: one target for all clips. */
int ast_set_targets(ast_ctx* ctx, const float* phi_c_dev, int phi_c_shared,
                    const float* phi_s_dev, int phi_s_shared);

/* One loss+grad evaluation of every clip: grad_dev [batch, T] = d loss / d x, parts_dev
 * [batch, 4] = (content + lambd*style + gamma*reg, content, style, reg).  reg is the STFT
 * regulariser of methods.py:121-123 (0 when T < 1024: no full frame); like TF it is evaluated
 * whatever gamma is, and enters the gradient only through gamma. */
int ast_loss_grad(ast_ctx* ctx, const float* x_dev, float* grad_dev, float* parts_dev, void* stream);
/* ast_loss_grad in two stream-ordered phases: phase 1 = the encoder forward, the content taps and
 * the Gram forward / style loss / Gram backward (grad_dev, parts_dev unused, may be NULL);
 * phase 2 = the backward chain through the blocks, d loss / d x, the loss parts, the STFT
 * regulariser and the range flags (needs phase 1 of the same x first: AST_E_STATE otherwise).
 * phase 0 = both (= ast_loss_grad).  Lets contexts of disjoint clip groups run phase-shifted on
 * separate streams (bench.py --groups): one group's HBM-bound Gram kernels overlap another's
 * MFMA-bound block kernels.  Graph-capturable. */
int ast_loss_grad_phase(ast_ctx* ctx, const float* x_dev, float* grad_dev, float* parts_dev,
                        int phase, void* stream);

/* Per-clip flags accumulated (OR) over every ast_loss_grad since the last reset, into flags_dev
 * (round 4 changed this from "the last call's flags" to sticky; ast_range_flags_last keeps the
 * old per-call meaning)
 * [batch] (int, device) -- sticky, so an out-of-range line-search trial inside a device
 * L-BFGS-B epoch stays visible after the epoch (the reference's ScipyOptimizerInterface sees
 * every evaluation, methods.py:164-181).  Reset: ast_range_flags_reset, ast_lbfgs_begin with
 * x0 or a continuation, and ast_create.  Bits:
 *   AST_RANGE_NONFINITE  the clip's loss parts or gradient hold a NaN / Inf (the reference
 *                        would hand them to the next L-BFGS-B step);
 *   AST_RANGE_ACT        precision 2: a per-clip max |e_l| or the forward intermediate bound
 *                        wdn max|e_l| + bdm (splitwave.h) is >= 2^74 or not finite, so the
 *                        power-of-two scale that keeps the split-fp16 halves in range clamps;
 *   AST_RANGE_GRAD       precision 2: the same for the backward chain max |d loss / d e_l| and
 *                        its bound wrn max|tot|;
 *   AST_RANGE_TINY       precision 2: some per-clip max is below 2^-60 (the halves of that
 *                        tensor lose significand bits; results stay finite).
 * 0 = the evaluation is within the split representation's range.  Graph-capturable. */
#define AST_RANGE_NONFINITE 1
#define AST_RANGE_ACT 2
#define AST_RANGE_GRAD 4
#define AST_RANGE_TINY 8
int ast_range_flags(ast_ctx* ctx, int* flags_dev, void* stream);
/* The same bits for the most recent ast_loss_grad alone (the per-call meaning ast_range_flags
 * had before round 4: a host that checks after every evaluation and never resets can use this
 * one).  Graph-capturable. */
int ast_range_flags_last(ast_ctx* ctx, int* flags_dev, void* stream);
/* Clear the accumulated range flags (stream-ordered; graph-capturable). */
int ast_range_flags_reset(ast_ctx* ctx, void* stream);

/* Workgroup budget of the persistent split block kernels (one workgroup per CU): at most cus
 * CUs (0 = every CU, the default).  Several contexts holding disjoint clip groups can then run
 * concurrently on one GPU, each on its own stream: while one group's HBM-bound Gram kernels run,
 * another's MFMA-bound block kernels use the other CUs (bench.py --groups).  A captured graph
 * bakes the grid in: recapture after a change.  No reference counterpart (a scheduling knob). */
int ast_set_cu_limit(ast_ctx* ctx, int cus);

/* Change gamma (methods.py:125) without rebuilding the context. */
int ast_set_gamma(ast_ctx* ctx, float gamma);

/* Fused Adam on the audio buffer: m, v, x updated in place from grad_dev. step >= 1. */
int ast_adam_step(ast_ctx* ctx, float* x_dev, float* m_dev, float* v_dev, const float* grad_dev,
                  int step, float lr, float beta1, float beta2, float eps, void* stream);
/* Same, with the step counter in device memory: uses *step_dev + 1 and stores it back, so a
 * captured hipGraph of {ast_loss_grad, ast_adam_step_dev} replays as consecutive steps. */
int ast_adam_step_dev(ast_ctx* ctx, float* x_dev, float* m_dev, float* v_dev, const float* grad_dev,
                      int* step_dev, float lr, float beta1, float beta2, float eps, void* stream);

/* Device-resident batched L-BFGS-B: one scipy.optimize.minimize(method='L-BFGS-B') call per
 * clip (no bounds; history m, maxiter, maxls, ftol = factr*eps, gtol = pgtol as scipy's
 * options), all clips advancing together, one loss+grad evaluation per step:
 *   ast_lbfgs_begin(x0)                       x_dev <- fp32(x0): the first point to evaluate
 *   repeat { ast_loss_grad(x_dev -> grad, parts); ast_lbfgs_step(grad, parts) -> next x_dev }
 *   until every clip's phase (ast_lbfgs_state) is 0
 * ws_dev: caller-owned device workspace of ast_lbfgs_workspace_bytes(m); it records the m it
 * was started with (begin with x0), and step / state / a continuation use that m, so loops of
 * different m may share a context.  x0_dev [batch, T] float64 (NULL: continue from each clip's
 * current point with the workspace's own m, the next epoch of methods.py:164);
 * active_dev [batch] int (NULL = all) selects the clips that run.  info_dev [batch, 4] =
 * (phase, iterations, evaluations, reason: 0 running, 1 maxiter, 2 pgtol, 3 rel. reduction
 * of f, 4 abnormal line search, 5 the workspace header is not one begin wrote for this batch
 * and T); x64_dev [batch, T] (may be NULL) the current float64 point.  step / state / a
 * continuation on a workspace this context never started with x0 fail with AST_E_STATE.
 * begin/step allocate nothing, so the step pair is hipGraph-capturable. */
int ast_lbfgs_workspace_bytes(ast_ctx* ctx, int m, size_t* out_bytes);
int ast_lbfgs_begin(ast_ctx* ctx, void* ws_dev, float* x_dev, const double* x0_dev,
                    const int* active_dev, int m, int maxiter, int maxls, double ftol,
                    double gtol, void* stream);
int ast_lbfgs_step(ast_ctx* ctx, void* ws_dev, float* x_dev, const float* grad_dev,
                   const float* parts_dev, void* stream);
int ast_lbfgs_state(ast_ctx* ctx, const void* ws_dev, int* info_dev, double* x64_dev,
                    void* stream);
/* The loss history of the current (or last) minimize call, every evaluation's
 * (total, content, style, regularizer) parts in evaluation order: what the reference's
 * loss_callback writes to its event file at every evaluation (methods.py:147-157, 167).
 * out_dev [batch, max_evals, 4] float; rows past a clip's evaluation count (info[2]) are NaN.
 * The workspace keeps the first AST_LBFGS_HISTORY evaluations of a call (scipy's maxiter 100
 * with maxls 20 makes at most 2001); max_evals in 1..AST_LBFGS_HISTORY. */
#define AST_LBFGS_HISTORY 4096
int ast_lbfgs_history(ast_ctx* ctx, const void* ws_dev, float* out_dev, int max_evals,
                      void* stream);

/* Per-kernel-family device timing (HIP events on the call's stream).  enable!=0 starts
 * recording; ast_timing_read fills out[0..n) with milliseconds summed since enable for
 * {block fwd, block bwd, gram fwd, gram bwd, other} and out[5] = number of ast_loss_grad
 * calls timed, out[6] = launches per family per call (blocks). */
int ast_timing(ast_ctx* ctx, int enable);
int ast_timing_read(ast_ctx* ctx, float* out, int n);

/* TensorFlow checkpoint-V2 reader (tf.train.NewCheckpointReader / Saver.restore, methods.py:
 * 79-84): <prefix>.index (SSTable of BundleEntryProto) + <prefix>.data-NNNNN-of-MMMMM.  Host
 * memory only, no device.  Entries are in name order; dtype is TF's DataType enum (1 float,
 * 2 double, 14 bfloat16, 19 half: read as float32; others refused). */
typedef struct ast_ckpt ast_ckpt;
int ast_ckpt_open(const char* prefix, ast_ckpt** out);
void ast_ckpt_close(ast_ckpt* ck);
int ast_ckpt_num_entries(const ast_ckpt* ck);
int ast_ckpt_entry(const ast_ckpt* ck, int i, char* name, size_t name_cap, int* dtype, int* ndim,
                   int64_t* dims, int max_dims);
int ast_ckpt_read_f32(const ast_ckpt* ck, const char* name, float* host, size_t n);
/* Saver.restore(sess, prefix) (methods.py:79-84): every encoder variable of the NSynth
 * checkpoint (ae_startconv, ae_dilatedconv_1..30, ae_res_1..30, ae_bottleneck; W and biases)
 * by its TF name into ctx, as ast_set_weight.  A missing variable fails with AST_E_NAME. */
int ast_restore(ast_ctx* ctx, const char* prefix);

/* Batched ADMM optimal transport between NMF palettes: OT_ADMM + transform_palette
 * (optimal_transport.py:77-162; compute_permutation = both).  For each of nprob problems,
 * p_mod_dev [n1, d] and p_ref_dev [n2, d] float64 -> plan_dev [n1, n2] (the transport plan),
 * palette_dev [n1, d] (p_ref moved onto p_mod's palette: plan p_ref / (row sums + 1e-10);
 * NULL = skip), iters_dev [nprob] int (ADMM iterations; NULL = skip).  eps, miter as OT_ADMM's
 * (1e-4, 1e5).  fp64, one workgroup per problem; no context.  n1 n2 <= 4096: iterates in
 * registers; larger (up to n1 n2 <= 2^16): iterates in a device workspace the call allocates
 * and frees stream-ordered (hipMallocAsync), so that form is not for capture in a graph that
 * outlives the call.  That kernel is one workgroup per problem streaming ~80 B per cell per
 * ADMM iteration (2^16 cells: ~0.1 ms per iteration); the NMF palettes of the reference are
 * 5..40 components per side. */
int ast_ot_admm(const double* p_mod_dev, const double* p_ref_dev, int nprob, int n1, int n2, int d,
                double eps, double miter, double* plan_dev, double* palette_dev, int* iters_dev,
                void* stream);

const char* ast_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* ASTYLE_H */

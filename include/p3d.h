/*
 * p3d.h -- C ABI of the MI355X-native 2D->3D pose-lifting MLP (libp3d.so).
 *
 * This is the drop-in boundary for the hot path of EsauPR/3d-pose-baseline:
 * the TF1 graph of src/linear_model.py (LinearModel.__init__ :34-151,
 * two_linear :154-201, step :203-245) and the MPJPE arithmetic of
 * src/predict_3dpose.py:evaluate_batches (:352-444).  The reference has no
 * FFI of its own (it is 100% Python over TensorFlow); each entry point below
 * replaces the TensorFlow op group named in its comment, and the Python host
 * (3d-pose-baseline_amd/linear_model.py) binds them through ctypes exactly as
 * INTEGRATION.md shows.
 *
 * Conventions
 *   - Plain C: int status return (P3D_OK = 0), message via p3d_last_error().
 *   - The library owns parameters, optimizer slots and workspace (device memory).
 *     The caller owns every I/O buffer passed in; all I/O pointers are DEVICE
 *     pointers, row-major, fp32 unless stated.
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream).
 *     Every call is asynchronous on that stream.
 *   - One model handle per stream/thread; calls on one handle are not thread-safe.
 */
#ifndef P3D_H_
#define P3D_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define P3D_OK 0
#define P3D_ERR_ARG 1      /* bad argument / shape (TF: InvalidArgumentError) */
#define P3D_ERR_HIP 2      /* HIP runtime failure                            */
#define P3D_ERR_STATE 3    /* call out of order (e.g. backward before fwd)   */
#define P3D_ERR_NOTFOUND 4 /* unknown parameter name                         */

/* p3d_forward ctr value meaning "use the device-resident global_step" (graph-capturable) */
#define P3D_CTR_GLOBAL_STEP 0xFFFFFFFFFFFFFFFFull

#define P3D_DTYPE_F32 0
#define P3D_DTYPE_BF16 1   /* bf16 weights/activations, fp32 accumulate + BN */
#define P3D_DTYPE_F64 2    /* float64 (data-pipeline entry points only)            */

typedef struct p3d_cfg {
  int32_t linear_size;  /* LinearModel(linear_size)            linear_model.py:35 */
  int32_t num_layers;   /* number of two_linear blocks          linear_model.py:36 */
  int32_t residual;     /* two_linear residual add              linear_model.py:199 */
  int32_t batch_norm;   /* tf.layers.batch_normalization        linear_model.py:112 */
  int32_t max_norm;     /* tf.clip_by_norm(w, 1)                linear_model.py:108 */
  int32_t input_size;   /* HUMAN_2D_SIZE = 32                   linear_model.py:62  */
  int32_t output_size;  /* HUMAN_3D_SIZE = 48 (42 if predict_14) linear_model.py:72 */
  int32_t dtype;        /* P3D_DTYPE_*                                              */
  int32_t max_batch;    /* largest B any call will use (workspace sizing)           */
  float bn_eps;         /* 1e-3 (TF default)                                        */
  float bn_momentum;    /* 0.99 (TF default)                                        */
} p3d_cfg;

typedef struct p3d_model p3d_model;

/* Last error message of the calling thread ("" if none). */
const char* p3d_last_error(void);

/* Build a model: allocates trainables (TF creation order), BN moving stats,
 * Adam slots, gradients and activation workspace.  Replaces the variable
 * creation + tf.global_variables_initializer of linear_model.py:84-151
 * (values are zero/one; the host writes kaiming weights via p3d_param_ptr). */
int p3d_create(const p3d_cfg* cfg, p3d_model** out);
int p3d_destroy(p3d_model* m);

/* Parameter table.  Names are TF1 variable names, e.g. "linear_model/w1",
 * "linear_model/two_linear_0/batch_normalization10/moving_mean".  Weights are
 * stored [in, out] row-major exactly like the TF variables (linear_model.py:103).
 * kind: 0 = trainable, 1 = BN moving statistic.  Indexing is 0..count-1. */
int p3d_param_count(const p3d_model* m, int32_t* count);
int p3d_param_info(const p3d_model* m, int32_t idx, const char** name, int64_t* numel,
                   int32_t* kind, int64_t* offset);
int p3d_param_ptr(p3d_model* m, const char* name, void** dptr, int64_t* numel);

/* Flat device buffers (trainables in TF order, 256-byte aligned segments):
 * params/grads/adam_m/adam_v share one layout; `numel` is the padded length.
 * grads is what data-parallel training all-reduces. */
int p3d_flat_ptr(p3d_model* m, int32_t which /*0 params,1 grads,2 adam_m,3 adam_v,4 moving*/,
                 void** dptr, int64_t* numel);

/* Must be called after the host writes parameters through p3d_param_ptr /
 * p3d_flat_ptr (refreshes derived device layouts, e.g. transposed weights). */
int p3d_params_updated(p3d_model* m, void* stream);

/* Bring the TF-layout weight masters (params buffer, p3d_param_ptr) up to date on `stream`.
 * The optimizers of a model without --max_norm read each weight from its packed data-gradient
 * copy and do not write the TF-layout master (4 of the 32 bytes per weight element of the fused
 * step's optimizer); call this before the host reads or writes weights through
 * p3d_param_ptr / p3d_flat_ptr(0).  No device work when the masters are current.
 * p3d_params_updated refuses (P3D_ERR_STATE) while they are behind. */
int p3d_params_sync(p3d_model* m, void* stream);

/* The parameters changed on the device without this library's host code issuing the change
 * (e.g. a replayed HIP graph of training steps, LinearModel.step's cached training graph):
 * host-scheduled derived tables (k_serve6's epilogue constants) are re-formed at their next
 * use.  Host-only, no device work.  Replaces nothing in the reference (TF re-reads variables
 * on every session.run). */
int p3d_params_changed(p3d_model* m);

/* Forward pass: y[B, output_size] = MLP(x[B, input_size]).
 *   training=0: BN uses moving statistics (isTraining=False, linear_model.py:239-245);
 *               at B <= 4 (env P3D_GEMV_MAXB) every layer is a weight-streaming GEMV kernel
 *               (the per-frame step of src/openpose_3dpose_sandbox.py:353-356); results
 *               equal the MFMA path's to fp32 rounding, rows independent of B.
 *   training=1: BN uses batch statistics, updates the moving averages
 *               (UPDATE_OPS, linear_model.py:138-140) and caches activations
 *               for p3d_backward.  Requires B <= max_batch.
 *   keep_prob:  tf.nn.dropout keep probability (1 = identity); the mask is
 *               Philox4x32-10 keyed by (seed, ctr, site, row_offset + row, col).
 * Replaces the forward ops of linear_model.py:103-128. */
int p3d_forward(p3d_model* m, const float* x, int64_t B, float* y, int32_t training,
                float keep_prob, uint64_t seed, uint64_t ctr, int64_t row_offset, void* stream);

/* p3d_forward on workspace rows [ws_row, ws_row + B) (ws_row a multiple of 16,
 * inference only): independent batches issued on different streams with disjoint
 * workspace rows run concurrently; results are bit-identical to p3d_forward. */
int p3d_forward_ex(p3d_model* m, const float* x, int64_t B, float* y, int32_t training,
                   float keep_prob, uint64_t seed, uint64_t ctr, int64_t row_offset, int64_t ws_row,
                   void* stream);

/* Evaluation forward of B rows as ceil(B/64) independent batch-64 steps -- the
 * per-batch LinearModel.step(isTraining=False) loop of predict_3dpose.py:evaluate_batches
 * (:352-444, step at :396) -- in ONE persistent launch (k_serve): each XCD runs whole
 * steps (all layers) out of its own L2, steps dealt round-robin over the XCDs.  Eval BN,
 * keep_prob 1; x [B, input_size], y [B, output_size] device pointers.  fp32 models with
 * linear_size % 128 == 0, input_size <= 64, output_size <= 64, at most 7 blocks.
 * Results equal p3d_forward's to fp32 rounding (the output layer sums 32-column partials
 * in fixed order; deterministic).  The launch is one workgroup per CU and needs all of
 * them resident together: do not run two p3d_serve launches concurrently on one device
 * (other kernels merely delay it).  A launch whose workgroups could not all synchronise
 * stops within ~0.5 s and is reported by the next p3d_serve_check (P3D_ERR_HIP). */
int p3d_serve(p3d_model* m, const float* x, int64_t B, float* y, void* stream);
/* p3d_serve with the evaluation loss of src/linear_model.py:129 (the `loss` output of the eval
 * step(), :239-245) fused into the launch: *loss = mean((y - t)^2) over B x output_size, t [B,
 * output_size] row-major.  x, y, t and loss may be pinned (mapped) host memory: the kernel reads
 * and writes them directly, so LinearModel.step(isTraining=False) is ONE launch from numpy.
 * B <= 4 (the batch-1 front end's evaluation): the persistent small-batch forward p3d_forward
 * runs at that batch, its last output workgroup reducing the loss -- y then has p3d_forward's
 * bits and *loss p3d_mse's on that y; it shares workspace slot 0 with the model's other batch
 * <= 4 calls, so keep those on one stream.  P3D_ERR_ARG where no form covers the launch (> 32
 * batch-64 steps, or a model shape it is not built for): the caller uses p3d_serve + p3d_mse
 * there. */
int p3d_serve_mse(p3d_model* m, const float* x, int64_t B, float* y, const float* t, float* loss, void* stream);
/* p3d_serve_mse that returns once y and *loss hold the results, for outputs in pinned host memory
 * (the reference's session.run returns its fetches: src/linear_model.py:239-245).  The launch's last
 * output tile stores the call's sequence number into a pinned completion word after every row and
 * the loss are system-visible, and the host waits on that word rather than on the runtime's
 * completion signal; the stream itself is not synchronised (later work on it is ordered behind the
 * launch).  Not capturable (P3D_ERR_STATE on a capturing stream).  Errors as p3d_serve_mse, plus
 * P3D_ERR_HIP when the launch ends without storing the word or when a kernel's error word is set
 * (p3d_error_flags reports which). */
int p3d_serve_mse_sync(p3d_model* m, const float* x, int64_t B, float* y, const float* t, float* loss, void* stream);
/* 0 if every p3d_serve launch so far completed its synchronisation (synchronises the device,
 * then reads the kernels' pinned error word).  After a failure p3d_serve refuses new launches
 * (P3D_ERR_HIP) until this call reports it once; the failed launch's rows hold NaN, never
 * unwritten or stale values.  k_serve6 launches pick their sync-word bank on the device, so a
 * captured p3d_serve replays correctly (its epilogue-constant table is re-formed in the graph). */
int p3d_serve_check(p3d_model* m);

/* 0 if every BN-train exchange so far completed (synchronises, then reads the pinned error word).
 * Training layers with batch norm run as one launch each whose row-tile workgroups swap their
 * column statistics inside the launch; a spin that ran out (workgroups not
 * co-resident, e.g. another persistent kernel holding CUs) sets a word this reports once, as
 * P3D_ERR_HIP. */
int p3d_sync_check(p3d_model* m);

/* The kernels' error words without any device round trip or synchronisation: they live in
 * pinned, mapped host memory the kernels write directly, so a caller reads them after a
 * synchronisation it makes anyway (a loss read, an output copy).  *flags: bit 0 a BN-train
 * exchange timed out, bit 1 a p3d_serve spin ran out, bit 2 a p3d_serve placement the launch
 * was not sized for.  clear != 0 resets what was reported (a serve error also re-zeroes the
 * serve sync words, which synchronises).  Replaces no reference interface: TF raised op
 * errors from session.run (src/linear_model.py:236,244). */
int p3d_error_flags(p3d_model* m, int32_t* flags, int32_t clear);

/* MSE loss of linear_model.py:129 and its gradient: loss = mean((y-t)^2) over
 * B*D, dy = (1/(B*D)) * 2*(y-t).  loss_dev: one device float (may be NULL),
 * dy may be NULL. */
int p3d_mse(const float* y, const float* t, int64_t B, int32_t D, float* loss_dev, float* dy,
            void* stream);

/* Backward pass of the last training forward: gradients of every trainable
 * into the flat grads buffer (opt.compute_gradients, linear_model.py:143). */
int p3d_backward(p3d_model* m, const float* dy, int64_t B, void* stream);

/* p3d_forward(training = 1, ctr = P3D_CTR_GLOBAL_STEP) + p3d_mse + p3d_backward in one
 * call (session.run of the train op up to compute_gradients, linear_model.py:129,143):
 * x [B,32], t [B,48] device row-major, 1 <= B <= max_batch; outputs y [B,48]; loss_dev = mean((y-t)^2);
 * gradients in the flat grads buffer.  The MSE runs in the output layer's epilogue. */
int p3d_train_fwd_bwd(p3d_model* m, const float* x, const float* t, int64_t B, float* y,
                      float keep_prob, uint64_t seed, int64_t row_offset, float* loss_dev,
                      void* stream);

/* Gradient-ready buckets for a data-parallel all-reduce that overlaps the backward (the DP
 * form of opt.compute_gradients -> apply_gradients, linear_model.py:143-145).
 * p3d_grad_buckets(m, n, lowest): bucket k covers the layers from the previous bucket's lowest
 * minus one down to lowest[k] (layers 0 = input .. 2N+1 = output; buckets in backward order,
 * lowest[] strictly decreasing, lowest[n-1] == 0; n == 0 turns the buckets off).  Every later
 * p3d_backward / p3d_train_fwd_bwd[_lr] then runs the weight gradients of bucket k as ONE
 * k_wgrad_multi launch as soon as its layers' dZ and BN-parameter gradients exist (right after
 * the data-gradient launch of the layer above lowest[k]) and records bucket k's event, so the
 * bucket's flat range (p3d_layer_grad_range of its layers, contiguous) is final at that event
 * and its all-reduce overlaps the rest of the backward.  p3d_stream_wait_grad makes another
 * stream wait for bucket k's event of the last backward.  p3d_grad_events(m, 1) = one bucket
 * per layer.  (--max_norm models: every event after the clip's gradient, i.e. at the end.) */
int p3d_grad_buckets(p3d_model* m, int32_t n, const int32_t* lowest);
int p3d_grad_events(p3d_model* m, int32_t enable);
int p3d_layer_grad_range(const p3d_model* m, int32_t layer, int64_t* begin, int64_t* end);
int p3d_stream_wait_grad(p3d_model* m, int32_t bucket, void* stream);

/* The data-parallel step (session.run of the train op with the gradient averaged over the
 * replicas, linear_model.py:137-145 + SURVEY 8e) in two calls around the caller's all-reduce of
 * the flat grads buffer: p3d_train_fwd_bwd_lr = p3d_train_fwd_bwd whose first backward launch
 * also forms the step's Adam alpha (lr0 * decay_rate^(global_step / decay_steps), TF1 bias
 * correction, from the device step state); p3d_adam_apply = TF1 ApplyAdam + weight re-pack with
 * that alpha, the step state (global_step, beta powers) advanced in the same launch.  Both are
 * graph-capturable (all step state on the device). */
int p3d_train_fwd_bwd_lr(p3d_model* m, const float* x, const float* t, int64_t B, float* y, float keep_prob,
                         uint64_t seed, int64_t row_offset, float lr0, float decay_steps, float decay_rate,
                         float* loss_dev, void* stream);
int p3d_adam_apply(p3d_model* m, void* stream);

/* p3d_adam_apply split by gradient bucket (p3d_grad_buckets), each part issued on the stream of
 * that bucket's all-reduce right after it: the stream waits until the last backward has issued
 * the last reader of the bucket's parameters (the data-gradient launch of its lowest layer),
 * then Adam + re-pack of the bucket's tensors; the last bucket's launch advances the step
 * state.  Every bucket exactly once per step, in bucket order on one stream; bit-identical
 * to p3d_adam_apply.  The optimizer then overlaps the rest of the backward.  max_norm models:
 * P3D_ERR_STATE (they take p3d_adam_apply). */
int p3d_adam_apply_bucket(p3d_model* m, int32_t bucket, void* stream);

/* ---------------------------------------------------------------------------------------
 * Data-parallel training with the gradient all-reduce issued by this library (the
 * reference is single-process, its step is one session.run of the train op, src/linear_model.py:
 * 230-237, with one optimizer step per batch, :137-145).  librccl is resolved at run time from
 * the library the process already uses (pass torch's librccl path; NULL = "librccl.so.1"):
 * libp3d.so has no link-time dependency on it.  The ranks build a communicator from a unique id
 * rank 0 draws and broadcasts over the caller's own channel (torch.distributed), attach it to a
 * model, and p3d_train_step_dp then runs the whole DP step -- forward, backward, the bucketed
 * all-reduce of the flat gradient on a library-owned stream overlapping the backward, TF1 Adam +
 * re-pack, step advance -- holding no object of the caller's runtime, so one HIP graph captures it
 * whole.  The reduction is the replica mean (one rank: the identity).
 * ------------------------------------------------------------------------------------- */
typedef struct p3d_comm p3d_comm;
int p3d_comm_load(const char* librccl_path);
int p3d_comm_unique_id(uint8_t* id, int64_t id_len /* >= 128 */);
int p3d_comm_create(const uint8_t* id, int64_t id_len, int32_t nranks, int32_t rank, p3d_comm** out);
int p3d_comm_destroy(p3d_comm* c);
/* in-place all-reduce of n elements (dtype P3D_DTYPE_F32 / F64; op 0 sum, 1 mean, 2 max) on `stream` */
int p3d_comm_allreduce(p3d_comm* c, void* buf, int64_t n, int32_t dtype, int32_t op, void* stream);
/* the communicator the model's data-parallel step reduces over (NULL detaches; not owned) */
int p3d_dp_attach(p3d_model* m, p3d_comm* c);
/* One data-parallel training step.  With gradient buckets (p3d_grad_buckets) bucket k's
 * all-reduce runs on the library's comm stream as soon as the backward recorded its event and its
 * TF1 Adam follows on `stream` (env P3D_DP_ADAM: 1 default; 0 one optimizer pass after the last
 * bucket; 2 each bucket's optimizer on the comm stream); without buckets one all-reduce after the
 * backward.  Arguments as p3d_train_fwd_bwd_lr.  Graph-capturable (the comm stream is forked from
 * and joined to `stream`). */
int p3d_train_step_dp(p3d_model* m, const float* x, const float* t, int64_t B, float* y, float keep_prob,
                      uint64_t seed, int64_t row_offset, float lr0, float decay_steps, float decay_rate,
                      float* loss_dev, void* stream);

/* One whole single-GPU TF1 training step (linear_model.py:225-237): p3d_train_fwd_bwd then
 * the TF1 Adam update, global_step += 1.  By default (env P3D_FUSE_ADAM=1 at p3d_create) the
 * update runs inside the batched weight-gradient launch (k_wgrad_multi: no separate optimizer
 * pass; the flat grads buffer then holds the bias and BN gradients, not dW), bit-identical to
 * the unfused sequence (tests/test_gpu_parity.py) and faster at cfg3;
 * P3D_FUSE_ADAM=0 runs k_adam_pack after the backward.
 * lr = lr0 * decay_rate^(global_step / decay_steps) on the device.  Equivalent to
 * p3d_train_fwd_bwd + p3d_adam_step_decay (which --max_norm models use internally).
 * Graph-capturable; data-parallel training uses the unfused calls around its all-reduce. */
int p3d_train_step(p3d_model* m, const float* x, const float* t, int64_t B, float* y,
                   float keep_prob, uint64_t seed, float lr0, float decay_steps, float decay_rate,
                   float* loss_dev, void* stream);

/* One TF1 ApplyAdam over all trainables (linear_model.py:137,145):
 *   alpha = lr*sqrt(1-beta2_power)/(1-beta1_power); m += (g-m)(1-b1);
 *   v += (g^2-v)(1-b2); w -= (m*alpha)/(sqrt(v)+eps)
 * then global_step += 1 and the beta powers advance.  The step state lives on the
 * device.  p3d_adam_step takes the already-decayed lr; p3d_adam_step_decay computes
 * tf.train.exponential_decay (lr0 * rate^(global_step/steps), linear_model.py:88-90)
 * on the device, so a whole training step can be captured in a HIP graph. */
int p3d_adam_step(p3d_model* m, float lr, void* stream);
int p3d_adam_step_decay(p3d_model* m, float lr0, float decay_steps, float decay_rate, void* stream);

/* Adam bookkeeping (for checkpoints): global_step and beta1/beta2 powers.  Both
 * synchronise the device (the state is device-resident). */
int p3d_get_step(const p3d_model* m, int64_t* global_step, float* beta1_power, float* beta2_power);
int p3d_set_step(p3d_model* m, int64_t global_step, float beta1_power, float beta2_power);

/* Fused MPJPE accumulation of src/predict_3dpose.py:399-430 for one batch:
 *   pred_n [B, 48] fp32 network outputs, gt_n [B, 48] fp32 normalized targets,
 *   mean96/std96 [96] fp64 (data_mean_3d / data_std_3d), dims48 [48] int32
 *   (dim_to_use_3d).  Un-normalizes both (x*std+mean, fp64, root dims = mean),
 *   takes the 17 joints [0,1,2] + dims48, and ADDS per-joint L2 sums (fp64) into
 *   joint_sum17[17]. */
int p3d_mpjpe_accum(const float* pred_n, const float* gt_n, const double* mean96,
                    const double* std96, const int32_t* dims48, int64_t B, double* joint_sum17,
                    void* stream);

/* General form (src/predict_3dpose.py:383,399-430 with FLAGS.predict_14 / FLAGS.procrustes):
 *   D = 48, n_joints = 17: the 17-joint protocol above (root joint prepended);
 *   D = 42, n_joints = 14: --predict_14 (dims = the 42 dim_to_use_3d, no root);
 *   procrustes != 0: per-frame similarity alignment of the prediction onto the target
 *   (src/procrustes.py:2-63, compute_optimal_scale=True) before the per-joint L2.
 * ADDS into joint_sum[n_joints]; if sq_sum is non-null also adds sum((pred_n - gt_n)^2)
 * over the B x D batch (the loss of src/linear_model.py:129 times B*D, fp64 sum). */
int p3d_mpjpe_accum_ex(const float* pred_n, const float* gt_n, int32_t D, const double* mean96,
                       const double* std96, const int32_t* dims, int64_t B, int32_t n_joints,
                       int32_t procrustes, double* joint_sum, double* sq_sum, void* stream);

/* rocprofv3 name of the kernel used for `what` under the model's tiling variants:
 * 0 = inference hidden layer at B <= 64, 1 = inference hidden layer at large M,
 * 2 = BN-train hidden-layer GEMM, 3 = the kernel of the last p3d_serve launch,
 * 4 = inference hidden layer at B <= 4 (weight-streaming GEMV), 5 = the kernel of the last bf16
 * hidden layer (empty before one ran), 6 = the optimizers' weight source: "packed" (W read from its
 * packed Wd copy, the TF-layout master not written) or "master".  (Measurement plumbing for bench.py.) */
int p3d_kernel_name(const p3d_model* m, int32_t what, char* out, int64_t out_len);

/* Host-binding plumbing: a DLPack v0.8 DLManagedTensor aliasing `data` (no copy; the
 * memory stays owned by its model), with a C deleter that frees only the record.  Wrap
 * it in a "dltensor" PyCapsule for torch.utils.dlpack.from_dlpack.  NULL on bad input. */
void* p3d_dlpack_alias(void* data, int32_t ndim, const int64_t* shape, int32_t device_id,
                       int32_t dtype_code, int32_t bits);

/* Live kernel timing (bench.py's roofline): while active, every kernel the model
 * launches is bracketed by a hipEvent pair.  p3d_profile_stop synchronises and writes
 * one line per kernel tag: "tag\tcount\ttotal_us\tmin_us\tmax_us\n". */
int p3d_profile_start(p3d_model* m, int32_t max_launches);
int p3d_profile_stop(p3d_model* m, char* out, int64_t out_len);

/* Host-overhead probe (bench.py's accounting of the timed region beyond the kernel): one launch
 * of an empty kernel of `grid` 256-thread workgroups on `stream`, through the same launch path as
 * the model's kernels (with the model's event pair while p3d_profile_start is active). */
int p3d_empty_launch(p3d_model* m, int32_t grid, void* stream);

/* Completion of a captured sequence without the runtime's completion signal (the reference's
 * session.run returns its fetches; LinearModel.step(isTraining=True) from numpy): p3d_host_signal
 * enqueues one small kernel that advances the model's signal counter and stores the new count into
 * a pinned word (system-scope release); it is capturable, and each replay of a graph holding it
 * signals once.  p3d_host_wait(m, count, stream) returns once the count has reached `count` -- the
 * kernels before the signal have completed and their writes to coherent host memory are visible --
 * then reports a set kernel error word as P3D_ERR_HIP (p3d_error_flags says which); it polls the
 * stream now and then, so a failed launch is reported instead of waited for.  The stream itself
 * is not synchronised.  p3d_host_alloc / p3d_host_free: coherent pinned host memory (mapped, not
 * cached on the device), where kernels' host-memory outputs must live for p3d_host_wait to cover
 * them. */
int p3d_host_signal(p3d_model* m, void* stream);
int p3d_host_wait(p3d_model* m, uint32_t count, void* stream);
void* p3d_host_alloc(int64_t bytes);
int p3d_host_free(void* p);

/* Roofline timing hook: `reps` back-to-back launches of hidden layer `layer`
 * (1 .. 2*num_layers) of the inference forward over workspace rows [0, B). */
int p3d_time_layer(p3d_model* m, int32_t layer, int64_t B, int32_t reps, void* stream);

/* ---------------------------------------------------------------------------------------
 * H3.6M data pipeline: float64 like the reference's numpy, row-major,
 * device pointers, asynchronous on `stream`.  These replace the per-sequence numpy loops of
 * the loaders; results are bit-identical to the reference.
 * A camera record is 21 float64: R row-major (9; X_cam = R (P - T)), T (3), f (2), c (2),
 * k (3), p (2) -- the tuple of src/cameras.py:92-140 (load_camera_params / load_cameras).
 * ------------------------------------------------------------------------------------- */

/* Rigid camera transforms of n points for each of C cameras into out [C, n, 3].
 * inverse = 0: world -> camera, src/cameras.py:55-72 (world_to_camera_frame; the batched
 *   form of data_utils.transform_world_to_camera, src/data_utils.py:233-257);
 * inverse = 1: camera -> world, src/cameras.py:74-90 (camera_to_world_frame).
 * P is [n, 3] shared by all cameras (in_cam_stride = 0) or [C, n, 3] (in_cam_stride = 3n). */
int p3d_cam_transform(const double* P, int64_t n, int64_t in_cam_stride, const double* cams,
                      int32_t C, int32_t inverse, double* out, void* stream);

/* Pinhole projection with radial (k1..k3) and tangential (p1, p2) distortion of n world
 * points for each of C cameras, src/cameras.py:13-53 (project_point_radial; the batched form
 * of data_utils.project_to_cameras, src/data_utils.py:339-364).  proj [C, n, 2]; depth,
 * radial, tan, r2 [C, n] are optional (NULL = not written). */
int p3d_cam_project(const double* P, int64_t n, const double* cams, int32_t C, double* proj,
                    double* depth, double* radial, double* tan, double* r2, void* stream);

/* Root-centring, src/data_utils.py:474-494 (postprocess_3d): out = poses - tile(poses[:, :3]),
 * root [F, 3] = poses[:, :3] (may be NULL).  width = 3 * joints; out must not alias poses. */
int p3d_root_center(const double* poses, int64_t F, int32_t width, double* out, double* root,
                    void* stream);

/* src/data_utils.py:260-280 (normalize_data): out [F, U] = (x[:, use] - mean[use]) / std[use]
 * from x [F, D]; out_dtype P3D_DTYPE_F64, or P3D_DTYPE_F32 (the float64 result rounded, as
 * feeding it to the model's float32 placeholders does). */
int p3d_normalize(const double* x, int64_t F, int32_t D, const double* mean, const double* stdv,
                  const int32_t* dims_to_use, int32_t U, void* out, int32_t out_dtype, void* stream);

/* src/data_utils.py:283-311 (unNormalizeData): scatter xn [F, U] (P3D_DTYPE_F32 or F64; the
 * reference rounds it to float32) into zeros [F, D], then out = that * std + mean (float64).
 * D <= 256. */
int p3d_unnormalize(const void* xn, int32_t in_dtype, int64_t F, int32_t U, const double* mean,
                    const double* stdv, const int32_t* dims_to_use, int32_t D, double* out,
                    void* stream);

/* src/openpose_3dpose_sandbox.py:347-356 per call (normalize_data of the mapped 2D rows, the
 * float32 placeholder cast, model.step at is_training False / keep 1, unNormalizeData): raw
 * [B, D2] float64 -> out [B, D3] float64.  U2 / U3 must equal the model's input / output size.
 * One launch where the batch <= 4 persistent chain runs, else p3d_normalize + p3d_forward_ex +
 * p3d_unnormalize; the same bits as those three calls either way.  Float32 models. */
int p3d_lift(p3d_model* m, const double* raw, int64_t B, int32_t D2, const double* mean2, const double* std2,
             const int32_t* use2, int32_t U2, const double* mean3, const double* std3, const int32_t* use3,
             int32_t U3, int32_t D3, double* out, void* stream);
/* p3d_lift that returns once out holds the results (pinned host rows; the per-frame call of
 * src/openpose_3dpose_sandbox.py:353-356): on the one-launch chain form the launch's output
 * workgroups store a completion word the host waits on, as p3d_serve_mse_sync; on the three-step
 * form the stream is synchronised.  Not capturable. */
int p3d_lift_sync(p3d_model* m, const double* raw, int64_t B, int32_t D2, const double* mean2, const double* std2,
                  const int32_t* use2, int32_t U2, const double* mean3, const double* std3, const int32_t* use3,
                  int32_t U3, int32_t D3, double* out, void* stream);

/* np.mean / np.std (population) over axis 0 of x [F, D], D <= 256 -- the statistics of
 * src/data_utils.py:210-211 (normalization_stats).  Deterministic two-level column sums;
 * `work` must hold p3d_moments_workspace(F, D) bytes of device memory. */
int64_t p3d_moments_workspace(int64_t F, int32_t D);
int p3d_moments(const double* x, int64_t F, int32_t D, double* mean, double* stdv, void* work,
                int64_t work_bytes, void* stream);

/* CRC-32C (Castagnoli) of host memory -- TF tensor-bundle checksums (checkpoint interop,
 * src/predict_3dpose.py:165-181,328 save/restore through tf.train.Saver).  crc = 0 starts a
 * buffer; pass a previous result to continue it.  Host only, no device work. */
uint32_t p3d_crc32c(const void* data, int64_t n, uint32_t crc);

#ifdef __cplusplus
}
#endif
#endif /* P3D_H_ */

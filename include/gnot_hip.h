/* gnot_hip.h — C ABI of the MI355X-native GNOT core (libgnot_hip.so).
 *
 * Drop-in boundary for the reference's hot path: `GNOT.forward` (reference model.py:154-173) and the
 * backward that `loss.backward()` (main.py:102) runs through it.  The reference is pure PyTorch and
 * has no FFI; these entry points are what its `GNOT` module binds in our host mirror
 * (gnot-replication_amd/gnot_amd/model.py, via ctypes — see INTEGRATION.md):
 *
 *   reference                                   replaced by
 *   GNOT.__init__(...)            model.py:143   gnot_plan_create (same 12 constructor arguments)
 *   nn.Linear parameters          model.py:9-14, 43-51  gnot_plan_bind_params (state_dict order)
 *   padding / batching       utils.py:3-4, main.py:60-89  gnot_plan_set_batch (packed offsets)
 *   GNOT.forward                  model.py:154-173  gnot_forward
 *   autograd backward             main.py:102    gnot_backward
 *
 * Conventions: plain pointers and sizes only, no torch types.  All device memory (inputs, outputs,
 * parameters, the workspace) is allocated and owned by the caller; the library never allocates
 * device memory.  Every compute entry point is asynchronous and stream-ordered on the hipStream_t
 * it is given (pass NULL for the default stream), launches kernels only (graph-capturable) and
 * returns 0 on success or a negative GNOT_E* code; gnot_last_error() then describes the failure.
 */
#ifndef GNOT_HIP_H
#define GNOT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gnot_plan gnot_plan; /* opaque */

/* GNOT constructor arguments, reference model.py:143 (positional order of main.py:44).
 * n_attn_hidden_dim, n_mlp_hidden_dim and n_input_hidden_dim must be equal (the reference's
 * residual adds, model.py:131/137, require it); any d and n_head with d/n_head up to 256 whose internal width
 * is at most 1024: a head width that is not a multiple of 4 runs on heads padded to one (n_head x that many
 * internal columns), and the internal width is the next multiple of 16 up to 192, 256 (heads of 16 / 32 / 64 /
 * 128 / 256, unpadded), the next multiple of 64 up to 512, else the next multiple of 128 (heads dividing 64),
 * with exact-zero pad columns; parameters, gradients and outputs keep d. */
typedef struct gnot_config {
  int input_dim;
  int theta_dim;
  int input_func_dim;
  int out_dim;
  int n_attn_layers;
  int n_attn_hidden_dim;
  int n_mlp_num_layers;
  int n_mlp_hidden_dim;
  int n_input_hidden_dim;
  int n_expert;
  int n_head;
  int n_input_functions;
} gnot_config;

enum {
  GNOT_OK = 0,
  GNOT_E_INVALID = -1,     /* bad argument / unsupported configuration */
  GNOT_E_HIP = -2,         /* a HIP runtime call failed */
  GNOT_E_STATE = -3,       /* call out of order (e.g. forward before bind) */
  GNOT_E_WORKSPACE = -4    /* workspace missing or too small */
};

/* Plan lifetime. */
int gnot_plan_create(const gnot_config* cfg, gnot_plan** out);
void gnot_plan_destroy(gnot_plan* plan);

/* Linears in reference state_dict order (named_parameters() order of model.py's GNOT).
 * dims[2*i] = out_features, dims[2*i+1] = in_features. */
int gnot_plan_num_linears(const gnot_plan* plan);
int gnot_plan_linear_dims(const gnot_plan* plan, int32_t* dims);

/* Device pointers of every Linear's weight [out, in] (row-major) and bias [out], fp32, in the order
 * above.  Pointers must stay valid (parameters are updated in place by the optimizer). */
int gnot_plan_bind_params(gnot_plan* plan, const float* const* weights, const float* const* biases);

/* Batch geometry.  x_off: host array [B+1] of point offsets (packed, no padding: sample b owns rows
 * x_off[b] .. x_off[b+1]-1); fn_off: host array [n_input_functions * (B+1)] of the same for every
 * input function.  A zero-padded batch (main.py:60-82) is simply x_off = {0, N, 2N, ...}.
 * training != 0 keeps the activations the backward needs.
 * Limits: fewer than 2^29 points per plan (query points, and points of each input function: the
 * kernels' job tables hold 32-bit point indices; their buffer resources are based per workgroup or per
 * split-K range, so no activation array size bounds a plan).  GNOT_E_INVALID beyond it; the real bound
 * is the workspace (gnot_plan_workspace_bytes) against the device memory. */
int gnot_plan_set_batch(gnot_plan* plan, int B, const int64_t* x_off, const int64_t* fn_off, int training);

/* MoE activation recompute (off by default): training keeps only each MoE call's input and the
 * backward re-runs that call's expert forward (model.py:128/134's ffn1/ffn2 experts) into one shared
 * save buffer just before its chain backward -- the E*nl*P*d saved pre-activations exist once instead
 * of once per MoE call (2 per block), at the cost of one more MoE forward per call.  Changing it
 * invalidates the batch: call gnot_plan_set_batch (and bind) again.  No reference counterpart (a
 * memory option of this library; torch.utils.checkpoint is the analogue). */
int gnot_plan_set_moe_recompute(gnot_plan* plan, int on);

/* Arithmetic mode of the MFMA kernels up to hidden width 256 (MLP chains, attention projections, weight
 * gradients): bf16 == 0 (default) runs them as bf16x6 -- three exact bf16 pieces per fp32 operand, six
 * products, fp32-level results (north_star's 1e-4 bar; the d <= 192 chain backward-data on exact fp32
 * MFMA); bf16 != 0 runs ONE round-to-nearest-even bf16 piece per operand with fp32 accumulation
 * (BASELINE configs[2]'s bf16 training, configs[1]'s "fp32 and bf16"; north_star's 1e-2 bar), and at
 * d = 256 the soft-MoE expert chains keep their training saves, dZ and Linear inputs as bf16 rows (the
 * MoE weight gradients read them directly).  Parameters, the other activations, states, gradients and
 * the attention contractions stay fp32 either way; above d = 256 the mode changes nothing.  Changing it
 * invalidates the batch (set_batch + bind again). */
int gnot_plan_set_precision(gnot_plan* plan, int bf16);

/* Input gradients (off by default).  The reference's autograd also differentiates w.r.t. x, theta and
 * the input functions when they require grad (model.py:154-173: x feeds the gating MLP and, through
 * torch.cat with the broadcast theta, the query encoder; the input functions feed their encoder
 * MLPs).  With on != 0 the backward also runs the first Linear's backward-data of those four encoders;
 * gnot_input_grads then writes dx [P, input_dim], dtheta [B, theta_dim] (sums over each sample's
 * points) and dfns[i] [Q_i, input_func_dim] (any pointer may be null: skipped).  Training plans only.
 * With point sharding dx holds this rank's rows, and dtheta / dfns -- one partial per rank, theta being
 * broadcast over all points and the input functions replicated -- are summed over the ranks through the
 * plan's gnot_comm (every rank must call gnot_input_grads).  Changing it invalidates the batch
 * (set_batch + bind again). */
int gnot_plan_set_input_grads(gnot_plan* plan, int on);
int gnot_input_grads(gnot_plan* plan, float* dx, float* dtheta, float* const* dfns, void* stream);

/* Workspace: bytes needed for the current config + batch; bind a device buffer of at least that
 * size (256-byte aligned).  Binding uploads the plan's small device tables: gnot_plan_bind_workspace
 * synchronously; gnot_plan_bind_workspace_async as one copy from pinned staging ordered on `stream`
 * (no host wait -- a per-batch geometry change, main.py:41's shuffled variable-size meshes, costs the
 * host planning (~0.1-0.3 ms) and that copy only).  Either replaces the reference's per-batch
 * padding/mask set-up, main.py:60-82. */
size_t gnot_plan_workspace_bytes(const gnot_plan* plan);
int gnot_plan_bind_workspace(gnot_plan* plan, void* workspace, size_t bytes);
int gnot_plan_bind_workspace_async(gnot_plan* plan, void* workspace, size_t bytes, void* stream);

/* Parameter-gradient arena inside the workspace: offsets (in floats) of every Linear's weight
 * gradient and bias gradient, grad_off[2*i] / grad_off[2*i+1]. */
int gnot_plan_grad_offsets(const gnot_plan* plan, int64_t* grad_off);

/* Re-pack the bound parameters into the kernels' MFMA operand images (call after every optimizer
 * step, before gnot_forward). */
int gnot_pack_weights(gnot_plan* plan, void* stream);

/* Forward (reference GNOT.forward, model.py:154-173).
 * x [P, input_dim], theta [B, theta_dim], fns[i] [Q_i, input_func_dim] (packed, device, fp32,
 * contiguous); out [P, out_dim]. */
int gnot_forward(gnot_plan* plan, const float* x, const float* theta, const float* const* fns,
                 float* out, void* stream);

/* Backward of the last gnot_forward: dout [P, out_dim] -> every parameter gradient, written
 * (overwritten) into the gradient arena. */
int gnot_backward(gnot_plan* plan, const float* dout, void* stream);

/* ---------------------------------------------------------------- point sharding (multi-GPU)
 * One process per GPU.  Every sample b of a batch is split over `world` ranks in contiguous point
 * ranges: rank r owns global points [floor(r*N_b/world), floor((r+1)*N_b/world)) (gnot_shard_range).
 * Everything per point stays local (gating, encoders, projections, MoE chains, residuals); the
 * reference's attention needs two exchanges:
 *   - the self-attention states S = sum k^T v, z = sum k (model.py:98-100), and in the backward
 *     dS, dz, are sums over ALL points of a sample: partial states are all-reduced (sum);
 *   - the head-major "scramble" of model.py:81/103-104 maps output token n' to flat rows
 *     n'*H .. n'*H+H-1 of [H, N, dh], i.e. to ALL points of a head range: the apply pass output is
 *     exchanged all-to-all (and the gradient back in the backward).
 * The input-function branch of cross attention is replicated on every rank; its backward needs no
 * exchange (every gradient downstream of dS is linear in it, so the per-rank partials add up in the
 * caller's gradient all-reduce).  The caller sums the parameter gradients over ranks.
 * The collectives are caller-provided callbacks (RCCL through torch.distributed in gnot_amd); they
 * are invoked synchronously from gnot_forward / gnot_backward and must be ordered on `stream`. */
typedef struct gnot_comm {
  void* user;
  /* in-place sum over ranks of `count` floats */
  int (*allreduce_sum)(void* user, float* buf, int64_t count, void* stream);
  /* all-to-all-v: send_counts[t] floats to rank t (packed in rank order in `send`), receive
   * recv_counts[s] floats from rank s (packed in rank order into `recv`) */
  int (*alltoallv)(void* user, const float* send, const int64_t* send_counts, float* recv,
                   const int64_t* recv_counts, void* stream);
} gnot_comm;

/* Gradient all-reduce overlapped with the backward (data-parallel training over ranks: sample-DP, or the
 * parameter gradients of a point-sharded batch).  With comm != NULL, gnot_backward sums every weight-
 * gradient group's contiguous (dW, db) ranges of the gradient arena over the ranks (comm->allreduce_sum,
 * in place) on a stream of its own as soon as that group's kernels have written them, and joins that
 * stream into `stream` before it returns -- the arena then holds the rank sums.  NULL switches it off
 * (the caller reduces the arena itself).  `comm` is copied; only allreduce_sum is used.  No reference
 * counterpart (main.py:27 is single-device); SURVEY.md section 5 "weight-grad all-reduce overlapped with
 * backward". */
int gnot_plan_set_grad_comm(gnot_plan* plan, const gnot_comm* comm);

/* Declare the rank's shard of the next batch: n_global[b] = points of sample b over all ranks.
 * Call before gnot_plan_set_batch, whose x_off then gives the LOCAL slices (validated against
 * gnot_shard_range).  world == 1 (or comm == NULL) switches sharding off.  `comm` is copied.
 * Padded hidden widths (see gnot_config) shard too: the exchanges move the real width's rows. */
int gnot_plan_set_shard(gnot_plan* plan, int rank, int world, int B, const int64_t* n_global, const gnot_comm* comm);

/* Host-only helpers (no GPU): the canonical point range of a rank, and the rank's side of the
 * scramble all-to-all.  Segments are rows of 4 int64 {dir, local_off, buf_off, len} in floats:
 * dir 0 copies local head-major apply output -> send buffer, dir 1 copies receive buffer -> local
 * token-order rows.  *nseg returns the number of segments (at most `cap` are written). */
int gnot_shard_range(int64_t n, int rank, int world, int64_t* lo, int64_t* hi);
int gnot_shard_exchange(int B, const int64_t* n_global, int n_head, int head_dim, int rank, int world,
                        int64_t* send_counts, int64_t* recv_counts, int64_t* segs, int64_t cap, int64_t* nseg);

/* ---------------------------------------------------------------- the training step around the path
 * (stateless, stream-ordered, no allocation)
 *
 * RelL2Loss (reference loss.py:14-23, the dgl SumPooling of main.py:87-98 as packed segment sums):
 * pred/tgt [rows, C] fp32 packed by the device offsets off_dev[B+1] (off_host = the same on the host,
 * for sizing); writes the scalar loss = mean over (sample, channel) of sqrt(sum (p-t)^2 / sum t^2)
 * to *loss (device) and, if dpred != NULL, d loss / d pred.  work: device scratch of
 * gnot_rel_l2_work_floats(off_host, B, C) floats.  Deterministic (fixed-order reductions). */
size_t gnot_rel_l2_work_floats(const int64_t* off_host, int B, int C);
int gnot_rel_l2_loss(const float* pred, const float* tgt, const int64_t* off_dev, const int64_t* off_host, int B,
                     int C, float* work, float* loss, float* dpred, void* stream);

/* One torch.optim.AdamW step (main.py:51) over flat fp32 arrays of n elements (param, grad, exp_avg,
 * exp_avg_sq), in torch's operation order.  hyper: DEVICE array of 8 floats {lr, beta1, beta2, eps,
 * weight_decay, 1 - beta1^t, 1 - beta2^t, grad_scale}, so a captured graph picks up the schedule the
 * host writes there (OneCycleLR changes lr and beta1, main.py:52). */
int gnot_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, const float* hyper,
                    void* stream);

/* Live kernel timing for the bench's roofline: while enabled, every launch of kernel class `kind`
 * ("moe_fwd" fused expert chains forward, "moe_bwd" their backward, "wgrad" weight-gradient GEMMs;
 * "" disables) is bracketed by hipEvents on its stream.  gnot_profile_read synchronizes on those
 * events and returns the summed device time, the launch count and the algorithmic FLOPs of those
 * launches, then resets the counters. */
int gnot_profile_enable(gnot_plan* plan, const char* kind);
int gnot_profile_read(gnot_plan* plan, double* ms_total, int64_t* launches, double* flops_total);

/* Debug/test hook: device pointer + row stride (floats) of a named intermediate buffer
 * ("scores", "query0", "out_h0", ...); returns GNOT_E_INVALID for unknown names. */
int gnot_debug_buffer(const gnot_plan* plan, const char* name, float** ptr, int64_t* ld);

const char* gnot_last_error(void);
const char* gnot_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GNOT_HIP_H */

/* C ABI of libcsa_hip.so — MI355X (gfx950) kernels for the CSA-Trans attention hot path.
 *
 * Every entry point replaces one piece of the reference's PyTorch-eager hot path
 * (paths relative to the reference repo saeyoon17/Code-Structure-Aware-Transformer):
 *
 *   csa_sbm_fwd        module/sbm_attn.py:32-66   SBMAttention.forward (+ STE.py:10-15 sampling)
 *                      module/sbm_attn.py:77-87   FullAttention.forward   (flags & CSA_FLAG_DENSE)
 *   csa_sbm_maps       module/sbm_attn.py:62,57   the returned `attn` / `graph` maps (optional)
 *   csa_sbm_bwd        autograd of the above incl. STE.py:17-19 (hardtanh straight-through)
 *   csa_dense_attn_fwd/_bwd  module/sbm_attn.py:69-87 FullAttention (csa_sbm_* with CSA_FLAG_DENSE)
 *   csa_ste_sample     module/STE.py:10-15        standalone sampler (bit-exact test surface)
 *   csa_rel_attn_fwd   module/disentangled_attn.py:44-65 DisentangledAttn.rel_attn
 *   csa_rel_attn_bwd   autograd of rel_attn (gather backward = deterministic scatter-add)
 *   csa_adamw_step     script/optimizer.py:49-106 AdamW.step (all parameters in one launch)
 *   csa_gen_logsoftmax_fwd/_bwd  module/components.py:95-102 Generator: log(softmax(dropout(logits)))
 *   csa_bias_grad      Linear bias gradient (column sums of dY) of the encoder/decoder glue
 *   csa_layernorm_fwd/_bwd  nn.LayerNorm of the encoder glue (module/components.py SublayerConnection)
 *   csa_ast_relations  my_ast.py:198-273 + dataset/base_data_set.py:33-36 (host C++, no GPU)
 *
 * Conventions (all entry points):
 *   - fp32 data; device pointers; sizes and strides are int64 ELEMENT counts; the last
 *     (feature) dimension is always contiguous, so a (B,H,N,d) operand is described by its
 *     b/h/n strides (the non-contiguous split_heads view of sbm_attn.py:137-140 is accepted).
 *   - The caller allocates every output, the saved state and the workspace (sizes from the
 *     *_bytes() queries), and owns every stream and event: the library never allocates, never
 *     creates a stream or event, never synchronises the host and never throws. It enqueues
 *     everything on `stream` (stream-ordered, graph-capturable, re-entrant) on the device that
 *     stream belongs to, whatever the calling thread's current device is. Its only state is a
 *     per-thread last-error string and a cache of which kernels already had their (idempotent)
 *     dynamic-LDS attribute raised on which device. Results are deterministic for fixed inputs
 *     (integer atomics only; float reductions use fixed-order partial slabs), whatever the
 *     backward schedule.
 *   - Errors: CSA_INVALID_ARG (null/inconsistent arguments), CSA_UNSUPPORTED_SHAPE (outside
 *     the compiled instantiations, see csa_sbm_supported), CSA_LAUNCH_FAILED (HIP error; text
 *     via csa_last_error_str on the calling thread).
 */
#ifndef CSA_HIP_H
#define CSA_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CSA_ABI_VERSION 9

typedef enum csa_status {
  CSA_OK = 0,
  CSA_INVALID_ARG = 1,
  CSA_UNSUPPORTED_SHAPE = 2,
  CSA_LAUNCH_FAILED = 3
} csa_status;

/* flags */
#define CSA_FLAG_DENSE 1u /* FullAttention (graph == 1, no cluster projection, no sampling) */
/* ABI v6: the caller will not run csa_sbm_bwd on this forward's state (inference / no_grad): the state omits the
 * projection MLP's saved activations, which only the backward reads (csa_sbm_state_bytes shrinks, the forward
 * skips their stores); csa_sbm_bwd rejects such a state. */
#define CSA_FLAG_FWD_ONLY 2u
/* ABI v8: the call pair runs with dtype CSA_DTYPE_BF16. csa_sbm_bwd_workspace_bytes then omits the fp32 backward's
 * ds / G tile handoff (bf16 mode recomputes S and dP on the query side instead), which is O(B*H*N*M) floats: with
 * clusters two (B,H,NQB,NKB,32,32) fp32 planes (at B=16, H=8, N=M=1024: 1.07 GB), without (DENSE) one plane.
 * csa_sbm_bwd lays a bf16 call's workspace out without the handoff whether or not the flag is set (a buffer sized
 * without it is merely larger); the flag on an fp32 call is CSA_INVALID_ARG. csa_sbm_state_bytes ignores it. */
#define CSA_FLAG_BF16_WS 4u

/* ABI v5: schedule of an attention backward's two halves (csa_rel_attn_bwd_args .schedule). The key half
 * may run on a caller-owned side stream beside the query half, forked from and joined back into `stream`
 * with two caller-owned events (capture-safe); outputs are bitwise the same either way. AUTO uses the side
 * stream when the query half's grid leaves a partial last round of workgroups on the device (side_stream
 * must be set, else it runs in order). ABI v6, csa_sbm_bwd: the projection backward's key-block items (they
 * need only the key half's dT) run on the side stream beside the query half (k_attn_bwd_qg) and its query-
 * block items on CSA_SCHED_CONCURRENT only (AUTO runs in order: faster at the headline shape, measured).
 * Bitwise-identical results either way. */
#define CSA_SCHED_AUTO 0u
#define CSA_SCHED_IN_ORDER 1u
#define CSA_SCHED_CONCURRENT 2u /* needs side_stream / side_fork / side_join */

/* operand precision of the N^2 attention contractions (dtype field of the args structs). Storage is
 * fp32 either way. CSA_DTYPE_F32 is the reference's precision (sbm_attn.py:120-126 forces fp32) and
 * the parity mode (rtol 1e-4 / atol 1e-5). CSA_DTYPE_BF16 rounds the operands of QK^T, dX V^T, PV, dQ,
 * dK, dV, of the projection MLP (three d x d layers, forward and backward chains and weight-gradient
 * products) and of sigmoid(. C^T) and its backward (SBM), and of the CSE's c2c, PV and their gradients
 * to bf16 for v_mfma_f32_32x32x16_bf16 (fp32 accumulation; north_star tolerance 2e-2). T = Kh S^T, expA,
 * the sampling threshold and every softmax / normalisation / elementwise step stay fp32. Inside the saved
 * state (opaque, csa_sbm_state_bytes unchanged) bf16 mode keeps the projection MLP's activations as bf16,
 * rounded as its MFMAs round them; the backward of the same call pair reads them back. */
#define CSA_DTYPE_F32 0
#define CSA_DTYPE_BF16 1

/* Optional per-stage timing: caller-created hipEvent_t handles; when start[s] and stop[s] are
 * non-NULL the library records them on `stream` around stage s (no library-side state). */
enum {
  CSA_STAGE_PREP = 0,       /* cluster softmax + fragment prep */
  CSA_STAGE_PROJ_FWD = 1,   /* k_proj_fwd */
  CSA_STAGE_ATTN_FWD = 2,   /* k_attn_fwd */
  CSA_STAGE_ATTN_BWD_Q = 3, /* k_attn_bwd_qg (bf16 mode: k_attn_bwd_qr) */
  CSA_STAGE_ATTN_BWD_KV = 4,/* k_attn_bwd_kv */
  CSA_STAGE_PROJ_BWD = 5,   /* k_proj_bwd (concurrent schedule: its query-block items only) */
  CSA_STAGE_REDUCE = 6,     /* slab reduction + cluster grad */
  CSA_STAGE_PROJ_BWD_K = 7, /* concurrent schedule: k_proj_bwd's key-block items, on the side stream */
  CSA_STAGE_ATTN_ROWPREP = 8, /* ABI v7: k_attn_rowprep, timed apart from k_attn_bwd_kv */
  CSA_STAGE_COUNT = 9
};
typedef struct csa_prof {
  void* start[CSA_STAGE_COUNT];
  void* stop[CSA_STAGE_COUNT];
} csa_prof;
/* ABI v9: the same profiling struct (slots 0..5) around the CSE relation attention's stages (d_k = 64 fused path):
 * csa_rel_attn_args.prof / csa_rel_attn_bwd_args.prof */
enum {
  CSA_REL_STAGE_LOGITS = 0, /* k_rel_logits + k_rel_prep (relation logits, code planes) */
  CSA_REL_STAGE_FWD = 1,    /* k_rel_fwd_f */
  CSA_REL_STAGE_QSTAT = 2,  /* k_rel_qstat (row statistics for the key side) */
  CSA_REL_STAGE_BWD_K = 3,  /* k_rel_bwd_kh (fp32) / k_rel_bwd_kf (bf16) */
  CSA_REL_STAGE_BWD_Q = 4,  /* k_rel_bwd_qg (fp32) / k_rel_bwd_qf (bf16) */
  CSA_REL_STAGE_LGRAD = 5   /* k_rel_lgrad + k_sum_splits2 (dlq, dlk) */
};

typedef struct csa_sbm_fwd_args {
  int64_t B, H, N, M, d, k; /* batch, heads, queries, keys, head_dim, clusters (k ignored if DENSE) */
  const float* Q; int64_t q_sb, q_sh, q_sn; /* (B,H,N,d) */
  const float* K; int64_t k_sb, k_sh, k_sn; /* (B,H,M,d) */
  const float* V; int64_t v_sb, v_sh, v_sn; /* (B,H,M,d) */
  const float* key_mask; int64_t mask_sb;   /* (B,M) 1.0 = padded key (sbm_attn.py:61); may be NULL */
  const float* cluster_w;                   /* layer.weight (H*k, d) contiguous (sbm_attn.py:19) */
  const float* proj_w[3]; const float* proj_b[3]; /* proj.0/.3/.6 weight (d,d) and bias (d) */
  const float* uniforms;      /* (B,H,N,M) contiguous host-supplied draws, or NULL = Philox */
  uint64_t seed, offset;      /* Philox key / counter offset (sampling + dropout) */
  float attn_dropout;         /* drop_attn p (0 in eval) — sbm_attn.py:14,63 */
  float proj_dropout;         /* proj Dropout p (0 in eval) — sbm_attn.py:24,27 */
  uint32_t flags;
  uint32_t dtype;             /* CSA_DTYPE_F32 or CSA_DTYPE_BF16 */
  float* X;                   /* out (B,H,N,d), strides x_* below */
  float* sparsity;            /* out (H,) head-wise sparsity (sbm_attn.py:64); NULL if DENSE */
  void* state;                /* csa_sbm_state_bytes(): saved for backward and csa_sbm_maps */
  const csa_prof* prof;       /* optional stage timing (NULL = off) */
  /* ABI v3: element strides of X; all three 0 = (B,H,N,d) contiguous. d stays contiguous; like
   * Q/K/V, X must be 16-byte aligned with strides multiple of 4 elements. A (B,N,H,d) buffer read
   * as (B,H,N,d) makes combine_heads (sbm_attn.py:143-146) a free view. */
  int64_t x_sb, x_sh, x_sn;
} csa_sbm_fwd_args;

typedef struct csa_sbm_bwd_args {
  const csa_sbm_fwd_args* fwd; /* the forward's arguments (same inputs and the filled state) */
  const float* dX;             /* (B,H,N,d), strides dx_* below */
  const float* dsparsity;      /* (H,) or NULL */
  const float* dgraph;         /* (B,H,N,M) grad of the returned graph map, or NULL */
  float* dQ; float* dK; float* dV; /* out (B,H,N|M,d), strides dq_* / dk_* / dv_* below */
  float* dcluster_w;           /* out (H*k, d); NULL if DENSE */
  float* dproj_w[3]; float* dproj_b[3]; /* out; NULL if DENSE */
  void* workspace;             /* csa_sbm_bwd_workspace_bytes(); required (ABI v6: also for DENSE) */
  const csa_prof* prof;        /* optional stage timing (NULL = off) */
  /* ABI v3: element strides (b, h, row) of dX, dQ, dK, dV; a zero triple = contiguous. E.g. dQ/dK/dV
   * as the three head-major views of one packed (B,N,3,H,d) gradient of a fused QKV projection. */
  int64_t dx_sb, dx_sh, dx_sn, dq_sb, dq_sh, dq_sn, dk_sb, dk_sh, dk_sn, dv_sb, dv_sh, dv_sn;
  /* ABI v4: (B,H,N,M) contiguous upstream gradient of the returned attn map (sbm_attn.py:62, the tensor the
   * reference returns), or NULL. */
  const float* dattn;
  /* ABI v5: CSA_SCHED_* and the caller's side lane: a hipStream_t of the same device as `stream` and two
   * hipEvent_t (hipEventDisableTiming) used only between this call's fork and join. NULL = in order. */
  uint32_t schedule;
  void* side_stream; void* side_fork; void* side_join;
} csa_sbm_bwd_args;

int csa_abi_version(void);
/* sha256 (hex) of the csrc/ sources + headers and this header the library was built from
 * (csa_amd/build.py:source_hash); lets a caller prove the loaded binary matches its source tree. */
const char* csa_source_hash(void);
const char* csa_status_str(csa_status s);
const char* csa_last_error_str(void);
/* 1 if (d, k, flags) is a compiled instantiation */
int csa_sbm_supported(int64_t d, int64_t k, uint32_t flags);
size_t csa_sbm_state_bytes(int64_t B, int64_t H, int64_t N, int64_t M, int64_t d, int64_t k, uint32_t flags);
size_t csa_sbm_bwd_workspace_bytes(int64_t B, int64_t H, int64_t N, int64_t M, int64_t d, int64_t k, uint32_t flags);

csa_status csa_sbm_fwd(const csa_sbm_fwd_args* a, void* stream);
/* Materialise attn (B,H,N,M) and/or graph (B,H,N,M) fp32 maps from a completed forward. */
csa_status csa_sbm_maps(const csa_sbm_fwd_args* a, float* graph, float* attn, void* stream);
csa_status csa_sbm_bwd(const csa_sbm_bwd_args* a, void* stream);
/* FullAttention (module/sbm_attn.py:77-87): the two calls above with CSA_FLAG_DENSE forced (k, cluster_w,
 * proj_*, uniforms and sparsity ignored). */
csa_status csa_dense_attn_fwd(const csa_sbm_fwd_args* a, void* stream);
csa_status csa_dense_attn_bwd(const csa_sbm_bwd_args* a, void* stream);

/* STE.py:10-15 as A = (u < clamp(p, lo, hi)); n elements, contiguous. */
csa_status csa_ste_sample(const float* p, const float* u, float* A, int64_t n, float lo, float hi, void* stream);
/* STE.py:17-19: gin = hardtanh(A * gout). */
csa_status csa_ste_backward(const float* A, const float* gout, float* gin, int64_t n, void* stream);

/* ---- CSE disentangled relation attention (module/disentangled_attn.py:44-65) ---- */
typedef struct csa_rel_attn_args {
  int64_t B, H, N, L, d; /* H must be 8 (4 parent + 4 sibling heads, disentangled_attn.py:29-33) */
  const float* q; int64_t q_sb, q_sh, q_sn;
  const float* k; int64_t k_sb, k_sh, k_sn;
  const float* v; int64_t v_sb, v_sh, v_sn;
  const float* lq; const float* lk; /* (H, L, d) contiguous (batch dim 1 dropped) */
  const uint8_t* rel;  int64_t rel_sb, rel_sh;  /* (B,*,N,N) relation index < L; head stride may be 0 */
  const uint8_t* mask; int64_t mask_sb, mask_sh;/* (B,*,N,N) 1 = masked (-1e9); head stride may be 0 */
  int64_t rel_head_group; /* heads [0,g) read plane 0, heads [g,H) plane 1 (CSE: 4); 0 = use rel_sh */
  uint32_t dtype;          /* CSA_DTYPE_F32 or CSA_DTYPE_BF16 (bf16: d = 64 only) */
  float* out;          /* (B,H,N,d), strides o_* below */
  float* row_stats;    /* (B,H,N,2) saved (row max, 1/row sum) for backward; kept separate because
                          fully masked rows sit at -1e9 where max + log(sum) is not representable */
  void* state;         /* csa_rel_attn_state_bytes(): relation logits q.lk^T, k.lq^T, kept for backward */
  /* ABI v3: element strides (b, h, row) of out; zero triple = (B,H,N,d) contiguous. Non-contiguous
   * layouts need d = 64 (the fused path); 16-byte aligned, strides multiple of 4 elements. */
  int64_t o_sb, o_sh, o_sn;
  const csa_prof* prof; /* ABI v9: optional stage timing (CSA_REL_STAGE_*; NULL = off) */
} csa_rel_attn_args;

typedef struct csa_rel_attn_bwd_args {
  const csa_rel_attn_args* fwd;
  const float* dout;   /* (B,H,N,d), strides do_* below */
  float* dq; float* dk; float* dv; /* (B,H,N,d), strides dq_* / dk_* / dv_* below */
  float* dlq; float* dlk;          /* (H,L,d) */
  void* workspace;
  /* ABI v3: element strides (b, h, row); a zero triple = contiguous; non-contiguous needs d = 64 */
  int64_t do_sb, do_sh, do_sn, dq_sb, dq_sh, dq_sn, dk_sb, dk_sh, dk_sn, dv_sb, dv_sh, dv_sn;
  /* ABI v5: schedule and side lane as in csa_sbm_bwd_args; only the d_k = 64 fused path uses them, and of it
   * only bf16 mode (CSA_DTYPE_BF16): the fp32 fused backward hands the key half's g tiles to the query half
   * (k_rel_bwd_kh -> k_rel_bwd_qg) and runs in order whatever the schedule */
  uint32_t schedule;
  void* side_stream; void* side_fork; void* side_join;
  const csa_prof* prof; /* ABI v9: optional stage timing (CSA_REL_STAGE_*; NULL = off) */
} csa_rel_attn_bwd_args;

size_t csa_rel_attn_state_bytes(int64_t B, int64_t H, int64_t N, int64_t L, int64_t d);
size_t csa_rel_attn_bwd_workspace_bytes(int64_t B, int64_t H, int64_t N, int64_t L, int64_t d);
csa_status csa_rel_attn_fwd(const csa_rel_attn_args* a, void* stream);
csa_status csa_rel_attn_bwd(const csa_rel_attn_bwd_args* a, void* stream);

/* ---- AdamW step (script/optimizer.py:49-106; script/train.py:80 uses correct_bias=False) ----
 * Per element, in the reference's op order:
 *   m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;  p += -step_size * m / (sqrt(v) + eps);
 *   p += -decay * p  (decay = lr * weight_decay, applied after the Adam update as in the reference)
 * step_size = lr, or lr * sqrt(1 - b2^t) / (1 - b1^t) with correct_bias (computed by the caller).
 * torch.amp GradScaler semantics without a host sync: when found_inf is non-NULL and *found_inf != 0
 * the whole step is skipped (nothing written); when grad_scale is non-NULL each gradient is used as
 * g * (float)(1.0 / (double)*grad_scale), GradScaler.unscale_'s inv_scale (grads are not written back). */
#define CSA_ADAMW_CHUNK 4096
typedef struct csa_adamw_tensor { /* one parameter tensor, contiguous fp32 (device pointers) */
  float* param; const float* grad; float* exp_avg; float* exp_avg_sq; int64_t numel;
} csa_adamw_tensor;

typedef struct csa_adamw_args {
  const csa_adamw_tensor* tensors; /* device array, ntensors entries */
  const int32_t* chunk_tensor;     /* device (nchunks): tensor of each CSA_ADAMW_CHUNK-element chunk */
  const int64_t* chunk_start;      /* device (ntensors): first chunk of each tensor */
  int64_t ntensors, nchunks;
  float beta1, beta2, one_minus_beta1, one_minus_beta2; /* 1-b as the reference's fp32 alpha/value */
  float eps, step_size, decay;
  const float* grad_scale;         /* device scalar or NULL (gradients already unscaled) */
  const float* found_inf;          /* device scalar or NULL (no inf check) */
} csa_adamw_args;

csa_status csa_adamw_step(const csa_adamw_args* a, void* stream);

/* ---- Generator head (module/components.py:95-102): logp = log(softmax(dropout(logits), -1)) ----
 * logits/logp/dlogp/dlogits: (rows, V) contiguous fp32. dropout p in [0,1) (0 = eval); the keep mask
 * is regenerated in the backward from (seed, offset): Philox stream 4, element (row, col) ->
 * u16 (col & 7) of philox({col >> 3, row, 0, (4 << 28) ^ offset}), keep <=> u16 >= ceil(p * 65536).
 * Backward is the reference autograd chain: t = dlogp / s, dz = keep / (1-p) * s * (t - sum(t * s)). */
csa_status csa_gen_logsoftmax_fwd(const float* logits, float* logp, int64_t rows, int64_t V, float dropout,
                                  uint64_t seed, uint64_t offset, void* stream);
csa_status csa_gen_logsoftmax_bwd(const float* dlogp, const float* logp, float* dlogits, int64_t rows, int64_t V,
                                  float dropout, uint64_t seed, uint64_t offset, void* stream);

/* ---- Linear bias gradient: db[c] (+)= sum_r dy[r, c], dy (rows, cols) contiguous fp32 ----
 * Two passes (row-slice partials into the caller's workspace, then a fixed-order sum): deterministic. */
size_t csa_bias_grad_workspace_bytes(int64_t rows, int64_t cols);
csa_status csa_bias_grad(const float* dy, float* db, int64_t rows, int64_t cols, int accumulate, void* workspace,
                         void* stream);

/* ---- LayerNorm over the last dim (nn.LayerNorm(cols), affine) of the encoder/decoder glue ----
 * x, y, dy, dx: (rows, cols) contiguous fp32, cols % 4 == 0 and cols <= 1024 (csa_layernorm_supported);
 * stats: (rows, 2) saved (mean, rstd). Backward writes dx, dgamma, dbeta (deterministic: fixed-order
 * column partials in the caller's workspace). */
int csa_layernorm_supported(int64_t cols);
size_t csa_layernorm_bwd_workspace_bytes(int64_t rows, int64_t cols);
csa_status csa_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y, float* stats,
                             int64_t rows, int64_t cols, float eps, void* stream);
csa_status csa_layernorm_bwd(const float* dy, const float* x, const float* stats, const float* gamma, float* dx,
                             float* dgamma, float* dbeta, int64_t rows, int64_t cols, void* workspace, void* stream);

/* ---- Residual + dropout of the pre-LN blocks (module/components.py SublayerConnection
 * `x + self.dropout(sublayer(self.norm(x)))`; module/sbm_model.py:29-31 `self.dropout1(out) + X` and
 * `self.mlpblock(self.norm2(X)) + X`, whose last mlpblock module is the Dropout) ----
 * x, o, y, dy, d_o: n fp32 elements in the same memory order, 16-byte aligned; 0 < p < 1.
 * y = x + keep * o / (1 - p); d_o = keep * dy / (1 - p) (the residual gradient is dy itself).
 * keep for element i: Philox4x32-7 stream 5 (oracle/philox.py:res_keep), regenerated by the backward. */
csa_status csa_residual_dropout_fwd(const float* x, const float* o, float* y, int64_t n, float p, uint64_t seed,
                                    uint64_t offset, void* stream);
csa_status csa_residual_dropout_bwd(const float* dy, float* d_o, int64_t n, float p, uint64_t seed, uint64_t offset,
                                    void* stream);

/* ---- GELU + dropout of the feed-forward blocks (module/components.py FeedForward
 * `linear2(dropout(gelu(linear1(x))))`; module/sbm_model.py:22-26 mlpblock GELU -> Dropout) ----
 * h, y, dy, dh: n fp32 elements in the same memory order, 16-byte aligned; 0 <= p < 1.
 * y = keep * gelu(h) / (1 - p) (exact erf GELU); dh = keep * dy / (1 - p) * gelu'(h).
 * keep for element i: Philox4x32-7 stream 6 (oracle/philox.py:ffn_keep), regenerated by the backward. */
csa_status csa_gelu_dropout_fwd(const float* h, float* y, int64_t n, float p, uint64_t seed, uint64_t offset,
                                void* stream);
csa_status csa_gelu_dropout_bwd(const float* dy, const float* h, float* dh, int64_t n, float p, uint64_t seed,
                                uint64_t offset, void* stream);

/* ---- Host data path: AST relation planes (my_ast.py:198-273, dataset/base_data_set.py:33-36) ----
 * parent: (B, max_size) int32, pre-order ids (parent[v] < v, parent[0] = -1); n_nodes: (B,) int32
 * (trees longer than max_size are truncated to their pre-order prefix). Outputs (B, max_size,
 * max_size) uint8 host arrays: L / T = clamp(raw + 75, 0, 149), L_mask / T_mask = (raw == 0).
 * Runs on the host (nthreads std::threads); no HIP call. */
csa_status csa_ast_relations(const int32_t* parent, const int32_t* n_nodes, int64_t B, int64_t max_size, uint8_t* L,
                             uint8_t* T, uint8_t* L_mask, uint8_t* T_mask, int nthreads);

/* collect_fn's encoding (dataset/base_data_set.py:33-36) of raw fp32 relation matrices (any shape, n
 * elements, e.g. a stacked (B, N, N) batch of split_matrices.npz L / T): idx = clamp(raw + 75, 0, 149),
 * mask = (raw == 0). Host only; replaces the per-item torch.clamp / eq / stack of the reference. */
csa_status csa_collate_relations(const float* L_raw, const float* T_raw, int64_t n, uint8_t* L, uint8_t* T,
                                 uint8_t* L_mask, uint8_t* T_mask, int nthreads);

#ifdef __cplusplus
}
#endif
#endif /* CSA_HIP_H */

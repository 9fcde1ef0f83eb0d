/*
 * mmfd.h — C ABI of libmmfd_hip.so, the MI355X (gfx950) kernels behind the multimodal
 * misinformation-detection training hot path.
 *
 * The reference (sakdag/multimodal-misinformation-detection) is pure Python: its "interface" for
 * this path is a set of torch.nn modules and torch ops. Each entry point below names the
 * reference call sites it replaces (file:line, relative to the reference repo root).
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer unless documented otherwise; the library never allocates,
 *     frees or synchronises; work is enqueued on `stream` (a hipStream_t; NULL = default stream);
 *   - tensors are dense row-major with an explicit leading dimension (elements, not bytes);
 *   - `dtype` is MMFD_F32 or MMFD_BF16 (storage type of activations / operands); accumulation,
 *     LayerNorm statistics, softmax statistics, optimizer state and all gradients of parameters are
 *     fp32;
 *   - return value 0 = success; otherwise an MMFD_ERR_* or hipError_t code, and
 *     mmfd_last_error_string() describes it (thread-local).
 *   - dropout is counter based: element e of call-site `salt` is dropped iff
 *     hash(*seed, salt, e) < p * 2^32 (hash = mmfd_hash in csrc/common.h), so backward kernels
 *     regenerate the forward mask and a CPU oracle can reproduce it exactly.
 */
#ifndef MMFD_H_
#define MMFD_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* mmfd_stream_t; /* hipStream_t */

enum { MMFD_F32 = 0, MMFD_BF16 = 1, MMFD_F16 = 2 /* retrieval corpora only */ };
enum {
  MMFD_ACT_NONE = 0,
  MMFD_ACT_GELU = 1,      /* exact erf GELU, nn.GELU() (layers.py:14) / HF "gelu" */
  MMFD_ACT_RELU = 2,      /* nn.ReLU() (model.py:264 ...) */
  MMFD_ACT_GELU_BWD = 3,  /* out *= gelu'(aux)  (aux = saved pre-activation) */
  MMFD_ACT_RELU_BWD = 4,  /* out *= (aux > 0)   */
  MMFD_ACT_TANH = 5,      /* tanh (HF BertPooler, the cross-encoder's [CLS] pooler), forward only */
  MMFD_ACT_SIGMOID = 6,   /* 1 / (1 + exp(-x)) (CrossEncoder's default score activation) */
  MMFD_ACT_GELU_D = 7,    /* GELU as MMFD_ACT_GELU, but aux <- gelu'(pre-activation) (training forward) */
  MMFD_ACT_MUL_AUX = 8    /* out *= aux  (aux = a saved derivative: the MMFD_ACT_GELU_D backward) */
};
enum { MMFD_OK = 0, MMFD_ERR_INVALID = 1000, MMFD_ERR_UNSUPPORTED = 1001 };

/* ------------------------------------------------------------------------------------------- */
/* library                                                                                      */
/* ------------------------------------------------------------------------------------------- */
const char* mmfd_last_error_string(void);
/* ABI version of this header: bumped on every change of an argument struct's layout (2: struct_size
   at the head of mmfd_gemm_args / mmfd_attn_args, mmfd_attn_args.drop_mask). mmfd_version() returns
   the library's; a caller compares it with MMFD_ABI_VERSION before its first call. */
#define MMFD_ABI_VERSION 3
int mmfd_version(void);
/* 32-bit dropout hash (host copy of the device function), for tests and the CPU oracle. */
uint32_t mmfd_dropout_hash(uint64_t seed, uint64_t salt, uint64_t index);

/* ------------------------------------------------------------------------------------------- */
/* GEMM with fused epilogue.                                                                    */
/* Replaces every nn.Linear forward/backward on the path: src/model/model.py:19-36, 137-152,   */
/* 252-288, 395-403; src/model/layers.py:12-18, 57 (out_proj); the HF BERT/ViT projections      */
/* called at train.py:137-143; the ViT patch conv (GEMM over patches).                         */
/*   C[m][n] = epilogue( alpha * sum_k A(m,k) B(k,n) ) (+ beta * C_old[m][n])                  */
/*   A(m,k) = trans_a ? A[k*lda + m] : A[m*lda + k]                                             */
/*   B(k,n) = trans_b ? B[k*ldb + n] : B[n*ldb + k]     (trans_b=0 is nn.Linear's W[N][K])     */
/* Epilogue order: z = alpha*acc + bias[n]; if act is a forward act: aux <- z, z = act(z);      */
/*   if act is a backward act: z *= act'(aux); dropout(z); z += residual; z += beta*C_old.      */
/* ------------------------------------------------------------------------------------------- */
typedef struct mmfd_epilogue {
  const float* bias;       /* [N] fp32, or NULL */
  const void* residual;    /* [M][ldr] in c_dtype, or NULL */
  int64_t ldr;
  void* aux;               /* [M][ldaux] in c_dtype: written by GELU/RELU, read by *_BWD */
  int64_t ldaux;
  int act;                 /* MMFD_ACT_* */
  float dropout_p;         /* 0 disables */
  const uint64_t* seed;    /* device pointer to the step seed (read by the kernel) */
  uint64_t salt;           /* call-site id; element index = m * N + n */
  int residual_first;      /* 1: z += residual BEFORE the (forward) activation, i.e. act(acc + bias +
                              residual) — the ResNet bottleneck's relu(bn3(conv3) + identity) */
  void* out_planes;        /* fp32 C only: bf16 [3][M][N] split planes of the final output (mmfd_split3
                              form, N % 8 == 0), written beside C, or instead of it when C is NULL
                              (beta = 0): a GEMM output whose only consumers are split-operand GEMMs */
} mmfd_epilogue;

/* Implicit-GEMM convolution geometry (mmfd_gemm_args.conv; the ResNet50 extractor's convolutions,
   im2im_retrieval.py:14-17, 29-36): A is the NHWC activation x[N][H][W][C] and
     op(A)[m][k] = x[n][oh*stride - pad + kh][ow*stride - pad + kw][c]   (0 outside the image)
   with m = (n*Ho + oh)*Wo + ow, k = (kh*KW + kw)*C + c — the im2col matrix, gathered by the GEMM's
   operand fill instead of being written. Requires trans_a = 0, M = N*Ho*Wo, K = KH*KW*C, C a
   multiple of 32 (fp32) / 64 (bf16), x 16-B aligned, no a_rowsum; lda is ignored. With fp32
   operands on the split-operand path a_planes, when given, are the planes [3][N*H*W][C] of x. */
typedef struct mmfd_conv_geom {
  int64_t N, H, W, C;      /* input images */
  int KH, KW, stride, pad;
  int64_t Ho, Wo;          /* output size */
} mmfd_conv_geom;

typedef struct mmfd_gemm_args {
  int64_t struct_size;     /* = sizeof(mmfd_gemm_args) of the caller's header; the library refuses
                              any other value (MMFD_ERR_INVALID): a caller built against another
                              layout of this struct fails loudly instead of passing shifted fields */
  int dtype;               /* operand dtype of A and B */
  int trans_a, trans_b;
  int64_t M, N, K;
  const void* A; int64_t lda;
  const void* B; int64_t ldb;
  void* C; int64_t ldc; int c_dtype;
  float alpha, beta;
  mmfd_epilogue ep;
  void* workspace; int64_t workspace_bytes; /* split-K fp32 slabs; may be NULL (no split) */
  int splits;              /* 0 = choose automatically (bounded by workspace_bytes) */
  /* optional fused row sums of op(A) (the bias gradient sum_tokens dY of a weight-gradient GEMM,
     replacing the reference's autograd of nn.Linear.bias): a_rowsum[m] = a_rowsum_beta *
     a_rowsum[m] + sum_k op(A)[m][k], fp32, M entries. NULL disables. */
  float* a_rowsum; float a_rowsum_beta;
  /* optional bf16 planes [3][rows][cols] of the stored fp32 A / B (mmfd_split3), for the split-
     operand fp32 GEMM (mmfd_set_fp32_gemm_mode): a product whose operand was already split — the
     forward input reused by the weight-gradient GEMM, the output gradient shared by the data- and
     weight-gradient GEMMs — reads them instead of splitting again. NULL = split here. Ignored by
     the other paths. */
  const void* a_planes; const void* b_planes;
  /* 1: the fp32 A / B was never written (its only form is the planes): mmfd_gemm fails with
     MMFD_ERR_UNSUPPORTED instead of reading it when the split-operand path is not taken */
  int a_planes_only, b_planes_only;
  /* ABI 3: non-NULL = A is an implicit convolution operand (mmfd_conv_geom above) */
  const mmfd_conv_geom* conv;
} mmfd_gemm_args;

int mmfd_gemm(const mmfd_gemm_args* args, mmfd_stream_t stream);
/* bytes of workspace the automatic split choice would like for this problem (incl. the per-split
   row-sum partials when a_rowsum is set, and the bf16 operand planes of a split-operand fp32 GEMM).
   This and the two queries below return -1 (mmfd_last_error_string set) for a struct_size other
   than this header's sizeof(mmfd_gemm_args). */
int64_t mmfd_gemm_workspace_bytes(const mmfd_gemm_args* args);
/* the split-K factor mmfd_gemm picks for these arguments (given the workspace it asked for) */
int mmfd_gemm_splits(const mmfd_gemm_args* args);
/* fp32 x fp32 -> fp32 GEMMs (the reference's nn.Linear arithmetic, model.py / layers.py Linears):
   mode 1 (default; env MMFD_FP32_GEMM=native selects 0 at load) splits each fp32 operand into three
   bf16 planes x = hi + mid + lo (written to the workspace) and accumulates the six products
   mid*mid, hi*lo, lo*hi, hi*mid, mid*hi, hi*hi on the bf16 MFMA in fp32 — 24 operand bits, products
   exact, the accumulation an fp32 sum (error measured at the fp32 MFMA's level, tests/
   test_kernels_gpu.py); mode 0 = the fp32 MFMA (v_mfma_f32_16x16x4f32). Used only when
   workspace_bytes covers mmfd_gemm_workspace_bytes. Returns the previous mode. */
int mmfd_set_fp32_gemm_mode(int mode);
/* whether mmfd_gemm runs these arguments as a split-operand fp32 GEMM (given the workspace it asks
   for): 0 = no (fp32 MFMA or bf16 path), 2 = the fused-plane kernel (all three planes of both
   operands staged per 32-deep K-step, the default), 1 = the segmented kernel (the K loop once per
   plane pair; env MMFD_X6_SEGMENTED). The host-side planning of which tensors may exist only as
   planes (mmfd.kernels.x6_ok) asks this, so it honours every switch the library does. */
int mmfd_gemm_runs_split(const mmfd_gemm_args* args);
/* the four-wave assembly-scheduled bf16 forward GEMM (gemm_g4.hip): mode 0 = off (those products run
   on the 256x256 eight-wave kernel), 1 = on for the bias / residual / dropout + residual epilogues,
   2 = also the GELU epilogues (default); -1 only queries. Load-time defaults from env MMFD_G4=0 /
   MMFD_G4_GELU=0. Returns the previous mode (A/B measurements and tests; not per
   stream: set it between launches). */
int mmfd_set_g4_mode(int mode);
/* the four-wave GEMM's grid: 1 = persistent (one workgroup per CU walking its tiles, the next tile's
   first K-tiles loaded during this tile's epilogue; default), 0 = one workgroup per tile (env
   MMFD_G4_PERSIST=0); -1 only queries. Returns the previous setting. */
int mmfd_set_g4_persist(int on);
/* the largest K the four-wave GEMM takes (default 1024, env MMFD_G4_KMAX); kmax <= 0 only queries.
   Returns the previous limit. */
int64_t mmfd_set_g4_kmax(int64_t kmax);
/* fp32 [rows][ld] -> bf16 planes [3][rows][cols] (hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid);
   cols % 8 == 0, 16-B aligned rows) */
int mmfd_split3(int64_t rows, int64_t cols, const float* x, int64_t ld, void* planes, mmfd_stream_t stream);

/* Column sums (bias gradients): out[n] = beta*out[n] + sum_m X[m*ldx + n]. workspace >= 4*N*256 B */
int mmfd_colsum(int dtype, int64_t M, int64_t N, const void* X, int64_t ldx, float* out, float beta,
                void* workspace, int64_t workspace_bytes, mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* Multi-head attention (unmasked fusion-head MHA layers.py:36-58 incl. the SDPA branch 44-49;  */
/* HF BERT/ViT/MPNet self-attention called at train.py:137-143).                              */
/* Q/K/V/O are addressed per (batch b, token t, head h) as base + b*s_b + t*s_t + h*D.         */
/*   S = scale * Q K^T (+ key_bias[b][k]) (+ rel_bias[b*rel_bias_sb + (h*Lq+q)*Lk + k]);        */
/*   P = softmax(S)                                                                           */
/*   O = dropout(P) V ;   lse[b][h][q] = log sum_k exp(S) (fp32)                                */
/* ------------------------------------------------------------------------------------------- */
typedef struct mmfd_attn_args {
  int64_t struct_size;             /* = sizeof(mmfd_attn_args); checked like mmfd_gemm_args.struct_size */
  int dtype;
  int64_t B, H, Lq, Lk, D;         /* D <= 64, D * element size a multiple of 16 B */
  float scale;
  const void* q; int64_t q_sb, q_st;
  const void* k; int64_t k_sb, k_st;
  const void* v; int64_t v_sb, v_st;
  void* o; int64_t o_sb, o_st;
  float* lse;                      /* [B][H][Lq] */
  const float* key_bias;           /* [B][Lk] additive (HF extended attention mask) or NULL */
  const float* rel_bias;           /* [H][Lq][Lk] additive (MPNet relative position; rel_bias_sb = 0)
                                      or [B][H][Lq][Lk] (DeBERTa c2p + p2c; rel_bias_sb = H*Lq*Lk) */
  float dropout_p; const uint64_t* seed; uint64_t salt;  /* index = ((b*H+h)*Lq+q)*Lk+k */
  /* backward only */
  const void* dout; int64_t do_sb, do_st;   /* same head layout as o */
  void* dq; int64_t dq_sb, dq_st;
  void* dk; int64_t dk_sb, dk_st;
  void* dv; int64_t dv_sb, dv_st;
  float* delta;                    /* workspace [B][H][Lq] fp32 */
  float* d_rel_bias;               /* must be NULL (the relative bias is inference-only, MPNet) */
  int accumulate_dq;               /* 1: dq += result (else overwrite) */
  int accumulate_dkv;              /* 1: dk += ..., dv += ... */
  int64_t rel_bias_sb;             /* batch stride of rel_bias in floats (0 = shared by the batch) */
  int64_t rel_bias_mod;            /* > 0: batch row b reads bias row b % rel_bias_mod (Swinv2 windows:
                                      [nW][H][L][L] shift masks, batch = images x nW windows) */
  const float* cos_logit_scale;    /* forward only, NULL = plain attention. Otherwise Swinv2 cosine
                                      attention: q_h, k_h are L2-normalised (eps 1e-12) and q_h scaled
                                      by exp(min(cos_logit_scale[h], cos_max_log)) while staged (bf16,
                                      Lk <= 256, rel_bias required); replaces mmfd_swin_qk_norm */
  float cos_max_log;
  /* backward, fp32 only: bf16 split planes [3][B*Lq][3*H*D] (mmfd_split3 form) of the packed
     gradient [dq | dk | dv] — dq, dk, dv must be the three column blocks of one contiguous
     [B, Lq, 3*H*D] buffer starting at dq (Lq == Lk) — written beside it, or instead of it with
     planes_only (no accumulate): the operand of the QKV data- and weight-gradient GEMMs */
  void* dqkv_planes; int planes_only;
  /* forward, fp32 only: bf16 split planes [3][B*Lq][H*D] of the output o (o a contiguous
     [B, Lq, H*D] buffer), written beside it — the operand of the output projection's forward and
     weight-gradient GEMMs */
  void* o_planes;
  /* dropout keep-bitmask, uint32 [B*H*Lq][ceil(Lk/32)]: word ((b*H+h)*Lq+q)*ceil(Lk/32) + k/32, bit k%32
     = 1 when element (q, k) is kept. With dropout_p > 0 the forward writes it when non-NULL, and the
     backward reads it instead of re-hashing the mask when non-NULL (the same buffer, unchanged
     between the calls); NULL: both hash (identical masks either way) */
  uint32_t* drop_mask;
} mmfd_attn_args;

int mmfd_attn_fwd(const mmfd_attn_args* args, mmfd_stream_t stream);
int mmfd_attn_bwd(const mmfd_attn_args* args, mmfd_stream_t stream);
/* fp32 attention (the reference's SDPA / softmax(QK^T)V in fp32, layers.py:44-56 and the HF encoders'
   self-attention): mode 1 (default; env MMFD_FP32_ATTN=native, or MMFD_FP32_GEMM=native without it,
   selects 0 at load) runs every product on split bf16 operands (x = hi + mid + lo, six MFMA products
   accumulated in fp32, as mmfd_set_fp32_gemm_mode) when D <= 64, D % 8 == 0, there is no relative
   bias and the resident length (keys; and queries in the backward) is <= 208; mode 0 = the fp32
   MFMA kernels. Returns the previous mode. */
int mmfd_set_fp32_attn_mode(int mode);

/* ------------------------------------------------------------------------------------------- */
/* LayerNorm over the last dim (fusion head nn.LayerNorm model.py:39-46, 155-162, eps 1e-5;     */
/* BERT/ViT LayerNorm eps 1e-12). mean/rstd are saved per row (fp32).                          */
/* ------------------------------------------------------------------------------------------- */
int mmfd_layernorm_fwd(int dtype, int64_t rows, int64_t width, const void* x, int64_t ldx,
                       const float* gamma, const float* beta, float eps, void* y, int64_t ldy,
                       float* mean, float* rstd, mmfd_stream_t stream);
/* y = res + LN(x) (Swinv2's res-post-norm, modeling_swinv2.py Swinv2Layer.forward:
 * `shortcut + layernorm_before(attn)` and `h + layernorm_after(mlp)`); 16-B aligned rows;
 * mean/rstd may both be NULL (inference). */
/* fp32 LayerNorm forward that also writes the output's bf16 split planes [3][rows][width]
   (mmfd_split3 form, width % 8 == 0): the Linear inputs of the encoder layers, split in the same
   pass (split-operand fp32 GEMMs, mmfd_set_fp32_gemm_mode) */
int mmfd_layernorm_fwd_split(int64_t rows, int64_t width, const float* x, int64_t ldx, const float* gamma,
                             const float* beta, float eps, float* y, int64_t ldy, float* mean, float* rstd,
                             void* planes, mmfd_stream_t stream);
/* fp32 LayerNorm backward (as mmfd_layernorm_bwd) that also writes the bf16 split planes
   [3][rows][width] of the gradient the next GEMMs read: dx_drop when given, else dx */
int mmfd_layernorm_bwd_split(int64_t rows, int64_t width, const float* dy, int64_t lddy, const float* x,
                             int64_t ldx, const float* gamma, const float* mean, const float* rstd,
                             float* dx, int64_t lddx, const float* dx_add, int64_t ldadd, float* dgamma,
                             float* dbeta, float beta_acc, float* dx_drop, float dropout_p,
                             const uint64_t* seed, uint64_t salt, void* workspace,
                             int64_t workspace_bytes, void* planes, mmfd_stream_t stream);
int mmfd_layernorm_fwd_res(int dtype, int64_t rows, int64_t width, const void* x, int64_t ldx,
                           const float* gamma, const float* beta, float eps, const void* res, int64_t ldr,
                           void* y, int64_t ldy, float* mean, float* rstd, mmfd_stream_t stream);
/* dx = LN'(dy) (+ dx_add); dgamma/dbeta (fp32, [width]) are written (beta_acc=0) or accumulated
 * (beta_acc=1) through a deterministic two-pass reduction; workspace >= 8*width*256 bytes.
 * If dx_drop != NULL it also receives dropout(dx) for call-site (seed, salt, p) with element
 * index row*width+col (the mask the producing GEMM epilogue applied). */
int mmfd_layernorm_bwd(int dtype, int64_t rows, int64_t width, const void* dy, int64_t lddy,
                       const void* x, int64_t ldx, const float* gamma, const float* mean,
                       const float* rstd, void* dx, int64_t lddx, const void* dx_add, int64_t ldadd,
                       float* dgamma, float* dbeta, float beta_acc, void* dx_drop,
                       float dropout_p, const uint64_t* seed, uint64_t salt,
                       void* workspace, int64_t workspace_bytes, mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* Sequence mean pooling S.mean(dim=1) (model.py:308-317, 332-345, 448)                         */
/* ------------------------------------------------------------------------------------------- */
int mmfd_seq_mean_fwd(int dtype, int64_t B, int64_t L, int64_t D, const void* x, void* out,
                      int64_t ldo, mmfd_stream_t stream);
int mmfd_seq_mean_bwd(int dtype, int64_t B, int64_t L, int64_t D, const void* dout, int64_t ldo,
                      void* dx, mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* Summed per-path cross entropy (train.py:165-169: sum over PRESENT paths idx of                */
/* CrossEntropyLoss(y_idx, labels[:, idx]); absent paths (None outputs) contribute nothing).     */
/* logits: HOST array of n_paths device pointers, each [B][C] fp32; path_cols: HOST array of    */
/* n_paths label columns (the reference's path index idx, train.py:165; NULL = 0..n_paths-1);   */
/* labels int64 (device) [B][label_ld]. loss (device, n_slots >= 1 + max column) receives       */
/* loss[0] = total, loss[1+col] = that path's mean loss and 0 for columns with no present path.  */
/* dlogits (optional host array of n_paths device pointers) receive d(total)/d(logits) *        */
/* (*dloss_scale or 1), dloss_scale being a device scalar (NULL = 1).                            */
/* ------------------------------------------------------------------------------------------- */
int mmfd_xent_fwd_bwd(int n_paths, int64_t B, int64_t C, const float* const* logits,
                      const int* path_cols, const int64_t* labels, int64_t label_ld, float* loss,
                      int n_slots, float* const* dlogits, const float* dloss_scale,
                      mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* BERT embeddings (HF BertEmbeddings: word + position + token_type, LayerNorm, dropout).       */
/* ------------------------------------------------------------------------------------------- */
int mmfd_embed_ln_fwd(int dtype, int64_t B, int64_t L, int64_t D, const int64_t* input_ids,
                      const int64_t* token_type_ids, const float* word, const float* pos,
                      const float* type, const float* gamma, const float* beta, float eps,
                      void* sum_out, void* y, float* mean, float* rstd, float dropout_p,
                      const uint64_t* seed, uint64_t salt, mmfd_stream_t stream);
/* Generalised embeddings (HF MPNetEmbeddings / RoBERTa-style, text2text_retrieval.py:21,125 bi-encoder):
   position_ids (NULL = 0..L-1 per sequence), token_type_ids/type (NULL = no type table),
   sum_out/mean/rstd (NULL = not saved; inference). */
int mmfd_embed_ln_fwd_ex(int dtype, int64_t B, int64_t L, int64_t D, const int64_t* input_ids,
                         const int64_t* position_ids, const int64_t* token_type_ids, const float* word,
                         const float* pos, const float* type, const float* gamma, const float* beta, float eps,
                         void* sum_out, void* y, float* mean, float* rstd, float dropout_p,
                         const uint64_t* seed, uint64_t salt, mmfd_stream_t stream);
/* position ids = padding_idx + running count of non-pad tokens (pads get padding_idx), int64 [B][L] */
int mmfd_position_ids(int64_t B, int64_t L, const int64_t* input_ids, int64_t padding_idx, int64_t* out,
                      mmfd_stream_t stream);
/* relative position bias (MPNet encoder.relative_attention_bias): out[h][q][k] = table[bucket[q][k]][h];
   bucket int32 [Lq][Lk] (host-computed with the reference's bucket formula), table fp32 [nb][H] */
int mmfd_rel_bias(int64_t H, int64_t Lq, int64_t Lk, const int32_t* bucket, const float* table, float* out,
                  mmfd_stream_t stream);
/* DeBERTa-v3 (the reference's default text encoder, train.py:330-331; transformers
   modeling_deberta_v2.py). Disentangled bias for the attention's rel_bias ([B][H][L][L] fp32):
   out[b][h][i][j] = c2p[h][b*L+i][c2p_idx[i][j]] * inv_scale + p2c[h][b*L+j][p2c_idx[j][i]] * inv_scale
   with c2p = Q_h . posK_h^T and p2c = K_h . posQ_h^T ([H][B*L][ld], dtype), the clamped log-bucket
   indices int32 [L][L] computed on the host (modeling_deberta_v2.py:276-346). */
int mmfd_deberta_rel_bias(int dtype, int64_t B, int64_t H, int64_t L, const void* c2p, const void* p2c, int64_t ld,
                          const int32_t* c2p_idx, const int32_t* p2c_idx, float inv_scale, float* out,
                          mmfd_stream_t stream);
/* x[r][:] = 0 where mask[r] == 0 (DebertaV2Embeddings: embeddings * mask, :552-559), x [rows][ldx] */
int mmfd_mask_rows(int dtype, int64_t rows, int64_t D, void* x, int64_t ldx, const int64_t* mask,
                   mmfd_stream_t stream);
/* attention rows of fully masked queries (mask[b][i] == 0): masked_fill(finfo.min) + softmax gives
   them uniform weights over ALL Lk keys (modeling_deberta_v2.py:252-256), i.e. o = mean_k v.
   q-layout views as in mmfd_attn_args (v: base + b*v_sb + t*v_st + h*D). */
int mmfd_attn_fill_masked_rows(int dtype, int64_t B, int64_t H, int64_t L, int64_t Dh, const void* v, int64_t v_sb,
                               int64_t v_st, void* o, int64_t o_sb, int64_t o_st, const int64_t* mask,
                               mmfd_stream_t stream);
/* scatter-add the gradient of the pre-LN sum into the three tables (modeling_bert.py BertEmbeddings:
   word[id] += row, pos[t] += row, type[tt] += row), deterministically: the word rows are stably
   radix-sorted by id and each id's rows summed in row order by one writer; the type table reduces
   fixed row slabs in order. vocab = rows of the word table (ids in [0, vocab)): the sort runs over
   the ceil(log2(vocab)) id bits only (<= 0: all 32 bits; ABI 3 added it). workspace >=
   mmfd_embed_bwd_workspace_bytes(B, L, D); ids < 2^32, B*L < 2^31. dword / dpos / dtype_emb may each
   be NULL (that table is skipped). */
int64_t mmfd_embed_bwd_workspace_bytes(int64_t B, int64_t L, int64_t D);
int mmfd_embed_bwd(int dtype, int64_t B, int64_t L, int64_t D, int64_t vocab, const int64_t* input_ids,
                   const int64_t* token_type_ids, const void* dsum, float* dword, float* dpos,
                   float* dtype_emb, int64_t padding_idx, void* workspace, int64_t workspace_bytes,
                   mmfd_stream_t stream);
/* key-padding mask (int64 0/1) -> additive bias (0 or `neg`, HF uses finfo(float32).min) */
int mmfd_mask_to_bias(int64_t n, const int64_t* mask, float* out, float neg, mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* ResNet50 evidence-image extractor (im2im_retrieval.py:14-36, torchvision resnet50 minus fc): */
/* NHWC activations, convolutions as MFMA GEMMs (mmfd_gemm) over im2col gathers, eval-mode      */
/* BatchNorm folded into the weights, ReLU / residual add in the GEMM epilogue.                 */
/* ------------------------------------------------------------------------------------------- */
/* out_w[co][(kh*KW+kw)*Cin+ci] = w[co][ci][kh][kw]*s[co] (zero for k >= KH*KW*Cin < Kpad),
   out_b[co] = beta - mean*s, s = gamma/sqrt(var+eps); gamma == NULL: no BatchNorm (s=1, b=0) */
int mmfd_conv_weight_prep(int dtype, int64_t Cout, int64_t Cin, int64_t KH, int64_t KW, int64_t Kpad,
                          const float* w, const float* gamma, const float* beta, const float* mean,
                          const float* var, float eps, void* out_w, float* out_b, mmfd_stream_t stream);
/* NHWC im2col: out[(n*Ho+ho)*Wo+wo][(kh*KW+kw)*C+c] (zero outside the image and for k >= KH*KW*C);
   C a multiple of 16 B; also the strided 1x1 gather of the downsample shortcut */
int mmfd_im2col_nhwc(int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int KH, int KW, int stride,
                     int pad, int64_t Ho, int64_t Wo, int64_t Kpad, const void* x, void* out,
                     mmfd_stream_t stream);
/* stem im2col from fp32 NCHW pixels (same column order (kh, kw, c)) */
int mmfd_im2col_nchw(int dtype, int64_t N, int64_t C, int64_t H, int64_t W, int KH, int KW, int stride,
                     int pad, int64_t Ho, int64_t Wo, int64_t Kpad, const float* x, void* out,
                     mmfd_stream_t stream);
/* k x k max pooling on NHWC (nn.MaxPool2d(3, 2, 1)) */
int mmfd_maxpool_nhwc(int dtype, int64_t N, int64_t H, int64_t W, int64_t C, int k, int stride, int pad,
                      int64_t Ho, int64_t Wo, const void* x, void* out, mmfd_stream_t stream);
/* global average pool NHWC [N][HW][C] -> fp32 [N][C] (nn.AdaptiveAvgPool2d(1) + flatten) */
int mmfd_global_avgpool(int dtype, int64_t N, int64_t HW, int64_t C, const void* x, float* out,
                        mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* ViT patch embedding support (HF ViTPatchEmbeddings conv16/s16 == GEMM over patches).         */
/* patchify: pixels fp32 [B][C][Hh][Ww] -> out [B*np][C*P*P] in dtype (c, kh, kw order).        */
/* tokens: out[b][0] = cls + pos[0]; out[b][1+p] = patch[b*np+p] + pos[1+p].                     */
/* ------------------------------------------------------------------------------------------- */
int mmfd_patchify(int dtype, int64_t B, int64_t C, int64_t Hh, int64_t Ww, int64_t P,
                  const float* pixels, void* out, mmfd_stream_t stream);
int mmfd_vit_tokens_fwd(int dtype, int64_t B, int64_t NP, int64_t D, const void* patch,
                        const float* cls, const float* pos, void* out, mmfd_stream_t stream);
int mmfd_vit_tokens_bwd(int dtype, int64_t B, int64_t NP, int64_t D, const void* dout, void* dpatch,
                        float* dcls, float* dpos, void* workspace, int64_t workspace_bytes,
                        mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* Swinv2 image encoder (reference default image encoder: Swinv2Model swinv2-base-patch4-window8- */
/* 256, train.py:332, called at train.py:142-143 / preprocess_embeddings.py:91-92; transformers  */
/* modeling_swinv2.py). Inference only.                                                        */
/* ------------------------------------------------------------------------------------------- */
/* dst row (b, r) = concat_g src row (b, idx[r*G + g]); rows are row_bytes wide (multiple of 16).
 * Replaces torch.roll + window_partition / window_reverse and the patch-merging 2x2 concat. */
int mmfd_row_gather(int64_t B, int64_t rows_out, int64_t G, int64_t row_bytes, int64_t src_rows,
                    const void* src, const int32_t* idx, void* dst, mmfd_stream_t stream);
/* continuous position-bias MLP: out[t][h] = sum_k w2[h][k] relu(w1[k] . coords[t] + b1[k]),
 * 512 hidden units (Swinv2SelfAttention.continuous_position_bias_mlp), all fp32 */
int mmfd_swin_cpb(int64_t T, int64_t H, const float* coords, const float* w1, const float* b1,
                  const float* w2, float* out, mmfd_stream_t stream);
/* out[w][h][i][j] = 16 sigmoid(table[rpi[i*L+j]][h]) (+ mask[w][i][j] twice, as HF adds it);
 * mask NULL -> nW must be 1 */
int mmfd_swin_bias(int64_t nW, int64_t H, int64_t L, const float* table, const int32_t* rpi,
                   const float* mask, float* out, mmfd_stream_t stream);
/* cosine attention operands in place on packed [rows][ld] QKV (q at column 0, k at H*d):
 * q_h /= max(|q_h|, 1e-12) and *= exp(min(logit_scale[h], max_log)); k_h /= max(|k_h|, 1e-12) */
int mmfd_swin_qk_norm(int dtype, int64_t rows, int64_t H, int64_t d, void* qkv, int64_t ld,
                      const float* logit_scale, float max_log, mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* AdamW (torch.optim.AdamW defaults as used at train.py:356/188), multi-tensor, one launch.    */
/* table: device array of n_tensors records {param f32*, grad f32*, exp_avg f32*, exp_avg_sq     */
/* f32*, param_bf16 bf16* (optional shadow copy, may be NULL), step f32*, numel};             */
/* max_numel = largest numel. Step counters live in device memory: the launch first increments */
/* every *step, then updates with the new values, so a captured hipGraph replays correctly.     */
/* ------------------------------------------------------------------------------------------- */
typedef struct mmfd_adamw_tensor {
  float* param; const float* grad; float* exp_avg; float* exp_avg_sq; void* param_bf16;
  float* step;             /* per-tensor step counter (device fp32, like torch's state['step']) */
  int64_t numel;
} mmfd_adamw_tensor;
int mmfd_adamw(int n_tensors, const mmfd_adamw_tensor* table, int64_t max_numel, float lr,
               float beta1, float beta2, float eps, float weight_decay, mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* elementwise helpers                                                                          */
/* ------------------------------------------------------------------------------------------- */
/* out(dtype_out) = in(dtype_in) * scale (+ add) — casts / scaled copies / grad accumulation. */
int mmfd_cast(int dtype_in, int dtype_out, int64_t n, const void* in, void* out, mmfd_stream_t stream);
/* out[c][r] = in[r][c] (fp32 or bf16, row-major with leading dims ldi >= cols, ldo >= rows; no
   aliasing): the K-contiguous copy of an nn.Linear weight that lets its data-gradient GEMM run in
   the forward operand layout (the four-wave GEMM), refreshed once per step */
int mmfd_transpose(int dtype, int64_t rows, int64_t cols, const void* in, int64_t ldi, void* out, int64_t ldo,
                   mmfd_stream_t stream);
/* dst[0 .. bytes) = 0 on the stream, by a kernel (graph-capture safe); the scatter-add targets of
   the embedding backward */
int mmfd_zero(void* dst, int64_t bytes, mmfd_stream_t stream);
int mmfd_axpby(int dtype, int64_t n, float a, const void* x, float b, const void* y, void* out,
               mmfd_stream_t stream);
/* generic dropout (out = keep ? x/(1-p) : 0), index = element index. */
int mmfd_dropout(int dtype, int64_t n, const void* x, void* out, float p, const uint64_t* seed,
                 uint64_t salt, mmfd_stream_t stream);
/* out = dropout(dy) * act'(aux) over n contiguous elements (standalone layers.MLP backward) */
int mmfd_act_bwd(int dtype, int64_t n, const void* dy, const void* aux, int act, float dropout_p,
                 const uint64_t* seed, uint64_t salt, void* out, mmfd_stream_t stream);
/* seed[0] += 1 (advances the step seed inside a captured graph) */
int mmfd_seed_advance(uint64_t* seed, mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* Evidence retrieval scoring.                                             */
/* Replaces the per-image Python loop of ImageCorpus.retrieve_similar_images                    */
/* (src/evidence/im2im_retrieval.py:80-92: nn.CosineSimilarity(dim=1, eps=1e-6) per corpus      */
/* entry, then sorted(reverse=True) at :94-96) and the bi-encoder stage of                      */
/* SemanticSimilarity.search (src/evidence/text2text_retrieval.py:49-66: util.semantic_search,  */
/* i.e. cos_sim of normalised fp16 embeddings + top-k).                                         */
/* cosine_scores: scores[q][n] (fp32, leading dim lds) for fp32 queries [Q][ldq] against a      */
/*   corpus [N][ldc] of corpus_dtype (MMFD_F32 / MMFD_BF16 / MMFD_F16; 16-byte aligned rows,    */
/*   D % 8 == 0). mode MMFD_COS_PAIR: dot / sqrt(max(|q|^2 |c|^2, eps^2)) (nn.CosineSimilarity); */
/*   MMFD_COS_NORMALIZED: dot / (max(|q|, eps) max(|c|, eps)) (util.cos_sim, eps 1e-12); OR     */
/*   MMFD_COS_ROUND_F16 to round each score to fp16 (scores of fp16 embeddings).               */
/* topk: per query, the k largest scores in descending order, ties broken by the LOWER corpus   */
/*   index (the order of Python's stable sort over the reference's insertion-ordered corpus);   */
/*   k <= 2048; missing entries (k > N) are -inf / -1. Workspace from mmfd_topk_workspace_bytes.*/
/* ------------------------------------------------------------------------------------------- */
enum { MMFD_COS_PAIR = 0, MMFD_COS_NORMALIZED = 1, MMFD_COS_ROUND_F16 = 4 };
int mmfd_cosine_scores(int corpus_dtype, int64_t Q, int64_t N, int64_t D, const float* queries,
                       int64_t ldq, const void* corpus, int64_t ldc, int mode, float eps, float* scores,
                       int64_t lds, mmfd_stream_t stream);
int64_t mmfd_topk_workspace_bytes(int64_t Q, int64_t N, int64_t k);
int mmfd_topk(int64_t Q, int64_t N, const float* scores, int64_t lds, int64_t k, float* out_val,
              int64_t* out_idx, void* workspace, int64_t workspace_bytes, mmfd_stream_t stream);

/* ------------------------------------------------------------------------------------------- */
/* Raw-image preprocessing: PIL bilinear resize (as torchvision's Resize on */
/* PIL images: src/model/dataset.py:14-19 Resize(256)+CenterCrop(256), and                     */
/* src/evidence/im2im_retrieval.py:19-27 Resize((224,224))) + crop + ToTensor + Normalize, for a */
/* batch of decoded RGB uint8 HWC images already on the device. The host supplies PIL's taps:   */
/* coef holds, per image and axis, one record [xmin, n, k_0 .. k_{K-1}] (int32, 22-bit fixed    */
/* point, K = kx_size / ky_size) per output position; the result is bit-identical to PIL +      */
/* torchvision. out: fp32 [n_images][3][Ho][Wo]; the crop window starts at (crop_y, crop_x) of  */
/* the resized (out_h x out_w) image. workspace: per image h * out_w * 3 bytes at tmp_off.      */
/* mean3 / std3 are HOST arrays of 3 floats.                                                    */
/* ------------------------------------------------------------------------------------------- */
typedef struct mmfd_image_desc {
  const uint8_t* src; int64_t h, w, stride;  /* device pointer, rows of stride bytes, RGB      */
  int32_t out_h, out_w, crop_y, crop_x;      /* resized size and crop origin                  */
  int64_t kx_off, ky_off;                    /* int32 offsets of the x / y tap tables in coef */
  int32_t kx_size, ky_size;                  /* taps per record (K)                           */
  int64_t tmp_off;                           /* byte offset of the image's pass-1 rows        */
} mmfd_image_desc;
int mmfd_resize_normalize(int64_t n_images, const mmfd_image_desc* descs, int64_t max_h, int64_t max_out_w,
                          const int32_t* coef, void* workspace, int64_t Ho, int64_t Wo, const float* mean3,
                          const float* std3, float* out, mmfd_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MMFD_H_ */

/*
 * mme.h — C ABI of libmme, the MI355X (gfx950) hot path of the
 * multimodal-embedding retrieval engine.
 *
 * Drop-in boundary: the reference (sariekr/multimodal-embedding,
 * main.py) has no native code; its hot path is the duck-typed HF model /
 * processor pair consumed by
 *   encode_data               main.py:386-438
 *   compute_similarity_scores main.py:440-475
 *   compute_metrics_detailed  main.py:305-383
 * Every entry point below replaces one arithmetic step those functions reach
 * through PyTorch / HF / PIL / colpali_engine; the step is cited per function.
 *
 * Conventions
 *   - all tensor pointers are DEVICE pointers owned by the caller; libmme never
 *     allocates or frees caller memory. Scratch comes from a caller workspace.
 *   - `stream` is a hipStream_t passed as void* (0 = legacy default stream).
 *   - bf16 tensors are IEEE bfloat16 bit patterns (uint16), row-major, with an
 *     explicit leading dimension (`ld*`, in elements).
 *   - return value: MME_OK (0) or an error code; mme_last_error() gives text
 *     (thread-local). Kernels are only launched after all argument checks pass.
 */
#ifndef MME_H_
#define MME_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MME_OK 0
#define MME_ERR_ARG 1         /* bad shape / pointer / alignment           */
#define MME_ERR_HIP 2         /* HIP runtime error at launch               */
#define MME_ERR_UNSUPPORTED 3 /* valid request this build does not handle  */

#define MME_ABI_VERSION 9  /* 6: mme_gemm_res_stats row_part is [M][N / 64][2]; 7: mme_build_flags, mme_topk_rows_torch;
                              8: mme_recall_hits skip mask, mme_sim_scores, mme_tie_rows; per-call kernel
                                 forms (mme_*_form) replace the process-global *_variant switches, which
                                 remain in the development build only;
                              9: mme_attention_qs (+ _form), Q pre-scaled */

/* mme_build_flags() bits */
#define MME_BUILD_DEV 1 /* development / diagnostic kernel forms compiled in (libmme_dev.so) */

/* activation codes for mme_gemm (HF config.hidden_act) */
#define MME_ACT_NONE 0
#define MME_ACT_GELU_TANH 1  /* "gelu_pytorch_tanh" (SigLIP)        */
#define MME_ACT_QUICK_GELU 2 /* "quick_gelu" (OpenAI CLIP, DFN5B)   */
#define MME_ACT_GELU_ERF 3   /* "gelu" (LAION ViT-H/14)             */
#define MME_ACT_GEGLU_TANH 4 /* gated: gelu_tanh(gate) * up (GemmaMLP, ColPali); see mme_gemm */

/* output kinds for mme_preprocess_u8 */
#define MME_PIX_F32_NCHW 0 /* pixel_values fp32 [n,3,S,S] (HF processor output)   */
#define MME_PIX_PATCHES 1  /* bf16 im2col patches [n*(S/p)^2, kpad] (fused path)  */

const char* mme_last_error(void);
int mme_abi_version(void);
int mme_build_flags(void); /* MME_BUILD_* bits of this library */

/* ---------------------------------------------------------------- a2 ----
 * PIL-exact bicubic resize of u8 RGB images + rescale(1/255) + normalise.
 * Replaces processor(images=...) main.py:407 -> HF PIL backend
 * (image_processing_backends.py PilBackend._preprocess: resize, center_crop,
 * rescale, normalize) -> PIL Image.resize(BICUBIC) (libImaging/Resample.c).
 * imgs  : u8 [n, H, W, 3] (NHWC, as PIL's RGB raster)
 * (rh, rw) resized size, then a crop of S x S at (top, left) (CLIP center crop;
 *          SigLIP: rh = rw = S, top = left = 0).
 * out   : MME_PIX_F32_NCHW -> float [n,3,S,S]
 *         MME_PIX_PATCHES  -> bf16 [n*G*G, kpad], G = floor(S/patch) (Conv2d 'valid'), column c*p*p+ky*p+kx
 *                             (Conv2d weight flattening), zero for col >= 3*p*p.
 * mean3/std3: HOST float[3] (per-channel, copied into the kernel arguments).
 * workspace: >= mme_preprocess_workspace_bytes(n, H, W, rh, rw) bytes. */
size_t mme_preprocess_workspace_bytes(int n, int H, int W, int rh, int rw);
int mme_preprocess_u8(const uint8_t* imgs, int n, int H, int W, int rh, int rw, int top, int left,
                      int S, const float* mean3, const float* std3, int out_kind, int patch, int kpad,
                      void* out, void* workspace, size_t ws_bytes, void* stream);

/* im2col of fp32 / bf16 pixel_values [n,3,S,S] -> bf16 patches [n*(S/p)^2, kpad].
 * Replaces the Conv2d(k=s=patch) input side of SiglipVisionEmbeddings /
 * CLIPVisionEmbeddings (TF:models/siglip/modeling_siglip.py:175-186). in_is_f32:1/0 */
int mme_im2col(const void* pixels, int in_is_f32, int n, int S, int patch, int kpad, void* out,
               void* stream);

/* ---------------------------------------------------------------- a4/a5 ----
 * C[M,N] = act(A[M,K] . B[N,K]^T + bias[N]) + residual[r(row), N]
 * r(row) = row if res_period == 0 else row % res_period (position-table add).
 * Replaces nn.Linear / Conv2d GEMMs of the SigLIP / CLIP towers
 * (TF:models/siglip/modeling_siglip.py:268-322, TF:models/clip/modeling_clip.py).
 * bf16 in, fp32 accumulate (MFMA 16x16x32), bf16 out (or fp32 if out_f32).
 * Requires K % 64 == 0, lda/ldb % 8 == 0 and 16-B aligned A/B rows (C/residual: any ld).
 * act == MME_ACT_GEGLU_TANH (GemmaMLP act_fn(gate_proj(x)) * up_proj(x),
 * TF:models/gemma/modeling_gemma.py:95-96): B holds gate and up rows interleaved in
 * groups of 4 (rows 8k..8k+3 = gate 4k..4k+3, rows 8k+4..8k+7 = up 4k..4k+3), and
 * C[r, 4k+e] = bf16( bf16(gelu_tanh(bf16 g)) * bf16 u ) is [M, N/2] (N % 8 == 0,
 * ldc % 4 == 0, no residual, bf16 out). */
int mme_gemm(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
             const void* bias, const void* residual, int ldr, int res_period, int act, int out_f32,
             void* stream);

/* GEMM with the preceding LayerNorm folded into the weights: for
 * LN(x) = (x - mean) * rstd * gamma + beta feeding nn.Linear(W, b),
 *   C[r, n] = act( rstd_r * (A[r,:] . B[n,:] - mean_r * col_sum[n]) + bias_f32[n] )
 * with A = x (the un-normalised residual stream), B = bf16(W * gamma) (per input
 * column), col_sum[n] = sum_k B[n, k] (fp32) and bias_f32 = b + W . beta (fp32);
 * row_stats = [M][2] (mean, rstd) from mme_rowstats. Replaces the
 * LayerNorm -> Linear pairs of SiglipEncoderLayer / CLIPEncoderLayer
 * (TF:models/siglip/modeling_siglip.py:341-357, layer_norm1 -> q/k/v_proj and
 * layer_norm2 -> mlp.fc1) without writing the normalised rows. act: NONE .. GELU_ERF;
 * bf16 out; same shape rules as mme_gemm. */
int mme_gemm_lnfold(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                    const float* row_stats, const float* col_sum, const float* bias_f32, int act, void* stream);

/* Residual GEMM that also leaves the next LayerNorm's statistics: C = A . B^T + bias +
 * residual (bf16, as mme_gemm with res_period 0, act NONE) and row_stats = [M][2]
 * (mean, rsqrt(var + eps)) of the bf16 rows of C, i.e. what mme_rowstats(C) returns
 * up to fp32 summation order. The pipelined kernel's epilogue reduces each 64-column
 * slice of every output row two-pass into row_part = [M][N / 64][2] (mean, M2;
 * caller-provided scratch) and a per-row pass combines the slices (Chan), so the
 * residual stream is not re-read. Replaces the o_proj / fc2 residual adds followed by
 * layer_norm2 / the next layer's layer_norm1 (TF:models/siglip/modeling_siglip.py:341-357)
 * on the LayerNorm-folded path. N % 64 == 0. */
int mme_gemm_res_stats(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                       const void* bias, const void* residual, int ldr, float eps, float* row_part,
                       float* row_stats, void* stream);

/* LayerNorm statistics per row: stats[2r] = mean, stats[2r+1] = rsqrt(var + eps)
 * (fp32, biased variance; the arithmetic of mme_layernorm) for mme_gemm_lnfold. */
int mme_rowstats(const void* x, int ldx, int rows, int d, float eps, float* stats, void* stream);

/* LayerNorm over the last dim (fp32 statistics), bf16 in/out.
 * y[r] = (x[r]-mean)*rsqrt(var+eps)*gamma + beta. Replaces nn.LayerNorm
 * (TF:models/siglip/modeling_siglip.py:329-331). If `rows_idx` is non-null,
 * output row r reads input row rows_idx[r] (fused gather for pooling). */
int mme_layernorm(const void* x, int ldx, const void* gamma, const void* beta, void* y, int ldy, int rows,
                  int d, float eps, const int32_t* rows_idx, void* stream);

/* Multi-head attention softmax(Q K^T * scale + mask) V over packed QKV rows.
 * qkv: bf16 [B*T, ld_qkv], Q at column 0, K at H*hd, V at 2*H*hd; head h at h*hd.
 * out: bf16 [B*T, ld_out], head h at column h*hd.
 * seq_lens (int32[B], nullable): key padding (keys >= len masked).
 * causal: keys > query masked (CLIP text, TF:models/clip/modeling_clip.py:543-555).
 * hd in {64, 72, 80}. Replaces eager/SDPA attention (TF:…siglip.py:228-247). */
int mme_attention(const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H, int hd,
                  const int32_t* seq_lens, int causal, float scale, void* stream);

/* mme_attention with Q pre-scaled (ABI 9): the Q columns of qkv already hold q * scale * log2(e)
 * (mme/ops.py LNFolded(row_scale=...) folds the factor into the Q rows of the projection before its
 * single bf16 rounding), so the kernels compute exp2(Q'K^T - M) and hd 72 runs kind 98, whose QK^T
 * MFMA also subtracts the running max (Q^T row 72 = -M against a ones row of K): the per-score FMA of
 * the softmax goes. Same masks, outputs and errors as mme_attention. */
int mme_attention_qs(const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H, int hd,
                     const int32_t* seq_lens, int causal, void* stream);

/* Per-call kernel forms (ABI 8; bit-identity tests and A/B measurements). Each takes the
 * arguments of its plain entry point after an int `form`; the library holds no switch
 * (the plain entry points always run the production dispatch):
 *   mme_gemm_form / mme_gemm_lnfold_form / mme_gemm_res_stats_form: -1 = production,
 *     47 = pipe6 (the bit-identity reference of pipe8 / pipe9), 48 = the per-row statistics
 *     combine (res_stats); other forms exist in the development build (libmme_dev.so) only;
 *   mme_attention_form: 0 = production, 30 + kind = kernel kind `kind` (production: 16 T <= 64, 102 hd 64 with
 *     64 < T <= 128 (round 6: the CLIP causal text towers), 83 hd 72, 86 / 87 hd 80, 89 hd 64; through mme_attention_qs(_form) 98 hd 72, 101 / 100 hd 80 -- 97 and 99 are
 *     measured forms, 99-101 need Q pre-scaled; 94 = the persistent form of 86, measured and not dispatched);
 *   mme_gemm_mx_form (below): -1 = production (mx11 where its geometry holds -- with the bias loaded up
 *     front, the mx8 block absmax by DPP and quick_gelu in packed f32 where N % 4 == 0 (form 17) -- else
 *     mx10), 11 = mx11 without those, 10 = mx10, 0 / 2 / 3 = earlier forms, 15 = mx11 with the
 *     bias loaded up front alone (N % 4 == 0, 8-B aligned bias), 16 = production there until round 6, 17 = 16 with
 *     the mx8 output packed without the inactive clamp (what production runs there since round 6);
 *     12 / 14 = mx12 (persistent mx11 with / without the next tile's DMA under the epilogue; measured
 *     slower, not dispatched) exist in the development build only;
 *   two NON-dispatched GEMM forms stay in the production build on purpose, because production-suite
 *     bit-identity tests and A/B runs select them: mme_gemm_form 95 = pipe10 on every non-split GEMM
 *     (measured slower) and 93 = the production kernels with their epilogues branching on the operands
 *     at run time (the dispatch before round 5's compiled epilogues; bit-identical, slower). The plain
 *     entry points never run them. */
int mme_gemm_form(int form, const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                  const void* bias, const void* residual, int ldr, int res_period, int act, int out_f32,
                  void* stream);
int mme_gemm_lnfold_form(int form, const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N,
                         int K, const float* row_stats, const float* col_sum, const float* bias_f32, int act,
                         void* stream);
int mme_gemm_res_stats_form(int form, const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N,
                            int K, const void* bias, const void* residual, int ldr, float eps, float* row_part,
                            float* row_stats, void* stream);
int mme_attention_form(int form, const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H, int hd,
                       const int32_t* seq_lens, int causal, float scale, void* stream);
int mme_attention_qs_form(int form, const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H, int hd,
                          const int32_t* seq_lens, int causal, void* stream);

/* SigLIP MAP pooling-head attention: one probe query per head against the
 * T keys/values of each image. q: bf16 [H*hd] (already projected);
 * kv: bf16 [B*T, ld_kv], K at col 0, V at col H*hd. out: bf16 [B, ld_out].
 * Replaces nn.MultiheadAttention in SiglipMultiheadAttentionPoolingHead
 * (TF:models/siglip/modeling_siglip.py:622-644). */
int mme_probe_attention(const void* q, const void* kv, int ld_kv, void* out, int ld_out, int B, int T, int H,
                        int hd, float scale, void* stream);

/* SigLIP MAP pooling head with the probe query absorbed into the key projection
 * (round 3): S: fp32 [B*T, ld_s] = x . [U_hi; U_lo]^T, the two bf16 halves of
 * U_h = W_k,h^T q_h / sqrt(hd) (cols 0..H-1 and H..2H-1); x: bf16 [B*T, ld_x], the
 * post-LayerNorm tokens. out: bf16 [B*H, ld_out], row b*H + h = sum_t softmax_t(S_h) x_t
 * over the first D columns; W_v,h (out row) + b_v,h then gives the head's attention output.
 * T <= 1024, H <= 16, D even <= 1152. Replaces the K / V projections and the attention of
 * SiglipMultiheadAttentionPoolingHead (TF:models/siglip/modeling_siglip.py:622-644). */
int mme_map_pool(const float* S, int ld_s, const void* x, int ld_x, void* out, int ld_out, int B, int T, int H,
                 int D, void* stream);

/* out[b*L + t, :] = tok[ids[b,t]] + pos[t] (bf16). Replaces SiglipTextEmbeddings /
 * CLIPTextEmbeddings (TF:models/siglip/modeling_siglip.py:189-224). */
int mme_token_embed(const int64_t* ids, int B, int L, const void* tok, const void* pos, int d, void* out,
                    int ld_out, void* stream);

/* CLIP vision embedding assembly + pre_layrnorm (fused):
 * x[b,0] = cls + pos[0]; x[b,1+p] = patch[b*P+p] + pos[1+p]; y = LN(x).
 * Replaces CLIPVisionEmbeddings.forward + pre_layrnorm (TF:…clip.py:203-218,642). */
int mme_clip_embed_ln(const void* patch, int ld_patch, const void* cls, const void* pos, const void* gamma,
                      const void* beta, float eps, void* out, int ld_out, int B, int P, int d, void* stream);

/* Pooling positions for text towers: pos[b] = first t with ids[b,t]==eos_id
 * (mode 0), argmax_t ids[b,t] (mode 1, legacy eos_token_id==2 configs), or
 * L-1 (mode 2, SigLIP last position TF:…siglip.py:539). Output is the ROW
 * index b*L + pos. Replaces TF:models/clip/modeling_clip.py:561-581. */
int mme_text_pool_rows(const int64_t* ids, int B, int L, int64_t eos_id, int mode, int32_t* rows_out,
                       void* stream);

/* ---------------------------------------------------------------- a6 ----
 * y = bf16( x / bf16( sqrt( sum_fp32 x^2 ) ) ) per row — the exact semantics of
 * `out / out.norm(dim=-1, keepdim=True)` on a bf16 tensor (main.py:414,434). */
int mme_l2norm(const void* x, int ldx, void* y, int ldy, int rows, int d, void* stream);

/* ---------------------------------------------------------------- a7/a9 ----
 * Fused similarity + row top-k:
 *   S = Q[nq,D] . Db[nd,D]^T (fp32 acc), keep the k best columns per row,
 *   ordered (score desc, column asc).  k <= 16, D % 64 == 0.
 * Replaces torch.matmul at main.py:473 + torch.topk at main.py:335,365,375.
 * workspace >= mme_sim_topk_workspace_bytes(nq, nd, k). */
size_t mme_sim_topk_workspace_bytes(int nq, int nd, int k);
int mme_sim_topk(const void* Q, int ldq, const void* Db, int ldd, int nq, int nd, int D, int k, int col_offset,
                 int32_t* out_idx, float* out_score, void* workspace, size_t ws_bytes, void* stream);

/* Merge `parts` sorted top-k lists per row (e.g. per-rank partial results):
 * in_idx/in_score [rows, parts*k] -> out [rows, k], order (score desc, idx asc). */
int mme_topk_merge(const int32_t* in_idx, const float* in_score, int rows, int parts, int k, int32_t* out_idx,
                   float* out_score, void* stream);

/* Row top-k of a materialised fp32 score matrix S [rows, ld] (first `cols` columns):
 * out [rows, k], order (score desc, column asc), indices + col_offset. k <= 16.
 * Replaces torch.topk at main.py:335,365,375 on the MaxSim (ColPali) score matrices. */
int mme_topk_rows(const float* scores, int ld, int rows, int cols, int k, int col_offset, int32_t* out_idx,
                  float* out_score, void* stream);

/* Row top-k in torch.topk's CPU order (main.py:335,365,375: torch.topk(row, k) per row).
 * torch's CPU kernel (aten SortingKernel.cpp topk_impl_loop) selects with libstdc++'s
 * std::partial_sort when k * 64 <= cols, else std::nth_element + std::sort of the first
 * k - 1, comparing values only: exact ties (ColPali's bf16-quantised MaxSim sums) come
 * out in that algorithm's order, which this replays step for step. Same arguments as
 * mme_topk_rows; workspace >= mme_topk_rows_torch_workspace_bytes (0 when k * 64 <= cols). */
size_t mme_topk_rows_torch_workspace_bytes(int rows, int cols, int k);
int mme_topk_rows_torch(const float* scores, int ld, int rows, int cols, int k, int col_offset, int32_t* out_idx,
                        float* out_score, void* workspace, size_t ws_bytes, void* stream);

/* Bootstrap resampling (§8f-3; run_bootstrap_benchmark main.py:586-634): the score
 * matrices of B resamples as index gathers of the full matrices,
 *   out[b][i][p] = S[rows[b*R + i]][g * cols[b*C + p/g] + p % g],   out fp32 [B*R, C*g]
 * (T2I: S = full T2I, rows = cols = sample, g = 1; I2T: S = full I2T, g = 5; I2T-Sym:
 * S = T2I transposed). ld = row stride of S in elements. */
int mme_gather_scores(const float* S, long ld, const int32_t* rows, const int32_t* cols, int B, int R, int C, int g,
                      float* out, void* stream);

/* Recall hits per resample: row r (of B groups of R rows) targets columns
 * [(r % R) * tgt_count, +tgt_count); hits [B, nk] += rows whose first kk[j] indices hold a target. */
int mme_recall_hits_groups(const int32_t* topk_idx, int rows, int k, int R, int tgt_count, const int32_t* kk, int nk,
                           int64_t* hits, void* stream);

/* Winoground 2x2 scores (§8f-4; run_winoground, run_benchmark_grand_slam_v28_publication_ready.py:413-461):
 * text, image: bf16 [n, 2, D] L2-normalised embeddings of (caption_0, caption_1) and (image_0, image_1).
 * scores: fp32 [n, 4] = bf16(<t_a, i_b>) for (a,b) = 00, 01, 10, 11 (the bf16 torch.matmul);
 * counts[0..2] += text / image / group successes (strict comparisons of the reference).
 * counts must be zeroed by the caller. */
int mme_winoground(const void* text, const void* image, int n, int D, float* scores, int64_t* counts, void* stream);

/* Recall hit counts. For row r the targets are columns
 *   [tgt_start[r], tgt_start[r] + tgt_count)   (tgt_start nullable -> (r + row_offset)*tgt_count)
 * hits[j] += #rows whose first kk[j] indices contain a target, j < nk; rows with
 * skip[r] != 0 are not counted (skip nullable; ABI 8: the rows re-ranked in torch's order).
 * Replaces the counting loops of compute_metrics_detailed (main.py:331-378). */
int mme_recall_hits(const int32_t* topk_idx, int rows, int k, const int32_t* tgt_start, int tgt_count,
                    int row_offset, const int32_t* kk, int nk, const uint8_t* skip, int64_t* hits, void* stream);

/* Exact score ties on the dense path (ABI 8). torch.topk (main.py:335,365,375) orders EXACTLY
 * tied values as its libstdc++ selection leaves them, not by column; only rows whose sorted
 * top-(k+1) holds two equal neighbours can differ from mme_sim_topk's (score desc, column asc)
 * order (duplicated images / captions tie in every row).
 *   mme_tie_rows:   flags[r] = 1 iff scores[r][j] == scores[r][j-1] for some 0 < j < k
 *                   (scores [rows, k] = a sorted mme_sim_topk table).
 *   mme_sim_scores: out[r][c] = Q[r] . Db[c] fp32 [nq, ldo], through mme_sim_topk's own main
 *                   loop, so every score is bit-identical to the one it ranked; the flagged rows
 *                   are re-selected from these by mme_topk_rows_torch, once per k. */
int mme_tie_rows(const float* scores, int rows, int k, uint8_t* flags, void* stream);
int mme_sim_scores(const void* Q, int ldq, const void* Db, int ldd, int nq, int nd, int D, float* out, long ldo,
                   void* stream);

/* ---------------------------------------------------------------- a8 ----
 * ColPali late-interaction MaxSim (colpali_engine processor.score,
 * main.py:467; in-container port TF:models/colpali/processing_colpali.py:256-270):
 *   score[q,d] = bf16( sum_{i<q_len} bf16( max_{j<d_len} <Q[q,i], D[d,j]> ) )
 * Q: bf16 [nq, Lq, dim], D: bf16 [nd, Ld, dim] (rows beyond the lengths ignored),
 * d_zero (u8[nd], nullable): 1 -> the doc was zero-padded in the reference's
 * chunk, so 0 joins its max (pad_sequence semantics). dim == 128, Ld % 16 == 0.
 * out: fp32 [nq, nd]. workspace >= mme_maxsim_workspace_bytes(nq, Lq, nd). */
size_t mme_maxsim_workspace_bytes(int nq, int Lq, int nd);
int mme_maxsim(const void* Q, const int32_t* q_lens, int nq, int Lq, const void* D, const int32_t* d_lens,
               const uint8_t* d_zero, int nd, int Ld, int dim, float* out, void* workspace, size_t ws_bytes,
               void* stream);

/* ------------------------------------------------------- config 5: fp8 ----
 * MX-fp8 encoder GEMMs ("Apple-DFN5B-H fp8 weights on CDNA4 fp8 MFMA",
 * BASELINE.json configs[4]; the reference runs the same CLIP layers in bf16,
 * TF:models/clip/modeling_clip.py CLIPAttention q/k/v + CLIPMLP fc1/fc2).
 * mx8 tensor: values u8 [rows][k] e4m3fn (row stride ld bytes) + E8M0 scale
 * bytes [k/32][rows_pad] (block-major planes, rows_pad % 256 == 0); since ABI 8 row r's
 * byte of plane b sits at column srow(r) = (r & ~127) | (r & 31) << 2 | (r >> 5) & 3 (the
 * four rows i*32 + r of one MFMA lane in one aligned dword, loaded by one buffer_load_dword);
 * element (r,c) = e4m3(q[r][c]) * 2^(S[c/32][srow(r)] - 127). Block rule: absmax a,
 * S = clamp(expfield(a) - 8 + (mantissa(a) > 0x600000), 1, 254) (127 when a == 0),
 * q = RNE_e4m3(clamp(x * 2^(127-S), +-448)).  */

/* bf16 rows [rows, k] (k % 32 == 0) -> mx8. */
int mme_mx_quant(const void* x, int ldx, int rows, int k, void* q, int ldq, void* scales, int rows_pad, void* stream);

/* mme_layernorm (same statistics, output rounded to bf16) -> mx8 (d % 32 == 0). */
int mme_layernorm_mx(const void* x, int ldx, const void* gamma, const void* beta, int rows, int d, float eps,
                     const int32_t* rows_idx, void* q, int ldq, void* scales, int rows_pad, void* stream);

/* C = act(A . B^T + bias) (+ residual[row % res_period or row]) with A [M,K], B [N,K] in mx8
 * (sa_rows / sb_rows = their planes' rows_pad), fp32 accumulation on the block-scaled
 * MFMA. out_mx == 0: C bf16 [M, ldc elements]; out_mx == 1: C re-quantised to mx8
 * (values [M, ldc bytes], scale planes c_scales with c_rows_pad rows; N % 32 == 0, no
 * residual) -- fc1's output as fc2's operand. K % 64 == 0, lda/ldb % 16 == 0. */
int mme_gemm_mx(const void* A, int lda, const void* sa, int sa_rows, const void* B, int ldb, const void* sb,
                int sb_rows, void* C, int ldc, void* c_scales, int c_rows_pad, int M, int N, int K, const void* bias,
                const void* residual, int ldr, int res_period, int act, int out_mx, void* stream);
int mme_gemm_mx_form(int form, const void* A, int lda, const void* sa, int sa_rows, const void* B, int ldb,
                     const void* sb, int sb_rows, void* C, int ldc, void* c_scales, int c_rows_pad, int M, int N,
                     int K, const void* bias, const void* residual, int ldr, int res_period, int act, int out_mx,
                     void* stream);

/* ------------------------------------------------ §8f-1: ColPali encoder ----
 * ColPali-v1.3 = PaliGemma-3B (SigLIP-448 vision tower + Gemma-2B) + 128-d head,
 * the model behind the colpali branch of encode_data (main.py:402-405,422-425;
 * in-container port TF:models/colpali/modeling_colpali.py:107-146). The vision
 * tower and every GEMM reuse the entry points above; these are the Gemma pieces. */

/* GemmaRMSNorm (TF:models/gemma/modeling_gemma.py:64-78):
 * y = bf16( x * rsqrt(mean_fp32(x^2) + eps) * (unit_offset + w) ), unit_offset 1 = Gemma's (1 + w).
 * rows_idx (nullable): output row r reads input row rows_idx[r]. d <= 2048, d % 8 == 0. */
int mme_rmsnorm(const void* x, int ldx, const void* w, void* y, int ldy, int rows, int d, float eps,
                int unit_offset, const int32_t* rows_idx, void* stream);

/* Rotary position embedding, in place on heads [0, nheads) of packed rows
 * (q heads then the k head; GemmaRotaryEmbedding + apply_rotary_pos_emb,
 * TF:models/gemma/modeling_gemma.py:100-187): position = (row % T) + pos_offset
 * (PaliGemma: 1, TF:models/paligemma/modeling_paligemma.py:234-237); cos/sin in fp32
 * rounded to bf16, each product and the sum rounded to bf16 as the bf16 module does. */
int mme_rope(void* qkv, int ld, int rows, int T, int nheads, int hd, int pos_offset, float theta, void* stream);

/* Gemma decoder input: rows t < P of each length-L sequence take image feature
 * img[b*P + t] (PaliGemma masked_scatter, the <image> tokens lead a ColPali sequence,
 * TF:models/paligemma/modeling_paligemma.py:231-246), rows t >= P take
 * bf16(tok[ids[b,t]] * scale) (GemmaTextScaledWordEmbedding, scale = bf16(sqrt(d))). */
int mme_gemma_embed(const int64_t* ids, int B, int L, const void* tok, int d, float scale, const void* img,
                    int ld_img, int P, void* out, int ld_out, void* stream);

/* ColPali head tail: y = bf16( bf16(x / bf16(||x||)) * mask[row] ) (mask: int64
 * attention_mask rows, nullable = all ones; TF:models/colpali/modeling_colpali.py:136-140). */
int mme_l2norm_masked(const void* x, int ldx, void* y, int ldy, int rows, int d, const int64_t* mask,
                      void* stream);

/* Multi-query attention, head dim 256, ONE shared K/V head (Gemma-2B, Hq in {1,2,4,8};
 * GemmaAttention, TF:models/gemma/modeling_gemma.py:202-292). qkv: bf16 [B*T, ld_qkv],
 * q head h at column h*256, K at Hq*256, V at (Hq+1)*256. Bidirectional (PaliGemma
 * prefix attention, use_bidirectional_attention); keys valid in [kstart[b], kend[b])
 * (nullable -> [0, T); left padding -> kstart = pad count), kend > kstart.
 * out: bf16 [B*T, ld_out], head h at column h*256. */
int mme_attention_mqa(const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int Hq, int hd,
                      const int32_t* kstart, const int32_t* kend, float scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MME_H_ */

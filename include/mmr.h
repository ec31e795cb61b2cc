/* libmmr — MI355X (gfx950) joint-embedding retrieval hot path behind a C ABI.
 *
 * Every entry point takes plain pointers + sizes (no torch types), returns an mmr_status and, on
 * failure, leaves a message in the thread-local mmr_last_error().  No exceptions cross the ABI.
 * Ownership: the caller owns every input/output buffer (device pointers unless a parameter says
 * host); the library owns mmr_index state and its workspaces.  Launches are asynchronous on the
 * caller's HIP stream (`stream` = hipStream_t, NULL = default stream).
 *
 * Reference interfaces replaced (file:line in ppddddpp/multi-modal-retrieval-predict-project):
 *   mmr_index_create   RetrievalEngine.__init__  src/Retrieval/retrieval.py:24-32
 *                      (np.load(...).astype(float32) -> self.embs (N,D)); norms precomputed once
 *                      instead of sklearn normalize() per call (retrieval.py:128).
 *   mmr_index_search   exact brute-force top-K: sklearn cosine_similarity + np.argsort(...)[::-1][:K]
 *                      src/Evaluate/retrieval_overlap.py:84-90, src/Retrieval/retrieval.py:128-137;
 *                      reached via RetrievalEngine.retrieve retrieval.py:34-39.
 *   mmr_merge_topk     (new) k-way merge of per-shard top-K lists after the RCCL all-gather.
 *   tower ops          timm SwinTransformer.forward_features (src/Model/fusion.py:198-199),
 *                      HF BertModel(...).last_hidden_state (fusion.py:322-325), heads
 *                      src/Model/model.py:365-373,462-479; see the per-function comments.
 */
#ifndef MMR_H
#define MMR_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  MMR_OK = 0,
  MMR_ERR_INVALID = 1,     /* bad argument (shape, null pointer, unsupported K/D) */
  MMR_ERR_HIP = 2,         /* a HIP runtime call failed */
  MMR_ERR_OOM = 3,         /* device allocation failed */
  MMR_ERR_UNSUPPORTED = 4, /* dtype / geometry not built */
  MMR_ERR_CAPACITY = 5     /* a per-query candidate buffer overflowed (see out_status) */
} mmr_status;

typedef enum { MMR_F32 = 0, MMR_F16 = 1, MMR_BF16 = 2 } mmr_dtype;

typedef struct mmr_index mmr_index;

const char* mmr_last_error(void);
int mmr_version(void);
int mmr_max_k(void);

/* ---------------------------------------------------------------- gallery index (kNN) */
/* Copy an (n, d) row-major gallery (host pointer if `gallery_is_host`, else device) into a
 * library-owned device layout on `device`, computing per-row inverse norms (f32) and norms (f64).
 * `idx_base` is added to every returned index (row-sharded galleries: global = local + base).
 * dtype MMR_F32: f32 rows (every scan mode).  MMR_F16: a native fp16 index — the raw fp16 rows are its only
 * device copy (2 B per element + f32 inverse norms + f64 norms per row), scanned in mode 2 only (its exact
 * f64 re-score reads the same rows: fp16 is exact in f64), results bit-identical to an MMR_F32 index of the
 * f32-upcast rows; mmr_index_set_mode(0 / 1) returns MMR_ERR_UNSUPPORTED.  MMR_BF16: not built. */
mmr_status mmr_index_create(const void* gallery, int64_t n, int32_t d, mmr_dtype dtype,
                            int gallery_is_host, int64_t idx_base, int device, mmr_index** out);
mmr_status mmr_index_destroy(mmr_index* index);
mmr_status mmr_index_info(const mmr_index* index, int64_t* n, int32_t* d, int64_t* idx_base);
/* Device bytes the index holds: gallery_bytes = the rows + norms + the scan copies of the current mode.
 * MMR_F32 index: f32 rows (4 B per element) + the current mode's copies (x3: bf16 hi/lo split + tile16 f32,
 * 8 B per element; f16: ONE fp16 unit-row copy in the tile32h layout, 2 B per element; f32: none — copies
 * of other modes are freed at a mode switch).  MMR_F16 index: the fp16 rows only (2 B per element).
 * workspace_bytes = the query / per-unit-maxima workspace.  Either pointer may be NULL. */
mmr_status mmr_index_device_bytes(const mmr_index* index, int64_t* gallery_bytes, int64_t* workspace_bytes);
/* Pre-allocate the workspace for up to `max_q` queries in the CURRENT scan mode so that later
 * searches allocate nothing (required before capturing a search into a HIP graph). */
mmr_status mmr_index_reserve(mmr_index* index, int64_t max_q);

/* Scan precision of the candidate pass (the ranking is always exact f64): 0 = f32 MFMA,
 * 1 = bf16 3-term split MFMA (default; ~5x the f32 rate at the same bytes; queries chunks of
 * <= 32 take the HBM-streaming f32 skinny scan), 2 = fp16 unit-row copy of the gallery (built on
 * the first switch to this mode: half the scan bytes, one fp16 MFMA per product, a wider candidate
 * margin — the same exact results). */
mmr_status mmr_index_set_mode(mmr_index* index, int32_t mode);

/* Exact cosine top-K of q (q, d) f32 device queries against the gallery.
 * Semantics: s(q,g) = <q,g> / (|q| |g|) in f64 (0 when either norm is 0 — sklearn's normalize()
 * leaves zero rows at 0), ranked by score descending, ties by lower gallery index.  Outputs
 * (q, k) int64 indices (+idx_base) and f32 scores; slots beyond n are (-1, -inf).
 * out_status (q,) int32 (may be NULL): per-query status, always 0 — more candidates inside the scan
 * margin than the selection buffer holds (massive near-ties) are merged batch by batch inside the
 * selection kernel, exactly, never truncated (a non-zero value would flag an inexact list).
 * Asynchronous on `stream`.  Threading: calls on one index may come from several host threads and
 * several streams; the index's workspace follows the stream (a search on a new stream first waits
 * for the previous search's last use), so concurrent searches serialise on the device but never race.
 * The hand-over event is recorded on the previous search's stream at the switch (not after every
 * search: a per-search event record cost 3-5 us of device time), so that stream must still exist
 * when a search on another stream, or a workspace growth, follows. */
mmr_status mmr_index_search(mmr_index* index, const float* q, int64_t nq, int32_t k,
                            int64_t* out_idx, float* out_score, double* out_score64,
                            int32_t* out_status, void* stream);
/* out_score64 (q, k) f64 (may be NULL): the exact scores the ranking used; the shard merge ranks
 * on these so a row-sharded search returns exactly the single-device result. */

/* DLS link graph (DLSRetrievalEngine._build_link_graph, src/Retrieval/retrieval.py:121-138): the
 * self-join of gallery rows [row0, row0+nrows) against the whole index — per row its neighbours
 * in exact-cosine order (score desc, index asc), the row itself excluded (the reference's diagonal
 * -1), score >= threshold, at most max_links.  out_nbr (nrows, max_links) int64 LOCAL row indices,
 * -1 padded; out_cnt (nrows,) int32.  Device buffers, asynchronous on `stream`. */
mmr_status mmr_index_link_graph(mmr_index* index, double threshold, int32_t max_links, int64_t row0,
                                 int64_t nrows, int64_t* out_nbr, int32_t* out_cnt, void* stream);

/* KG / label reranker fused after the top-K (Reranker.rerank, src/Retrieval/reranker.py:240-333):
 * per query the kc candidates cand (nq, kc) int64 (global indices into this index, -1 = empty,
 * kc <= 64) are re-scored with alpha*minmax(cos(q_emb, row)) + beta*minmax(Jaccard(label sets)) +
 * gamma*minmax(cos(kg vectors)) — cosines in f64, 0 for a zero norm — and the first topk written
 * in final-score order (equal finals: later candidate first, as np.argsort(final)[::-1]).
 * q_emb (nq, d) f32; q_labels (nq) / g_labels (n) uint64 label bitsets; q_kg (nq, dk) /
 * g_kg (n, dk) f32 record KG vectors (g_* in local row order).  Outputs (nq, topk): out_idx int64
 * (-1 beyond the valid candidates), optional out_final / out_emb / out_lab / out_kg f64 (the
 * scaled components, like the reference's result tuples). */
mmr_status mmr_index_rerank(const mmr_index* index, const float* q_emb, int64_t nq, const int64_t* cand,
                            int32_t kc, const uint64_t* q_labels, const uint64_t* g_labels, const float* q_kg,
                            const float* g_kg, int32_t dk, double alpha, double beta, double gamma,
                            int32_t topk, int64_t* out_idx, double* out_final, double* out_emb,
                            double* out_lab, double* out_kg, void* stream);

/* Merge n_lists per-shard lists laid out [n_lists][nq][k_in] (f64 scores, int64 idx; empty slots
 * idx -1) into the global top-k_out per query: score desc, then index asc.  out_score f32 (may be
 * NULL), out_score64 f64 (may be NULL). */
mmr_status mmr_merge_topk(const double* scores, const int64_t* idx, int32_t n_lists, int64_t nq,
                          int32_t k_in, int32_t k_out, int64_t* out_idx, float* out_score,
                          double* out_score64, void* stream);
/* mmr_merge_topk over queries [q0, q0 + nq) of lists laid out [n_lists][nq_total][k_in] (a rank
 * merges only its own queries after the all-gather), with an optional f64 payload of
 * payload_width (<= 16) values per entry, [n_lists][nq_total][k_in][width], carried into
 * out_payload [nq][k_out][width] (zeros for empty slots).  payload and out_payload are both NULL or
 * both set.  The sharded rerank's per-candidate components ride here (reranker.py:240-333 needs
 * them over the MERGED candidate list). */
mmr_status mmr_merge_topk_payload(const double* scores, const int64_t* idx, const double* payload,
                                  int32_t payload_width, int32_t n_lists, int64_t nq_total, int64_t q0,
                                  int64_t nq, int32_t k_in, int32_t k_out, int64_t* out_idx, float* out_score,
                                  double* out_score64, double* out_payload, void* stream);

/* mmr_merge_topk_payload over ONE packed all-gather buffer (the sharded search's single collective,
 * SURVEY.md §8e): packed = [n_lists][nq_total][k_in][2 + payload_width] 8-byte words per entry =
 * {f64 score, int64 global index (-1 = empty), payload_width f64 payload values}; merges queries
 * [q0, q0 + nq) (score desc, index asc) into out_idx / out_score / out_score64 / out_payload
 * [nq][k_out][payload_width] (each output but out_idx may be NULL). */
mmr_status mmr_merge_topk_packed(const void* packed, int32_t payload_width, int32_t n_lists, int64_t nq_total,
                                 int64_t q0, int64_t nq, int32_t k_in, int32_t k_out, int64_t* out_idx,
                                 float* out_score, double* out_score64, double* out_payload, void* stream);

/* Sharded KG / label rerank (Reranker.rerank, src/Retrieval/reranker.py:240-333, over a row-sharded
 * gallery).  Shard side: mmr_index_rerank_components writes, for each of this shard's candidates
 * cand (nq, kc) (global indices into this index, -1 = empty), the three RAW components
 * out_comp (nq, kc, 3) f64 = {emb cosine, label Jaccard, KG cosine} — the same f64 arithmetic as
 * mmr_index_rerank (zeros for an empty slot).  They travel with the (score, index) lists through
 * the all-gather and mmr_merge_topk_payload; mmr_rerank_mix then min-max scales them over the
 * merged list, mixes alpha/beta/gamma and ranks exactly as mmr_index_rerank does, so a sharded
 * rerank returns bit-identical results to the single-index one.  Arguments as mmr_index_rerank. */
mmr_status mmr_index_rerank_components(const mmr_index* index, const float* q_emb, int64_t nq,
                                       const int64_t* cand, int32_t kc, const uint64_t* q_labels,
                                       const uint64_t* g_labels, const float* q_kg, const float* g_kg,
                                       int32_t dk, double* out_comp, void* stream);
mmr_status mmr_rerank_mix(const int64_t* cand, const double* comp, int64_t nq, int32_t kc, double alpha,
                          double beta, double gamma, int32_t topk, int64_t* out_idx, double* out_final,
                          double* out_emb, double* out_lab, double* out_kg, void* stream);

/* ---------------------------------------------------------------- tower ops (bf16 = uint16) */
/* Y[m][n] = act(X[m][k] . W[n][k]^T + bias[n]) (+ R[m][n]); X, W, R, Y bf16; bias f32 or NULL;
 * act: 0 none, 1 GELU(erf).  nn.Linear semantics (weight [out][in]).  f32 accumulation. */
mmr_status mmr_linear_bf16(const uint16_t* x, const uint16_t* w, const float* bias,
                           const uint16_t* residual, uint16_t* y, int64_t m, int32_t n, int32_t k,
                           int32_t act, void* stream);

/* The launch variant mmr_linear_bf16 settled on for this shape / epilogue on the current device
 * (the first call per shape times the variants and keeps the fastest), or -1 before that call.
 * Diagnostic: lets a benchmark name the kernel it measured. */
int32_t mmr_linear_bf16_variant(int64_t m, int32_t n, int32_t k, int32_t act, int32_t has_bias,
                                int32_t has_residual);
/* The BERT linears with the residual LayerNorm folded in, so no LayerNorm pass runs between the
 * GEMMs of a layer (HF BertLayer: LN(dense(x) + residual), reference fusion.py:322-325 via BertModel).
 * Persistent 8-phase bf16 GEMM, 256-row tiles: m % 256 == 0, k % 128 == 0, n % 192 == 0 or n % 256 == 0.
 *   stats_out (optional, act == 0): per row, parts = mmr_linear_bf16_ln_parts(m, n, ln_mode) f32 pairs
 *     (sum, M2) of the bf16 outputs as stored — [m][parts][2]: part p covers the n / parts columns
 *     [p n / parts, (p + 1) n / parts) and M2 is its CENTRED sum of squares, sum (y - part mean)^2 (not
 *     a raw sum of squares); mmr_ln_row_coef merges the parts with Chan's parallel formula into the
 *     row's LayerNorm statistics (deterministic: one pair per tile column and wave column, no atomics).
 *   ln_mode 0: y = act(x W^T + bias) (+ residual).
 *   ln_mode 1: x is a raw residual-stream row y_in produced with stats, ln_coef = its mmr_ln_row_coef
 *     (f32 [m][2]); w = W diag(gamma) (bf16), ln_v1 = c = row sums of w (f32 [n]),
 *     bias = W beta + b:  y = act(LN(y_in) W^T + b) = act(rstd (y_in w^T) - rstd mean c + bias).
 *   ln_mode 2: residual is a raw row r produced with stats, ln_coef its coefficients; ln_v1 / ln_v2 =
 *     gamma / beta (f32 [n]):
 *     y = x W^T + bias + LN(r)  (n % 192 == 0).
 * Built: mode 1 with or without GELU (no residual, no stats); mode 2 with or without stats; mode 0
 * with stats, with or without a residual.  bias is required.  MMR_ERR_UNSUPPORTED otherwise. */
mmr_status mmr_linear_bf16_ln(const uint16_t* x, const uint16_t* w, const float* bias,
                              const uint16_t* residual, uint16_t* y, int64_t m, int32_t n, int32_t k,
                              int32_t act, int32_t ln_mode, const float* ln_coef, const float* ln_v1,
                              const float* ln_v2, float* stats_out, void* stream);

/* The row statistics of a producer (stats [m][nparts][2] = per part (sum, centred M2) over n / nparts
 * columns each, as mmr_linear_bf16_ln writes them; nparts even, n % nparts == 0 — checked) -> LayerNorm
 * coefficients coef [m][2] = (rstd, -mean rstd) over the row width n, rstd = 1 / sqrt(var + eps):
 * mean = sum_p sum_p / n, M2 = sum_p M2_p + (n / nparts) sum_p (mean_p - mean)^2 (Chan). */
mmr_status mmr_ln_row_coef(const float* stats, int64_t m, int32_t nparts, int32_t n, float eps, float* coef,
                           void* stream);

/* Row-statistics pairs per row mmr_linear_bf16_ln writes for an m x n output in ln_mode (0: not built). */
int32_t mmr_linear_bf16_ln_parts(int64_t m, int32_t n, int32_t ln_mode);

/* Number of launch variants mmr_linear_bf16 chooses among (indices 0 .. n-1 of its table). */
int32_t mmr_linear_bf16_n_variants(void);

/* Test / A-B hook (the product path never calls it): pin a launch variant for the whole process.
 *   MMR_PIN_GEMM_BF16: value = mmr_linear_bf16 variant index, or -1 = per-shape tuning (default);
 *   MMR_PIN_X3_WAVES:  value = 4 or 8 waves per mmr_linear_x3 tile (8 only where K % 256 == 0),
 *                      or -1 = automatic (default).
 *   MMR_PIN_X3_MLP:    value = 0 (8-wave workgroups) or 1 (4-wave workgroups, two per CU) for
 *                      mmr_x3_swin_mlp at C = 96, or -1 = automatic (1).  Both give bit-identical outputs.
 * MMR_ERR_INVALID for an unknown pin or value. */
enum { MMR_PIN_GEMM_BF16 = 0, MMR_PIN_X3_WAVES = 1, MMR_PIN_X3_MLP = 2 };
mmr_status mmr_pin_variant(int32_t which, int32_t value);

/* Resident-weight streaming linear for the short-K, narrow tower linears (Swin patch embed, stage-2
 * qkv / proj, PatchMerging 1->2; timm nn.Linear, reference fusion.py:198-199):
 * y = x @ W^T + bias (+ residual), K in {64, 192}.  W is kept in LDS for the whole launch, as
 * mmr_linear_rw_parts(n, k) parts of N / P channels, from an image built once by
 * mmr_linear_rw_pack (n * k bf16 elements, caller-allocated).  mmr_linear_rw_parts returns 0 for
 * shapes it does not take (then use mmr_linear_bf16). */
int32_t mmr_linear_rw_parts(int32_t n, int32_t k);
mmr_status mmr_linear_rw_pack(const uint16_t* w, int32_t n, int32_t k, uint16_t* img, void* stream);
mmr_status mmr_linear_rw(const uint16_t* x, const uint16_t* img, const float* bias, const uint16_t* residual,
                         uint16_t* y, int64_t m, int32_t n, int32_t k, void* stream);

/* Per-query f32 linears on bf16x3 MFMA (the multimodal head's per-vector chain, reference model.py:375-459):
 * y = act(x @ W^T + bias) (+ residual), x / y / residual f32 rows (strides ldx / ldy / ldr), W given as its
 * bf16 split W_hi = bf16(W), W_lo = bf16(W - W_hi) ([cout][cin] each); x is split the same way in
 * registers and each product summed as hi*hi + hi*lo + lo*hi in f32 (~2^-17 relative per product).
 * nbatch independent problems at element strides bsx / bsw / bsb / bsr / bsy (nbatch = 1: one linear).
 * cin % 128 == 0, cout % 32 == 0; residual may alias y. */
mmr_status mmr_linear_x3(const float* x, int64_t ldx, int64_t bsx, const uint16_t* w_hi, const uint16_t* w_lo,
                         int64_t bsw, const float* bias, int64_t bsb, const float* residual, int64_t ldr, int64_t bsr,
                         float* y, int64_t ldy, int64_t bsy, int32_t nbatch, int32_t b, int32_t cin, int32_t cout,
                         int32_t act, void* stream);

/* ---------------------------------------------------------------- MX-fp8 linears (config 5) */
/* Quantise bf16 x [rows][k] to OCP e4m3 q [rows][kp] (zero-padded, kp >= k, kp % 256 == 0) with one
 * E8M0 scale per 32 consecutive k of a row: 2^e, the smallest e with amax <= 448 * 2^e (no clipping);
 * q = RNE(x * 2^-e).  The scale bytes are written in the GEMM's per-lane LDS image order:
 * layout 0 (activations, rows % 256 == 0): [rows/256][kp/128][2][4][16][8] (1 byte per row-block);
 * layouts 1 / 2 (weights, rows % 192 / 256 == 0, for 256 x 192 / 256 x 256 GEMM tiles):
 * [rows/PR][kp/128][4][4][16][4] = rows/PR * kp/128 * 1024 bytes (PR = 192 / 256).  Replaces the bf16 operand of the Swin / BERT nn.Linear (fusion.py:198-199, 322-325) on the
 * fp8 tower path. */
mmr_status mmr_quantize_mxfp8(const uint16_t* x, int64_t rows, int32_t k, int32_t kp, int32_t layout,
                              uint8_t* q, uint8_t* scales, void* stream);

/* Y[m][n] = act(dequant(Xq) . dequant(Wq)^T + bias[n]) (+ R[m][n]) with gfx950 block-scaled MFMA
 * (v_mfma_scale_f32_16x16x128_f8f6f4, e4m3 x e4m3, f32 accumulation); Xq/xs from layout 0, Wq/ws
 * from layout w_layout (1 or 2) of mmr_quantize_mxfp8; Y, R bf16.  m % 256 == 0, kp % 256 == 0,
 * n % 192 == 0 (w_layout 1) or n % 256 == 0 (w_layout 2). */
mmr_status mmr_linear_mxfp8(const uint8_t* xq, const uint8_t* xs, const uint8_t* wq, const uint8_t* ws,
                            int32_t w_layout, const float* bias, const uint16_t* residual, uint16_t* y,
                            int64_t m, int32_t n, int32_t kp, int32_t act, void* stream);

/* mmr_linear_mxfp8 (weights in layout 2, no residual) whose output is written directly as the next
 * GEMM's MX-fp8 activation operand: yq [m][n] e4m3 + ys layout-0 scales (m/256 * n/128 * 1024 bytes),
 * bit-identical to mmr_quantize_mxfp8 of the bf16 output (BERT FFN1 -> FFN2, Swin fc1 -> fc2). */
mmr_status mmr_linear_mxfp8_q8(const uint8_t* xq, const uint8_t* xs, const uint8_t* wq, const uint8_t* ws,
                               const float* bias, uint8_t* yq, uint8_t* ys, int64_t m, int32_t n,
                               int32_t kp, int32_t act, void* stream);

/* LayerNorm(x (+ residual, may be NULL)) as mmr_layernorm_bf16 / mmr_add_layernorm_bf16, also
 * emitting the row as an MX-fp8 activation operand (q8 [rows][c] e4m3 + layout-0 scales,
 * rows % 256 == 0, c % 256 == 0), bit-identical to mmr_quantize_mxfp8 of y (the fp8 towers' QKV / FFN1
 * inputs). */
mmr_status mmr_layernorm_bf16_q8(const uint16_t* x, const uint16_t* residual, const float* gamma,
                                 const float* beta, uint16_t* y, uint8_t* q8, uint8_t* q8_scales, int64_t rows,
                                 int32_t c, float eps, void* stream);

/* mmr_layernorm_bf16_q8 with the operand's K padded to kp (kp % 256 == 0, kp >= c, c % 32 == 0; q8 is
 * [rows][kp], the padding written as zero bytes with zero scale bytes, bit-identical to
 * mmr_quantize_mxfp8(y, k=c, kp)), and y may be NULL when only the operand is consumed (the fp8 Swin
 * stages: C = 384 -> kp 512 for stage 3, C = 768 for stage 4). */
mmr_status mmr_layernorm_bf16_q8p(const uint16_t* x, const uint16_t* residual, const float* gamma,
                                  const float* beta, uint16_t* y, uint8_t* q8, uint8_t* q8_scales, int64_t rows,
                                  int32_t c, int32_t kp, float eps, void* stream);

/* Row LayerNorm over c channels (bf16 in/out, f32 math, gamma/beta f32). */
mmr_status mmr_layernorm_bf16(const uint16_t* x, const float* gamma, const float* beta,
                              uint16_t* y, int64_t rows, int32_t c, float eps, void* stream);

/* Post-LN residual block: y = LayerNorm(x + residual) (sum in f32), bf16 in / out.  BERT's
 * BertSelfOutput / BertOutput (HF modeling_bert; reference fusion.py:322-325 via AutoModel):
 * the attention-output and FFN2 GEMMs then need no residual epilogue. */
mmr_status mmr_add_layernorm_bf16(const uint16_t* x, const uint16_t* residual, const float* gamma,
                                  const float* beta, uint16_t* y, int64_t rows, int32_t c,
                                  float eps, void* stream);

/* y = LayerNorm(alpha * x + residual) with alpha a DEVICE f32 scalar (NULL = 1) and residual may be
 * NULL: PreFusionEnhancer's norm1(alpha * x + x2) (src/Model/fusion.py:34) on the vectorised
 * row kernel.  bf16 in / out, contiguous rows of c channels (c % 8 == 0). */
mmr_status mmr_scaled_add_layernorm_bf16(const uint16_t* x, const float* alpha, const uint16_t* residual,
                                         const float* gamma, const float* beta, uint16_t* y, int64_t rows,
                                         int32_t c, float eps, void* stream);

/* mmr_scaled_add_layernorm_bf16 that also writes y as the next GEMM's MX-fp8 activation operand
 * (q8 [rows][c] e4m3 + q8_scales in the layout-0 image, bit-identical to mmr_quantize_mxfp8 of y):
 * the fusion stack's enhanced tokens feeding the folded cross projections (config 5, fp8 towers).
 * rows % 256 == 0, c % 256 == 0. */
mmr_status mmr_scaled_add_layernorm_bf16_q8(const uint16_t* x, const float* alpha, const uint16_t* residual,
                                            const float* gamma, const float* beta, uint16_t* y, uint8_t* q8,
                                            uint8_t* q8_scales, int64_t rows, int32_t c, float eps, void* stream);

/* BERT embeddings (HF BertEmbeddings): LN(word[id] + pos[l] + type[0]) -> bf16 (b*l, c). */
mmr_status mmr_bert_embed(const int64_t* ids, const float* word, const float* pos,
                          const float* type0, const float* gamma, const float* beta, uint16_t* y,
                          int32_t b, int32_t l, int32_t c, float eps, void* stream);
/* mmr_bert_embed also writing y as the first QKV GEMM's MX-fp8 activation operand (q8 [b*l][c] e4m3 +
 * layout-0 scales), bit-identical to mmr_quantize_mxfp8 of y (the fp8 BERT tower; c % 256 == 0,
 * c <= 1024, b*l % 256 == 0).  q8 / q8_scales NULL = mmr_bert_embed. */
mmr_status mmr_bert_embed_q8(const int64_t* ids, const float* word, const float* pos, const float* type0,
                             const float* gamma, const float* beta, uint16_t* y, uint8_t* q8, uint8_t* q8_scales,
                             int32_t b, int32_t l, int32_t c, float eps, void* stream);

/* BERT self-attention core (HF BertSelfAttention, eval): qkv bf16 (b*l, 3*h*dh) [q|k|v],
 * additive mask from mask01 (b, l) int64 (0 -> masked), softmax(q k^T / sqrt(dh)) v -> ctx bf16
 * (b*l, h*dh).  Any l; dh % 8 == 0, dh <= 192 (the mmr_mha kernel with a key mask). */
mmr_status mmr_bert_attention(const uint16_t* qkv, const int64_t* mask01, uint16_t* ctx,
                              int32_t b, int32_t l, int32_t h, int32_t dh, void* stream);

/* mmr_bert_attention that writes the context as the O-proj GEMM's MX-fp8 activation operand (q8
 * (b*l, h*dh) e4m3 + q8_scales in the layout-0 image, bit-identical to mmr_quantize_mxfp8 of ctx);
 * ctx may be NULL (no bf16 copy).  Config 5's fp8 BERT: no quantise pass between attention and
 * O-proj.  dh % 32 == 0, (b*l) % 256 == 0, (h*dh) % 256 == 0. */
mmr_status mmr_bert_attention_q8(const uint16_t* qkv, const int64_t* mask01, uint16_t* ctx, uint8_t* q8,
                                 uint8_t* q8_scales, int32_t b, int32_t l, int32_t h, int32_t dh, void* stream);

/* Swin (shifted-)window attention core (timm WindowAttention + cyclic shift, eval):
 * qkv bf16 (b*hw*hw, 3*c) in natural token order; the kernel applies roll(-shift), window
 * partition, q*dh^-0.5, k^T, + the dense bias from mmr_swin_attn_bias, softmax, v, window reverse
 * and roll(+shift) -> out bf16 (b*hw*hw, c).  ws*ws <= 64, head_dim 32. */
mmr_status mmr_swin_window_attention(const uint16_t* qkv, const float* bias, uint16_t* out,
                                     int32_t b, int32_t hw, int32_t c, int32_t heads, int32_t ws,
                                     int32_t shift, void* stream);
/* mmr_swin_window_attention writing its output as the proj GEMM's MX-fp8 activation operand (q8
 * [b*hw*hw][kp] e4m3 + layout-0 scales, K padded to kp with zero bytes / zero scale bytes) instead of
 * bf16 rows, bit-identical to mmr_quantize_mxfp8 of the bf16 output (the fp8 Swin stages 3-4; rows %
 * 256 == 0, kp % 256 == 0, kp >= c). */
mmr_status mmr_swin_window_attention_q8(const uint16_t* qkv, const float* bias, uint8_t* q8, uint8_t* q8_scales,
                                        int32_t b, int32_t hw, int32_t c, int32_t kp, int32_t heads, int32_t ws,
                                        int32_t shift, void* stream);
/* Dense additive attention bias for one Swin block, built once at load: f32
 * [t][heads][64][64], t = 4 window types when shift > 0 (2*last-row + last-col), else 1:
 * relative_position_bias_table[(yi-yj+ws-1)*(2ws-1) + (xi-xj+ws-1)][head] (timm index), + -100
 * where the shift regions of i and j differ, -FLT_MAX for padded keys j >= ws*ws. */
mmr_status mmr_swin_attn_bias(const float* relpos_table, float* bias, int32_t heads, int32_t ws,
                              int32_t hw, int32_t shift, void* stream);

/* Fused Swin MLP sub-block for C in {96, 192} (the memory-bound stages 1-2):
 * y = x + fc2(GELU(fc1(LayerNorm(x)))) with the 4C hidden activation kept on chip.
 * x, y bf16 (tokens, C) (x != y); ln_g/ln_b, b1 (4C), b2 (C) f32; `pack` = weights repacked once by
 * mmr_swin_mlp_pack from fc1.weight [4C][C] and fc2.weight [C][4C] (bf16) into
 * mmr_swin_mlp_pack_elems(C) bf16 elements. */
int64_t mmr_swin_mlp_pack_elems(int32_t c);
mmr_status mmr_swin_mlp_pack(const uint16_t* w1, const uint16_t* w2, uint16_t* pack, int32_t c,
                             void* stream);
mmr_status mmr_swin_mlp(const uint16_t* x, const float* ln_g, const float* ln_b,
                        const uint16_t* pack, const float* b1, const float* b2, uint16_t* y,
                        int64_t tokens, int32_t c, float eps, void* stream);

/* Fused Swin attention sub-block for C = 96 (3 heads of 32, window 7; Swin-T stage 1):
 * y = x + proj(W-MSA(LayerNorm1(x))) with torch.roll shift, window partition / reverse,
 * relative-position bias and shift mask (timm SwinTransformerBlock, fusion.py:198-199).
 * x, y bf16 (b, hw, hw, 96) (x != y); `bias` = the block's dense table from mmr_swin_attn_bias;
 * `pack` = mmr_swin_attn_block_pack_bytes(96) bytes built once from attn.qkv.weight [288][96] /
 * .bias, attn.proj.weight [96][96] / .bias (bf16 weights, f32 vectors) and norm1.weight / .bias. */
int64_t mmr_swin_attn_block_pack_bytes(int32_t c);
mmr_status mmr_swin_attn_block_pack(const uint16_t* qkv_w, const float* qkv_b, const uint16_t* proj_w,
                                    const float* proj_b, const float* ln_g, const float* ln_b,
                                    void* pack, int32_t c, void* stream);
mmr_status mmr_swin_attn_block(const uint16_t* x, const void* pack, const float* bias, uint16_t* y,
                               int32_t b, int32_t hw, int32_t c, int32_t ws, int32_t shift, float eps,
                               void* stream);

/* Swin patch embedding im2col: image f32 NCHW (b,3,224,224) -> bf16 (b*56*56, 48) columns in
 * conv-weight order (cin, kh, kw) for a 4x4/s4 conv as a GEMM. */
mmr_status mmr_patch_im2col(const float* image, uint16_t* cols, int32_t b, int32_t cin,
                            int32_t hw, int32_t patch, void* stream);

/* Swin PatchMerging gather + LayerNorm(4c): x bf16 (b, hw, hw, c) -> y bf16 (b*(hw/2)^2, 4c) in
 * timm order [x(0,0), x(1,0), x(0,1), x(1,1)]. */
mmr_status mmr_patch_merge_ln(const uint16_t* x, const float* gamma, const float* beta,
                              uint16_t* y, int32_t b, int32_t hw, int32_t c, float eps,
                              void* stream);
/* mmr_patch_merge_ln also (y may be NULL: instead) writing the merged row as the reduction GEMM's
 * MX-fp8 activation operand (q8 [rows][4c] e4m3 + layout-0 scales), bit-identical to
 * mmr_quantize_mxfp8 of y (the fp8 Swin stages 3-4: 4c = 768 / 1536; rows % 256 == 0, 4c % 256 == 0). */
mmr_status mmr_patch_merge_ln_q8(const uint16_t* x, const float* gamma, const float* beta, uint16_t* y,
                                 uint8_t* q8, uint8_t* q8_scales, int32_t b, int32_t hw, int32_t c, float eps,
                                 void* stream);

/* Swin head (fusion.py:263-265 with swin_norm = swin.norm): x bf16 (b, t, c) = backbone tokens
 * BEFORE the final norm.  patches = LN(LN(x)) f32 (b,t,c), global = mean_t LN(x) f32 (b,c),
 * pool = mean over the t+1 rows [global; patches] f32 (b,c) — the image head's pooled input
 * (model.py:463-468: mean(cat[proj(g), proj(p)]) == proj(mean(cat[g, p])) for an affine proj).
 * Any output may be NULL. */
mmr_status mmr_swin_head(const uint16_t* x, const float* gamma, const float* beta, float* patches,
                         float* global, float* pool, int32_t b, int32_t t, int32_t c, float eps,
                         void* stream);

/* Unmasked mean over l tokens (model.py:370, PAD included): x bf16 (b,l,c) -> f32 (b,c). */
mmr_status mmr_mean_tokens(const uint16_t* x, float* y, int32_t b, int32_t l, int32_t c,
                           void* stream);

/* Fused projection head: y = W2 . GELU(W1 . (Wp . x + bp) + b1) + b2 (model.py:365-373 proj then
 * MultiHeadMLP model.py:61-75), f32 weights/activations, optional L2 normalise of the result.
 * w2/b2/w1/b1 may be NULL (projection only).  x (b, cin) f32, y (b, d) f32. */
mmr_status mmr_proj_head(const float* x, const float* wp, const float* bp, const float* w1,
                         const float* b1, const float* w2, const float* b2, float* y, int32_t b,
                         int32_t cin, int32_t d, int32_t l2norm, void* stream);

/* Small exact-f32 linear on strided rows: y[i*ldy + o] = act(x[i*ldx + :] . w[o][:] + bias[o])
 * (+ residual[i*ldr + o]); residual may alias y (in-place x += f(x)).  cin % 16 == 0,
 * cout % 32 == 0, ldx % 4 == 0.  The per-query vectors of the fusion stack (model.py:431-449). */
mmr_status mmr_linear_f32(const float* x, int64_t ldx, const float* w, const float* bias,
                          const float* residual, int64_t ldr, float* y, int64_t ldy, int32_t b,
                          int32_t cin, int32_t cout, int32_t act, void* stream);

/* nbatch independent mmr_linear_f32 problems in one launch; problem i reads x + i*bsx, w + i*bsw,
 * bias + i*bsb, residual + i*bsr and writes y + i*bsy (element strides; bsx, bsw % 4 == 0): the
 * per-query work of all fusion layers at once (each layer has its own weights). */
mmr_status mmr_linear_f32_batched(const float* x, int64_t ldx, int64_t bsx, const float* w, int64_t bsw,
                                  const float* bias, int64_t bsb, const float* residual, int64_t ldr,
                                  int64_t bsr, float* y, int64_t ldy, int64_t bsy, int32_t nbatch, int32_t b,
                                  int32_t cin, int32_t cout, int32_t act, void* stream);

/* ---------------------------------------------------------------- multimodal fusion stack */
/* model_type="multimodal": CrossModalFusion (src/Model/fusion.py:334-471) x num_fusion_layers +
 * the combiner (src/Model/model.py:375-459), eval.  Orchestrated host-side over these ops and
 * mmr_linear_bf16 / mmr_linear_f32. */

/* nn.MultiheadAttention core (no masks): per (batch, head) softmax(q k^T * scale) v.
 * q row (bi*lq + i) at q + row*ldq + head*dh (k, v likewise with lk); out (b*lq, ldo) bf16 and/or
 * mean_out (b, heads*dh) f32 = the mean over the lq query rows (either may be NULL, not both).
 * dh % 8 == 0, dh <= 192; strides multiples of 8 elements; any lq / lk (keys stream through LDS).
 * mean_out is bitwise deterministic for lq <= 128; longer query sets add per-128-row partials with
 * float atomics. */
mmr_status mmr_mha(const uint16_t* q, int64_t ldq, const uint16_t* k, int64_t ldk, const uint16_t* v,
                   int64_t ldv, uint16_t* out, int64_t ldo, float* mean_out, int32_t b, int32_t lq,
                   int32_t lk, int32_t heads, int32_t dh, float scale, void* stream);
/* mmr_mha emitting its output (also) as the next GEMM's MX-fp8 activation operand: e4m3 q8
 * [b*lq][heads*dh] + E8M0 scales in the layout-0 image of mmr_quantize_mxfp8 (bit-identical to
 * quantising the bf16 rows); out may be NULL.  head_dim % 32 == 0, b*lq % 256 == 0, heads*dh % 256 == 0. */
mmr_status mmr_mha_q8(const uint16_t* q, int64_t ldq, const uint16_t* k, int64_t ldk, const uint16_t* v, int64_t ldv,
                      uint16_t* out, int64_t ldo, float* mean_out, uint8_t* q8, uint8_t* q8_scales, int32_t b,
                      int32_t lq, int32_t lk, int32_t heads, int32_t dh, float scale, void* stream);

/* y = x + pos[row % l] -> bf16 (rows, c); x f32 (x_is_f32) or bf16; pos f32 [>= l][c]
 * (PreFusionEnhancer.pos_embed fusion.py:32). c % 8 == 0. */
mmr_status mmr_add_pos_bf16(const void* x, int32_t x_is_f32, const float* pos, uint16_t* y, int64_t rows,
                            int32_t l, int32_t c, void* stream);

/* mmr_add_pos_bf16 that also writes y as the next GEMM's MX-fp8 activation operand (as
 * mmr_scaled_add_layernorm_bf16_q8): the enhancer input x + pos feeding its in_proj GEMM (config 5).
 * rows % 256 == 0, c % 256 == 0. */
mmr_status mmr_add_pos_bf16_q8(const void* x, int32_t x_is_f32, const float* pos, uint16_t* y, uint8_t* q8,
                               uint8_t* q8_scales, int64_t rows, int32_t l, int32_t c, void* stream);

/* y = LayerNorm(alpha*x + residual) (+ post_scale*post), per row of c <= 1024 channels.
 * alpha / post_scale are DEVICE f32 scalars (learned parameters) or NULL (= 1); residual / post
 * may be NULL.  io_bf16: x, residual, y bf16 (else f32); post is always f32.  Row r uses parameter
 * set g = (r / group_div) % groups — gamma/beta + g*c, alpha/post_scale + g — so one launch
 * normalises the rows of several layers (groups = layers; group_div = 1 for [..][layer][c] rows,
 * = rows per layer for [layer][..][c]). */
mmr_status mmr_ln_rows(const void* x, int64_t ldx, const float* alpha, const void* residual, int64_t ldr,
                       const float* gamma, const float* beta, const float* post, int64_t ldp,
                       const float* post_scale, void* y, int64_t ldy, int64_t rows, int32_t c, float eps,
                       int32_t io_bf16, int32_t groups, int64_t group_div, void* stream);

/* f32 y = LayerNorm(alpha * x + residual) (alpha: a DEVICE f32 scalar or NULL = 1; residual may be NULL,
 * y may be NULL) that also writes xs, the x3 split GEMM's X operand: [hi | lo] bf16 rows 2 kp wide
 * (kp = mmr_x3_p8_kpad(c), zero columns c..kp), the split mmr_x3_split_rows would make of y.
 * c % 4 == 0, c <= 1024; rows 16-B aligned. */
mmr_status mmr_ln_rows_split(const float* x, int64_t ldx, const float* alpha, const float* residual, int64_t ldr,
                             const float* gamma, const float* beta, float* y, int64_t ldy, uint16_t* xs, int64_t rows,
                             int32_t c, float eps, void* stream);

/* seq (b, np+2, c) bf16 = [x1; patches_fused; x2] + pe[0..np+2) (fusion.py:468 + model.py:397);
 * x1, x2 f32 (b, c), patches_fused bf16 (b*np, c), pe f32 [>= np+2][c]. */
mmr_status mmr_assemble_seq(const float* x1, const uint16_t* patches_fused, const float* x2, const float* pe,
                            uint16_t* seq, int32_t b, int32_t np, int32_t c, void* stream);

/* mmr_assemble_seq written only as the combiner QKV GEMM's MX-fp8 activation operand (layout 0, as
 * mmr_quantize_mxfp8 of the bf16 sequence, bit-identical); b*(np+2) and c multiples of 256.
 * Replaces: the same cat + pos_encoder (reference src/Model/model.py:396-397) on the fp8 path. */
mmr_status mmr_assemble_seq_q8(const float* x1, const uint16_t* patches_fused, const float* x2, const float* pe,
                               uint8_t* q8, uint8_t* q8_scales, int32_t b, int32_t np, int32_t c, void* stream);

/* y (b, c) f32 = x[i*ldx + 0..c) (bf16 rows, e.g. the CLS token of each sequence). */
mmr_status mmr_rows_to_f32(const uint16_t* x, int64_t ldx, float* y, int32_t b, int32_t c, void* stream);

/* ---------------------------------------------------------------- fp32-faithful tower mode ("x3") */
/* The towers and the multimodal head with f32 activations and every contraction on bf16 MFMA with
 * three-term splits (a = a_hi + a_lo, a.b ~= a_hi.b_hi + a_hi.b_lo + a_lo.b_hi in f32, ~2^-17
 * relative per product); LayerNorm / softmax (expf) / GELU (erff) / means in f32.  The reference runs
 * the same towers in fp32 (src/Model/fusion.py:198-199, 322-325; model.py:365-479): this mode holds the
 * end-to-end lists to BASELINE.md §3's bar.  All activations f32. */

/* y = act(x @ W^T + bias) (+ residual) for any m: x (m, k) rows at stride ldx, W given as its bf16
 * split w_hi = bf16(W), w_lo = bf16(W - w_hi) ([n][k] each, contiguous); act 0 none, 1 GELU(erf).
 * k % 32 == 0; residual may alias y. */
mmr_status mmr_x3_linear(const float* x, int64_t ldx, const uint16_t* w_hi, const uint16_t* w_lo, const float* bias,
                         const float* residual, int64_t ldr, float* y, int64_t ldy, int64_t m, int32_t n, int32_t k,
                         int32_t act, void* stream);
/* The same linear at the 8-phase GEMM's rate: the split operands X = [x_hi | x_lo] and W = [w_hi | w_lo]
 * (bf16 rows, each segment kp = mmr_x3_p8_kpad(k) wide: k rounded up to 128, zero padding; 0 = k not
 * taken) in ONE GEMM whose K-tiles hold 32 k of both segments and issue x_hi.w_hi + x_hi.w_lo + x_lo.w_hi
 * into f32 accumulators (each operand staged once).
 * mmr_x3_split_rows writes X ([m][2 kp] bf16, caller-allocated) from f32 x rows at stride ldx;
 * mmr_ln_rows_split, the attention _xs forms below and a split output (out_hilo) write the same rows.
 * mmr_x3_linear_p8 takes X and the weight image W ([npad][2 kp] bf16, built once at load, npad =
 * mmr_x3_p8_npad(n): n itself when it is a multiple of 192 or 256, else n rounded up to 192 with zero
 * rows; 0 = n not taken) and writes y (m, n) f32 contiguous: m % 256 == 0, act 0 / 1 (GELU, erf), bias
 * NULL or npad floats (zero-padded), residual (m, n) f32 contiguous or NULL (may be y).
 * out_hilo != 0: y is written as the NEXT x3 GEMM's X operand, [y_hi | y_lo] bf16 rows 2 n wide
 * (the split of the f32 value mmr_x3_split_rows would make, bit for bit); needs n % 384 == 0 and no
 * residual — a FFN1 -> FFN2 pair then skips the f32 round trip and the split pass. */
int32_t mmr_x3_p8_kpad(int32_t k);
int32_t mmr_x3_p8_npad(int32_t n);
mmr_status mmr_x3_split_rows(const float* x, int64_t ldx, int64_t m, int32_t k, uint16_t* xs, void* stream);
mmr_status mmr_x3_linear_p8(const uint16_t* xs, const uint16_t* w2, const float* bias, const float* residual, void* y,
                            int64_t m, int32_t n, int32_t k, int32_t act, int32_t out_hilo, void* stream);
/* Attention core (nn.MultiheadAttention / BERT self-attention, eval): per (batch, head)
 * softmax(q k^T * scale (+ key mask)) v; rows as mmr_mha (q row bi*lq + i at q + row*ldq + head*dh);
 * mask01 (b, lk) int64 or NULL (0 -> key excluded, HF's additive finfo.min); out (b*lq, ldo) and/or
 * mean_out (b, heads*dh) = mean over the lq query rows (deterministic).  dh % 8 == 0, dh <= 128. */
mmr_status mmr_x3_attention(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v, int64_t ldv,
                            float* out, int64_t ldo, float* mean_out, const int64_t* mask01, int32_t b, int32_t lq,
                            int32_t lk, int32_t heads, int32_t dh, float scale, void* stream);
/* Swin (shifted-)window attention as mmr_swin_window_attention on f32 qkv (b*hw*hw, 3c) -> out
 * (b*hw*hw, c), q scaled by dh^-0.5 before q k^T (timm), bias from mmr_swin_attn_bias.  head_dim <= 32. */
mmr_status mmr_x3_swin_window_attention(const float* qkv, const float* bias, float* out, int32_t b, int32_t hw,
                                        int32_t c, int32_t heads, int32_t ws, int32_t shift, void* stream);
/* The two above writing their output as the x3 split GEMM's X operand instead (the O-proj / proj
 * input): xs = [hi | lo] bf16 rows 2 kp wide, kp = mmr_x3_p8_kpad(heads*dh) (columns heads*dh..kp zero),
 * the split mmr_x3_split_rows would make of the f32 output. */
mmr_status mmr_x3_attention_xs(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v, int64_t ldv,
                               uint16_t* xs, float* mean_out, const int64_t* mask01, int32_t b, int32_t lq, int32_t lk,
                               int32_t heads, int32_t dh, float scale, void* stream);  /* mean_out may be NULL */
mmr_status mmr_x3_swin_window_attention_xs(const float* qkv, const float* bias, uint16_t* xs, int32_t b, int32_t hw,
                                           int32_t c, int32_t heads, int32_t ws, int32_t shift, void* stream);
/* Patch-embed im2col, f32: (b, cin, hw, hw) -> (b*(hw/patch)^2, kp) columns (k = c*p^2 + ky*p + kx, zero
 * for k >= cin*p^2). */
mmr_status mmr_x3_patch_im2col(const float* image, float* cols, int32_t b, int32_t cin, int32_t hw, int32_t patch,
                               int32_t kp, void* stream);
/* PatchMerging gather (timm order) + LayerNorm(4c), f32 in / out; 4c <= 4096. */
mmr_status mmr_x3_patch_merge_ln(const float* x, const float* gamma, const float* beta, float* y, int32_t b,
                                 int32_t hw, int32_t c, float eps, void* stream);
/* The same writing the reduction linear's x3 split operand instead: xs = [hi | lo] bf16 rows 2 kp wide,
 * kp = mmr_x3_p8_kpad(4c) (zero columns 4c..kp); c % 4 == 0, 16-B aligned pointers. */
mmr_status mmr_x3_patch_merge_ln_xs(const float* x, const float* gamma, const float* beta, uint16_t* xs, int32_t b,
                                    int32_t hw, int32_t c, float eps, void* stream);
/* BERT embeddings LN((word[id] + type[0]) + pos[l]) -> f32 (b*l, c), c <= 1024. */
mmr_status mmr_x3_bert_embed(const int64_t* ids, const float* word, const float* pos, const float* type0,
                             const float* gamma, const float* beta, float* y, int32_t b, int32_t l, int32_t c, float eps,
                             void* stream);
/* y = x + pos[row % l], f32 (rows, c). */
mmr_status mmr_x3_add_pos(const float* x, const float* pos, float* y, int64_t rows, int32_t l, int32_t c, void* stream);
/* The same written as the x3 split GEMM's operand: xs = [hi | lo] bf16 rows 2 kp wide (kp =
 * mmr_x3_p8_kpad(c), zero columns c..kp), plus the f32 rows y when y != NULL; c % 4 == 0, 16-B aligned. */
mmr_status mmr_x3_add_pos_split(const float* x, const float* pos, float* y, uint16_t* xs, int64_t rows, int32_t l,
                                int32_t c, void* stream);
/* seq (b, np+2, c) f32 = [x1; patches_fused; x2] + pe. */
mmr_status mmr_x3_assemble_seq(const float* x1, const float* patches_fused, const float* x2, const float* pe,
                               float* seq, int32_t b, int32_t np, int32_t c, void* stream);
/* The same written only as the combiner QKV GEMM's x3 split operand rows (as mmr_x3_add_pos_split). */
mmr_status mmr_x3_assemble_seq_split(const float* x1, const float* patches_fused, const float* x2, const float* pe,
                                     uint16_t* xs, int32_t b, int32_t np, int32_t c, void* stream);
/* fp32-faithful fused Swin MLP (csrc/x3_mlp.hip): y = x + fc2(GELU_erf(fc1(LN(x)))) over tokens x (tokens, c)
 * f32 (c in {96, 192}; y != x, 16-B aligned), both linears on bf16x3 MFMA, the hidden never leaving the CU.
 * pack: mmr_x3_swin_mlp_pack_elems(c) bf16 elements, built once from the f32 fc1.weight [4c][c] and
 * fc2.weight [c][4c] by mmr_x3_swin_mlp_pack (0 elements / MMR_ERR_UNSUPPORTED for other c). */
int64_t mmr_x3_swin_mlp_pack_elems(int32_t c);
/* fp32-faithful row-linear for the narrow Swin stages (csrc/x3_mlp.hip): y (tokens, n) f32 = LN(x) W^T + b
 * (+ residual) with x f32 (tokens, c) and its LayerNorm (ln_g, ln_b), or = xs W^T + b (+ residual) with xs
 * the x3 split-operand rows [hi | lo] (tokens, 2 kp), kp = mmr_x3_p8_kpad(c) (the window attention's _xs
 * output) — exactly one of x / xs.  bf16x3 MFMA, W^T streamed through LDS.  c in {96, 192}, n % 32 == 0,
 * n <= 4096 (c = 96: n > 64); pack = mmr_x3_rowlin_pack_elems(n, c) bf16 elements built once from the f32
 * weight [n][c] by mmr_x3_rowlin_pack. */
int64_t mmr_x3_rowlin_pack_elems(int32_t n, int32_t c);
mmr_status mmr_x3_rowlin_pack(const float* w, uint16_t* pack, int32_t n, int32_t c, void* stream);
mmr_status mmr_x3_rowlin(const float* x, const uint16_t* xs, const float* ln_g, const float* ln_b, const uint16_t* pack,
                         const float* bias, const float* residual, float* y, int64_t tokens, int32_t n, int32_t c,
                         float eps, void* stream);
mmr_status mmr_x3_swin_mlp_pack(const float* w1, const float* w2, uint16_t* pack, int32_t c, void* stream);
/* fp32-faithful fused Swin attention sub-block for C = 96 (3 heads of 32, window 7; Swin-T stage 1,
 * csrc/x3_sab.hip): y = x + proj(W-MSA(LayerNorm1(x))) with torch.roll shift, window partition / reverse,
 * relative-position bias and shift mask (timm SwinTransformerBlock, fusion.py:198-199) in f32, every
 * contraction on bf16x3 MFMA — the x3_rowlin (norm1 + qkv) -> x3 window attention -> x3_rowlin (proj +
 * residual) chain in one pass.  x, y f32 (b, hw, hw, 96) (x != y, 16-B aligned); `bias` = the block's dense
 * table from mmr_swin_attn_bias; `pack` = mmr_x3_swin_attn_block_pack_bytes(96) bytes built once from the
 * f32 attn.qkv.weight [288][96] / .bias, attn.proj.weight [96][96] / .bias and norm1.weight / .bias
 * (0 bytes / MMR_ERR_UNSUPPORTED for other c). */
int64_t mmr_x3_swin_attn_block_pack_bytes(int32_t c);
mmr_status mmr_x3_swin_attn_block_pack(const float* qkv_w, const float* qkv_b, const float* proj_w, const float* proj_b,
                                       const float* ln_g, const float* ln_b, void* pack, int32_t c, void* stream);
mmr_status mmr_x3_swin_attn_block(const float* x, const void* pack, const float* bias, float* y, int32_t b, int32_t hw,
                                  int32_t c, int32_t ws, int32_t shift, float eps, void* stream);
mmr_status mmr_x3_swin_mlp(const float* x, const float* ln_g, const float* ln_b, const uint16_t* pack, const float* b1,
                           const float* b2, float* y, int64_t tokens, int32_t c, float eps, void* stream);
/* fp32-faithful Swin stem (csrc/x3_mlp.hip): y (b, hw/4, hw/4, 96) f32 = LayerNorm(Conv2d(3, 96, 4, stride 4)
 * (img) + bias) (timm PatchEmbed with its norm) for img (b, 3, hw, hw) f32 NCHW, the conv on bf16x3 MFMA, one
 * pass (no im2col rows).  hw % 4 == 0, (hw/4)^2 % 32 == 0, 16-B aligned pointers.  pack:
 * mmr_x3_patch_embed_pack_elems() bf16 elements built once from the f32 conv weight [96][3*4*4] by
 * mmr_x3_patch_embed_pack. */
int64_t mmr_x3_patch_embed_pack_elems(void);
mmr_status mmr_x3_patch_embed_pack(const float* w, uint16_t* pack, void* stream);
mmr_status mmr_x3_patch_embed_ln(const float* img, int32_t b, int32_t hw, const uint16_t* pack, const float* bias,
                                 const float* ln_g, const float* ln_b, float eps, float* y, void* stream);
/* The bf16 towers' stem on the same pack: y (b, hw/4, hw/4, 96) bf16 = LayerNorm(conv(img) + bias) with the
 * pixels rounded to bf16 and one bf16 product with the pack's hi image (= the bf16 conv weight), the
 * bias and LayerNorm on the f32 accumulators; replaces mmr_patch_im2col + the GEMM + mmr_layernorm_bf16
 * (timm PatchEmbed, fusion.py:198-199). */
mmr_status mmr_patch_embed_ln_bf16(const float* img, int32_t b, int32_t hw, const uint16_t* pack, const float* bias,
                                   const float* ln_g, const float* ln_b, float eps, uint16_t* y, void* stream);
/* y (b, c) = (extra[b] + sum_t x[b][t]) / (l + 1) with extra (b, c), or sum_t x[b][t] / l when extra is
 * NULL; x (b, l, c) f32, summed in token order (unmasked token mean, model.py:370; the Swin global /
 * pooled means, fusion.py:263-265, model.py:463-468). */
mmr_status mmr_x3_mean_rows(const float* x, const float* extra, float* y, int32_t b, int32_t l, int32_t c,
                            void* stream);
/* y (b, c) = x[i*ldx + 0..c), f32 (the CLS rows, fusion.py:447). */
mmr_status mmr_x3_gather_rows(const float* x, int64_t ldx, float* y, int32_t b, int32_t c, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MMR_H */

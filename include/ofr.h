/*
 * ofr.h — C ABI of libocvf_hip.so, the MI355X (gfx950) implementation of the
 * ocvfacerec / bytefish-facerec recognition hot path.
 *
 * The reference (sandykindy/opencv_facerecognizer, Python 2.7 + numpy) has no
 * FFI: its hot path is the Python class API of src/ocvfacerec/facerec/.
 * Each entry point below replaces the numpy expression cited next to it; the
 * Python host package (opencv_facerecognizer_amd/, importable as
 * `ocvfacerec`) keeps the reference's classes and calls these functions
 * through ctypes.  Reference paths are relative to
 * /root/reference/src/ocvfacerec/.
 *
 * Conventions
 *   - Every function returns int: 0 = OFR_OK, negative = ofr error code
 *     (enum below), positive = hipError_t passed through.  The library never
 *     aborts or exits.  ofr_last_error() returns a thread-local message.
 *   - All array arguments are caller-owned DEVICE pointers (e.g. torch
 *     tensor data_ptr()); the library keeps no pointer past a call.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *     calls are stream-ordered and asynchronous.
 *   - Matrices are row-major with an explicit leading dimension `ld*` in
 *     ELEMENTS.  Float operands of the MFMA GEMMs use ld % 32 == 0 and the
 *     columns [K, round_up(K,32)) of every row must be zero (the padding is
 *     part of the device layout the host package owns).
 *   - Element types are named by enum ofr_dtype where a function takes several.
 */
#ifndef OFR_H
#define OFR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ofr_status {
  OFR_OK = 0,
  OFR_E_INVALID = -1,     /* bad argument (shape, stride, alignment, null) */
  OFR_E_UNSUPPORTED = -2, /* valid but not implemented (e.g. k > OFR_MAX_K) */
  OFR_E_DEVICE = -3,      /* no usable gfx950 device */
  OFR_E_NUMERIC = -4,     /* numerical failure: matrix not positive definite, no convergence */
};

enum ofr_metric {
  OFR_METRIC_EUCLIDEAN = 0, /* distance.py:53-60  sqrt(sum((p-q)^2))            */
  OFR_METRIC_COSINE = 1,    /* distance.py:63-77  -p.q / sqrt((p.p)(q.q))        */
  OFR_METRIC_CHISQUARE = 2, /* distance.py:101-116 sum((p-q)^2/(p+q+eps))        */
};

enum ofr_dtype { OFR_DT_U8 = 0, OFR_DT_U16 = 1, OFR_DT_U32 = 2, OFR_DT_F32 = 3, OFR_DT_F64 = 4 };

#define OFR_MAX_K 16          /* largest k of the fused search (classifier.py:53-129) */
#define OFR_TILE_ROWS 256     /* gallery rows per search tile                          */

/* Library / context ------------------------------------------------------ */
int ofr_version(void);                 /* (major<<16)|(minor<<8)|patch */
const char* ofr_last_error(void);      /* thread-local, never NULL      */
int ofr_device_check(int device);      /* OFR_OK iff `device` is gfx950 */

/* Projection ---------------------------------------------------------------
 * Y[b][j] = sum_i X[b][i] * W[i][j] - shift[j]      (b < B, j < d, i < D)
 * Replaces Fisherfaces.project  feature.py:241-242 (np.dot(W.T, x), shift=NULL),
 *          PCA.project          feature.py:114-116 (shift = P^T mu),
 *          LDA.project          feature.py:184-185, and the per-sample
 *          projection loops feature.py:104-108, 178-182, 231-235.
 * EXACT integer path on v_mfma_i32_16x16x64_i8: W is prepared once into four
 * int8 slices with a power-of-two scale per output feature
 * (W[i][j] = s_j (q1 + q2/2^7 + q3/2^14 + q4/2^21), exact for every fp32
 * element within 2^4 of its column maximum); (x-128) . q is accumulated in
 * int32 without rounding and combined in fp64 without rounding; the shift is
 * subtracted in fp64 and the result rounded once to fp32 or fp64.
 * Wt: W transposed, [d][ldw] of OFR_DT_F32 or OFR_DT_F64.
 * Aq: int8 [ceil(d/64)*256][ldk], ldk % 128 == 0, ldk >= round_up(D,128)
 *     (ofr_qproj_bytes(D,d) bytes with ldk = round_up(D,128)); scale, K: fp64 [d].
 * X : uint8 [B][ldx], 16-byte aligned rows, ldx >= D.
 * Y : [B][ldy] of y_dtype (OFR_DT_F32 / OFR_DT_F64); columns j < d written.   */
size_t ofr_qproj_bytes(int64_t D, int64_t d);
int ofr_qproj_prepare(void* stream, int dtype, const void* Wt, int64_t d, int64_t D, int64_t ldw,
                      int8_t* Aq, int64_t ldk, double* scale, double* K);
int ofr_project_u8_exact(void* stream, const uint8_t* X, int64_t B, int64_t D, int64_t ldx,
                         const int8_t* Aq, int64_t ldk, const double* scale, const double* K,
                         int64_t d, const double* shift, void* Y, int64_t ldy, int y_dtype);
/* The same product as a launch over tiles [t0, t1) of its grid (one tile per CU and round):
 * ofr_project_u8_exact_tiles(B, d) = the tile count (0 when B <= 4 takes the split-K GEMV, which has
 * no tiles); every tile writes its own outputs, so launches over a partition of [0, tiles) give
 * ofr_project_u8_exact's output bit for bit (lets a caller run other work beside the last round). */
int64_t ofr_project_u8_exact_tiles(int64_t B, int64_t d);
int ofr_project_u8_exact_range(void* stream, const uint8_t* X, int64_t B, int64_t D, int64_t ldx,
                               const int8_t* Aq, int64_t ldk, const double* scale, const double* K,
                               int64_t d, const double* shift, void* Y, int64_t ldy, int y_dtype,
                               int64_t t0, int64_t t1);

/* Gallery preparation ------------------------------------------------------
 * For the search kernels: aux[n] = ||G[n]||^2 (EUCLIDEAN) or 1/||G[n]|| (COSINE),
 * computed in fp64 and stored fp32.  G [N][ldg] fp32.                       */
int ofr_row_aux(void* stream, int metric, const float* G, int64_t N, int64_t d, int64_t ldg,
                float* aux);
/* Certified Cosine search (CosineDistance, distance.py:74-77): the Cosine
 * ranking is the Euclidean ranking of unit vectors, so the certified Euclidean
 * tiers run on out = fp32(g / ||g|| - shift) (fp64, rounded once; shift
 * nullable, e.g. the mean unit row, which keeps the quantization relative to
 * the rows' spread rather than their common direction; zero rows stay zero,
 * pad columns [d, ldo) zeroed) and ofr_cosine_pairs then evaluates the reference
 * formula -p.q / sqrt(p.p q.q) in fp64 for the found (query, row) pairs
 * (out_i [B][k] in: local rows, -1 = none; out: sorted by (distance, row)).  */
int ofr_normalize_rows_f32(void* stream, const float* G, int64_t N, int64_t d, int64_t ldg, const double* shift,
                           float* out, int64_t ldo);
int ofr_cosine_pairs(void* stream, const float* Q, int64_t B, int64_t ldq, const float* G, int64_t N,
                     int64_t ldg, int64_t d, int k, double* out_d, int64_t* out_i);
/* out[n][j] = (float)(F[n][j] - shift[j]) for j < d: fp64 features -> the
 * fp32 search layout, centred BEFORE the rounding (shift may be NULL).       */
int ofr_center_round_f64(void* stream, const double* F, int64_t N, int64_t d, int64_t ldf,
                         const double* shift, float* out, int64_t ldo);
/* mean[j] = (1/N) sum_n G[n][j] in fp64 (column means of the gallery).      */
int ofr_col_mean(void* stream, const float* G, int64_t N, int64_t d, int64_t ldg, double* mean);
/* G[n][j] -= shift[j] for j < d (fp32).                                     */
int ofr_sub_rows(void* stream, float* G, int64_t N, int64_t d, int64_t ldg, const float* shift);

/* k-nearest-neighbour search ----------------------------------------------
 * Replaces NearestNeighbor.predict classifier.py:76-129 (the per-item
 * distance loop :104-108, argsort :113 and top-k slice :118-119) for a
 * BATCH of B queries against N gallery rows.
 *   pass 1  (MFMA tile kernel): coarse scores s = aux[n] - 2 q.g (EUCLIDEAN,
 *           on centred features) or -(q.g) aux[n] (COSINE); per 256-row
 *           gallery tile, the best OFR_KC candidates per query.
 *   pass 2  merge of the tile candidates, EXACT fp64 re-evaluation of the
 *           reference distance on the R best candidates, sort by
 *           (distance, index) — ties resolve to the lowest gallery index.
 * Outputs: out_d [B][k] fp64 distances, out_i [B][k] int64 gallery indices
 * (+ index_base); entries beyond N are (+inf, -1).
 * workspace: device scratch of ofr_knn_workspace_bytes(B, N, k) bytes.      */
size_t ofr_knn_workspace_bytes(int64_t B, int64_t N, int k);
int ofr_knn_f32(void* stream, int metric, const float* Q, int64_t B, int64_t ldq, const float* G,
                int64_t N, int64_t ldg, int64_t d, const float* aux, int k, int64_t index_base,
                double* out_d, int64_t* out_i, void* workspace, size_t workspace_bytes);
/* The two passes of ofr_knn_f32 as separate launches (same arguments; pass 1
 * ignores index_base/out_*, pass 2 reads the candidates pass 1 left in the
 * workspace).  Lets a caller time the MFMA pass alone on its stream.         */
int ofr_knn_tiles_f32(void* stream, int metric, const float* Q, int64_t B, int64_t ldq, const float* G,
                      int64_t N, int64_t ldg, int64_t d, const float* aux, int k, int64_t index_base,
                      double* out_d, int64_t* out_i, void* workspace, size_t workspace_bytes);
int ofr_knn_merge_f32(void* stream, int metric, const float* Q, int64_t B, int64_t ldq, const float* G,
                      int64_t N, int64_t ldg, int64_t d, const float* aux, int k, int64_t index_base,
                      double* out_d, int64_t* out_i, void* workspace, size_t workspace_bytes);

/* Certified int8 coarse pass (Euclidean, B > 32) -----------------------------
 * Rows (gallery once, query batch per call) are cut into int8 slices with a
 * power-of-two scale s (max|x|/s in (63.5, 127]):
 *   slices = 1:  x~ = s x1                 Xs [R][ld], ld % 128 == 0, ld >= round_up(d, 128)
 *   slices = 2:  x~ = s (x1 + x2/2^7)      Xs [R][ld], ld % 128 == 0, ld >= 2 round_up(d, 64);
 *                per 64 features, 64 bytes of x1 then 64 bytes of x2 (one 128-B line)
 * Per row stats[3] = (||x~||, ||x - x~||, s 2^-7 ||x2||) in fp64 (third = 0 for
 * one slice).  With maxima != NULL the gallery-wide maxima (A, E, T, max aux)
 * are reduced into maxima[4].                                                  */
int ofr_q8_quantize_rows(void* stream, int slices, const float* X, int64_t R, int64_t d, int64_t ldx,
                         int8_t* Xs, int64_t ld, float* scale, double* stats, const float* aux,
                         double* maxima);
/* The search: v_mfma_i32_32x32x32_i8 sums x1.y1 (and x1.y2 + x2.y1) exactly,
 * the coarse score ||g||^2 - 2 s_q s_g (P0 + P1/2^7) keeps the best 16 rows
 * per 256-row tile and query; the merge re-ranks the best 16 with the exact
 * fp64 distance (distance.py:60) and writes cert[q] = 1 iff the rigorous bound
 * |S - S~| <= dS(q) proves that no other row can reach the k-th neighbour
 * (DESIGN.md §3).  Queries with cert[q] == 0 must be re-run with more slices
 * or on ofr_knn_f32.  bound (nullable, [B]): a lower bound of the squared
 * distance of every row outside the candidates (+inf if all rows were
 * candidates); cert[q] = (d_k^2 < bound[q]).  A gallery sharded over ranks
 * certifies the GLOBAL top-k when its k-th squared distance is below every
 * rank's bound (opencv_facerecognizer_amd/parallel.py).  Q/G: the fp32 rows the slices were made from (centred),
 * for the re-rank.  phases: 1 = tiles, 2 = merge, 3 = both.  k <= 16.        */
size_t ofr_knn_q8_workspace_bytes(int64_t B, int64_t N);
int ofr_knn_q8(void* stream, int phases, int slices, const float* Q, int64_t B, int64_t ldq, const int8_t* Qs,
               const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg, int64_t d,
               const int8_t* Gs, int64_t ld, const float* gscale, const float* aux, const double* gmax,
               int k, int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound,
               void* workspace, size_t workspace_bytes);

/* fp6 first tier of the certified search (same contract as ofr_knn_q8) -----
 * Rows are cut into e2m3 fp6 values with a per-row fp32 scale s = max|x|/7.5
 * (x~ = s v, |v| <= 7.5) and stored in the "f6 tiled" layout: 256-row panels x
 * 128-feature stages, 24 KiB per (panel, stage) (layout: csrc/ofr_f6_tile.h);
 * ofr_f6_tiles_bytes(R, d) bytes, rows past R in the last panel zeroed.
 * stats[3] = (||x~||, ||x - x~||, 0); maxima as ofr_q8_quantize_rows.
 * Column-block scales (round 5; every f6 / f6x2 entry point's trailing bscale,
 * null = unit): one E8M0 byte per 32 features (4 * ceil(d / 128) bytes, 4-byte
 * aligned), shared by a gallery and every query batch searched against it:
 * feature k is quantized as x_k / 2^e with e = bscale[k / 32] - 127, the row
 * scale s = max_k |x_k| / 2^e_k / 7.5, x~_k = s 2^e_k v_k, and the MFMA applies
 * 2^e_k to both operands.  ofr_f6_block_sumsq accumulates per-block sums of
 * squares over rows (sums [ceil(d / 32)] fp64, +=, zero them first; shards
 * all-reduce them); ofr_f6_block_scales turns them into bytes with
 * e_b = rint(log2(rms_b / max rms)) in [-63, 0] (127 past d).  A trained
 * Fisherfaces W puts most of the feature variance into its leading columns; one
 * row scale alone then leaves the rest a few fp6 steps (residual 0.11 of the
 * row norm against 0.03).
 * ofr_knn_f6: v_mfma_scale_f32_32x32x64_f8f6f4 (fp6 x fp6, column-block scales)
 * sums v_q.v_g with fp32 accumulation, whose error (<= (2 nst + 64) 2^-23
 * a_q A) is added to the certificate bound; otherwise the ofr_knn_q8 contract
 * (exact fp64 re-rank of the best 16 coarse rows, cert[q], bound[q]).
 * B <= 32: one streaming pass, best 16 per 256-row tile.  B > 32: a sieve --
 * a sample pass over every 64th tile sets a per-query keep threshold, the
 * full pass keeps only rows at or below it (the certificate uses min(threshold,
 * 16th kept)); a query whose bucket (32768 rows) overflows comes back with
 * cert 0 and bound -inf.  Phase 1 state lives in the workspace:
 * ofr_knn_f6_workspace_bytes(B, N) bytes, 16-byte aligned, kept between the
 * phase-1 and phase-2 calls; after phase 1 the int32 kept-row counts [B] sit
 * at byte ofr_knn_f6_sieve_counts_offset(B, N) of it (SIZE_MAX: no sieve,
 * B <= 32).  The panel sample takes every 64th 256-row panel.
 * Phase 1 in two calls (a pipelined caller overlaps other work with the second
 * only): phases 4 = the sample pass + thresholds (B <= 32: the whole stream
 * pass), 8 = the sieve pass (after a phases-4 call on the same workspace;
 * a second sieve pass on the same thresholds would append every kept row
 * twice, so it marks every query's bucket overflowed instead: cert 0, bound
 * -inf); 1 = 4 + 8.  Phase bits combine (e.g. 10 = sieve, then merge).       */
size_t ofr_f6_tiles_bytes(int64_t R, int64_t d);
/* Append support (NearestNeighbor.update, classifier.py:65-70): quantize X's R rows
 * into rows row0 .. row0+R-1 of an existing tiled buffer (scale/stats indexed by
 * the destination row), zeroing the rest of the last panel; then recompute the
 * gallery maxima over all rows with ofr_q8_maxima.                           */
int ofr_f6_quantize_rows_at(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, int64_t row0,
                            void* tiles, size_t tiles_bytes, float* scale, double* stats, const uint8_t* bscale);
int ofr_q8_maxima(void* stream, const double* stats, const float* aux, int64_t R, double* maxima);
int ofr_f6_block_sumsq(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, double* sums);
int ofr_f6_block_scales(void* stream, const double* sums, int64_t d, uint8_t* bscale);
size_t ofr_knn_f6_workspace_bytes(int64_t B, int64_t N);
/* byte offset in that workspace of int32 [B]: after a merge (phase 2), the number of candidates each
 * query re-ranked exactly (its fp32 rows read: that many x d x 4 bytes) -- round 6, for the merge's
 * HBM roofline                                                                                  */
size_t ofr_knn_f6_merge_evals_offset(int64_t B, int64_t N);
size_t ofr_knn_f6_sieve_counts_offset(int64_t B, int64_t N);
/* Round 6: the sieve's keep thresholds given instead of a sample pass -- per query the coarse-score bound
 * smax[B] (fp64; NaN or +inf: keep every row), B > 32 -- for a following phases-8 (sieve) call on the same
 * workspace: a query a tier left open is searched again keeping every row whose coarse score could still
 * beat its k-th exact distance, smax = d_k^2 - |q|^2 + dS (FloatGallery._resieve), and the merge's deep
 * continuation re-ranks those rows.  Replaces the same search as ofr_knn_f6 (classifier.py:104-119). */
int ofr_knn_f6_set_thresholds(void* stream, const double* smax, int64_t B, int64_t N, void* workspace,
                              size_t workspace_bytes);
int ofr_f6_quantize_rows(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, void* tiles,
                         size_t tiles_bytes, float* scale, double* stats, const float* aux, double* maxima,
                         const uint8_t* bscale);
/* The fp6 sieve kernel ofr_knn_f6 launches for B > 32, as the profiler names it (profiling labels). */
const char* ofr_f6_sieve_kernel(void);
/* the kernel ofr_knn_f6p_sampled's sieve pass launches at pstages (B > 32): the persistent prefix pass
 * for pstages <= 2 (OFR_F6P_PERSIST=0: the per-tile pass above)                                    */
const char* ofr_f6p_sieve_kernel(int pstages);
int ofr_knn_f6(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
               const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg, int64_t d,
               const void* Gt, const float* gscale, const float* aux, const double* gmax, int k,
               int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound,
               void* workspace, size_t workspace_bytes, const uint8_t* bscale);
/* ofr_knn_f6 with a ROW sample for the sieve thresholds (B > 32; new, same contract otherwise).
 * St/sscale/saux: fp6 tiles (ofr_f6_tiles_bytes(Ns, d) bytes), row scales and aux terms of Ns <=
 * ceil(N / 64) gallery rows, written by ofr_f6_sample_rows (rows 0, 64, 128, ...).  The threshold
 * becomes the max(k, 4)-th best key of the sample instead of the 16th best of every 64th 256-row
 * panel: ~4 x 64 rows kept per query instead of ~16 x 64, and a gallery stored identity by identity
 * cannot put whole clusters of one face into the sample.  The sample only steers how many rows are
 * kept: results and certificates are those of ofr_knn_f6 (any sample, any threshold).           */
int ofr_knn_f6_sampled(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                       const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg, int64_t d,
                       const void* Gt, const float* gscale, const float* aux, const double* gmax, int k,
                       int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound, const void* St,
                       int64_t Ns, const float* sscale, const float* saux, void* workspace, size_t workspace_bytes,
                       const uint8_t* bscale);
/* Prefix tier f6p: ofr_knn_f6_sampled whose sample and sieve passes score only the
 * first pstages 128-feature stages of the same tiles (1 <= pstages <= ceil(d / 128)).  aux / saux are
 * the PREFIX terms |g_m|^2 of the rows and of the row sample (ofr_row_aux over the first
 * min(d, 128 pstages) features, saux[j] = aux[64 j]); Gt/gscale/gmax: see below.  A row's squared distance
 * is at least that of its first features, so the certificate and the bound (-> the merge's exact fp64
 * re-rank of the full rows) hold as for ofr_knn_f6; on features whose discriminating variance sits in
 * the leading columns (Fisherfaces / Eigenfaces output, eigenvalues descending) it certifies at a
 * fraction of the coarse work.  Replaces the same search as ofr_knn_f6 (classifier.py:94-129).     */
/* its query rows: only the first pstages stages of each row's f6 tiles written, from the first
 * min(d, 128 pstages) features, with their own row scale and (prefix) stats                       */
int ofr_f6_quantize_rows_prefix(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, int pstages,
                                void* tiles, size_t tiles_bytes, float* scale, double* stats,
                                const uint8_t* bscale);
/* The prefix tier's OWN gallery tiles (round 6): the first pstages stages of each row in the f6 tiled layout of
 * pstages stages per 256-row panel (ofr_f6p_tiles_bytes(R, pstages) bytes), quantized from the first
 * min(d, 128 pstages) features with power-of-two row scales (exact in the MFMA's E8M0 operand scale: the pass
 * folds 2 s_g and -|g_m|^2 into the MFMA) and their prefix stats; ofr_f6p_quantize_rows also writes the maxima
 * of those stats and of paux (the prefix terms |g_m|^2, ofr_row_aux): the f6p tier's gmax.  _at: rows
 * [row0, row0 + R) of a tile buffer (append).                                                              */
size_t ofr_f6p_tiles_bytes(int64_t R, int pstages);
int ofr_f6p_quantize_rows_at(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, int64_t row0,
                             int pstages, void* tiles, size_t tiles_bytes, float* scale, double* stats,
                             const uint8_t* bscale);
int ofr_f6p_quantize_rows(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, int pstages, void* tiles,
                          size_t tiles_bytes, float* scale, double* stats, const float* paux, double* maxima,
                          const uint8_t* bscale);
/* ofr_knn_f6p_sampled (and ofr_knn_f6p_merge_pruned): Gt, gscale, gmax are the prefix tier's own gallery tiles,
 * scales and maxima above (round 6; round 5 read the f6 tiles); St / sscale: the f6 tier's row sample.     */
int ofr_knn_f6p_sampled(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                        const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg, int64_t d,
                        const void* Gt, const float* gscale, const float* aux, const double* gmax, int k,
                        int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound, const void* St,
                        int64_t Ns, const float* sscale, const float* saux, void* workspace, size_t workspace_bytes,
                        const uint8_t* bscale, int pstages);
/* The row step of the sample (64) and its builder: gallery rows j * 64 for j in [j0, j1) (X = row 0
 * of the N-row fp32 gallery, ldx its leading dimension; j1 <= ceil(N / 64)) are quantized into sample
 * row j of tiles / scale / stats (as ofr_f6_quantize_rows_at) and saux[j] = aux[j * 64].  A gallery of
 * N rows has j1 = ceil(N / 64); an append of rows [N0, N1) extends it with j0 = ceil(N0 / 64),
 * j1 = ceil(N1 / 64) (N = N1).                                                                    */
int64_t ofr_f6_sample_step(void);
int ofr_f6_sample_rows(void* stream, const float* X, int64_t N, int64_t ldx, int64_t d, int64_t j0, int64_t j1,
                       const float* aux, void* tiles, size_t tiles_bytes, float* scale, double* stats, float* saux,
                       const uint8_t* bscale);
/* Phase 2 of ofr_knn_f6 split for a gallery sharded over ranks (new; replaces the
 * per-rank re-rank of classifier.py:104-119's loop at G > 1).  After phase 1 on every shard:
 *   stage 1 selects each query's 16 candidates into the workspace and writes ub[B][k] -- upper
 *           bounds of the squared distances of its best k candidates (ascending, +inf past the
 *           list);
 *   the caller takes, per query, the k-th smallest of every rank's ub values (an upper bound of
 *           the GLOBAL k-th squared distance) into ub[B];
 *   stage 2 re-ranks the selection exactly but skips every candidate whose lower bound exceeds
 *           ub[q] (it cannot be among the global k nearest), then writes out_d/out_i/cert/bound
 *           as phase 2 does (a shard holding none of a query's neighbours re-ranks nothing).
 * Same arguments as ofr_knn_f6 (phases replaced by stage; out_d/out_i/cert/bound only read by
 * stage 2); the workspace carries the selection between the stages.                          */
int ofr_knn_f6_merge_pruned(void* stream, int stage, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                            const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg,
                            int64_t d, const void* Gt, const float* gscale, const float* aux, const double* gmax,
                            int k, int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound,
                            double* ub, void* workspace, size_t workspace_bytes);
/* The same split for the prefix tier (round 6; after phase 1 of ofr_knn_f6p_sampled, aux = the prefix
 * terms): a prefix key bounds no distance from above, so stage 1 computes the exact squared distances
 * of each query's first k candidates (key order) and writes those, ascending, as ub[B][k] -- k real rows
 * of the shard lie that close.  Stage 2 as above (lower bounds from the prefix keys).              */
int ofr_knn_f6p_merge_pruned(void* stream, int stage, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                             const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg,
                             int64_t d, const void* Gt, const float* gscale, const float* aux, const double* gmax,
                             int k, int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound,
                             double* ub, void* workspace, size_t workspace_bytes, int pstages);

/* Two-slice fp6 tier "f6x2" of the certified chain (new: replaces the same loop,
 * classifier.py:104-119, for the queries the fp6 tier could not certify on crowded
 * galleries).  x~ = s (v1 + 2^-4 v2): v1 exactly the fp6 tier's codes and scale (a
 * gallery shares its f6 tiles as the first slice), v2 the e2m3 codes of
 * 2^4 (x/s - v1) in a second tiled buffer of ofr_f6_tiles_bytes(R, d) bytes.
 * stats[3] = (s(|v1| + 2^-4 |v2|), ||x - x~||, s 2^-4 |v2|).  tiles1 may be null
 * (only the second slice and the stats are written).
 * ofr_knn_f6x2: the ofr_knn_f6 sieve (B > 32 only) over three segments of stages,
 * [v1 | v1 | v2] . [w1 | w2 | w1] with E8M0 block scale 2^-4 on the second slices,
 * i.e. the coarse products v1.w1 + 2^-4 (v1.w2 + v2.w1); the certificate adds
 * 2 t_q T for the dropped 2^-8 v2.w2 term and the fp32 accumulation bound of
 * 3 nst MFMAs.  Same contract and workspace (ofr_knn_f6_workspace_bytes).        */
int ofr_f6x2_quantize_rows(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, void* tiles1,
                           void* tiles2, size_t tiles_bytes, float* scale, double* stats, const float* aux,
                           double* maxima, const uint8_t* bscale);
int ofr_f6x2_quantize_rows_at(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, int64_t row0,
                              void* tiles1, void* tiles2, size_t tiles_bytes, float* scale, double* stats,
                              const uint8_t* bscale);
/* ofr_knn_f6x2 with the sieve thresholds from the row sample (as ofr_knn_f6_sampled): St / sscale /
 * saux the fp6 tier's sample (ofr_f6_sample_rows), St2 the second slices of the same rows
 * (ofr_f6x2_sample_rows: rows j * 64 for j in [j0, j1) into sample row j of tiles2, with their scales
 * and f6x2 stats).                                                                               */
int ofr_f6x2_sample_rows(void* stream, const float* X, int64_t N, int64_t ldx, int64_t d, int64_t j0, int64_t j1,
                         void* tiles2, size_t tiles_bytes, float* scale, double* stats, const uint8_t* bscale);
int ofr_knn_f6x2_sampled(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                         const void* Qt2, const float* qscale, const double* qstats, const float* G, int64_t N,
                         int64_t ldg, int64_t d, const void* Gt, const void* Gt2, const float* gscale,
                         const float* aux, const double* gmax, int k, int64_t index_base, double* out_d,
                         int64_t* out_i, int* cert, double* bound, const void* St, const void* St2, int64_t Ns,
                         const float* sscale, const float* saux, void* workspace, size_t workspace_bytes,
                         const uint8_t* bscale);
int ofr_knn_f6x2(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt, const void* Qt2,
                 const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg, int64_t d,
                 const void* Gt, const void* Gt2, const float* gscale, const float* aux, const double* gmax, int k,
                 int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound, void* workspace,
                 size_t workspace_bytes, const uint8_t* bscale);

/* Any k (round 5; replaces NearestNeighbor.predict classifier.py:104-119 for the k the tiers
 * above do not serve -- they keep 16 candidates per tile): the reference's distance of every
 * (query, row) pair in fp64 (Euclidean distance.py:57-60, Cosine :74-77 with NaN for a zero row,
 * ChiSquare :112-116), then per query the k smallest by (distance, row), NaN last.  Q [B][ldq] of
 * qdtype, G [N][ldg] of gdtype (OFR_DT_*; integer rows are counts, value = count / denom as the
 * reference's float64 histograms; denom 1 for float rows).  out_d / out_i [B][k]; entries past
 * min(k, N) are (+inf, -1).  Any k: min(k, N) <= 4096 by a radix select in LDS, above it by a
 * stable segmented radix sort (buffers of up to ~1.5 GiB allocated per call).  Each distance is the
 * reference formula in fp64 summed in feature order: within ~1 ulp of numpy's pairwise sum.  Workspace
 * ofr_knn_deep_workspace_bytes(B, N) bytes (a block of the distance matrix, <= 2 GiB).          */
size_t ofr_knn_deep_workspace_bytes(int64_t B, int64_t N);
int ofr_knn_deep(void* stream, int metric, const void* Q, int64_t B, int64_t ldq, int qdtype, const void* G,
                 int64_t N, int64_t ldg, int gdtype, int64_t d, double denom, int k, int64_t index_base,
                 double* out_d, int64_t* out_i, void* workspace, size_t workspace_bytes);

/* Merge P sorted (distance, index) lists per query into the best k:
 * in_d/in_i [B][P*kin] (list p at columns [p*kin, (p+1)*kin)), ascending by
 * (distance, index); out [B][k].  Used after the RCCL all-gather of per-rank
 * results (gallery sharded across GPUs).                                     */
int ofr_topk_merge(void* stream, const double* in_d, const int64_t* in_i, int64_t B, int P,
                   int kin, int k, double* out_d, int64_t* out_i);

/* ExtendedLBP + SpatialHistogram --------------------------------------------
 * Replaces ExtendedLBP.__call__ lbp.py:80-130 and
 *          SpatialHistogram.spatially_enhanced_histogram feature.py:286-302.
 * imgs: uint8 [n][H][W] contiguous.  Geometry (from the host, lbp.py:84-121):
 * P sample points, offs[P][4] = (fy, fx, cy, cx) int32, w[P][4] fp64
 * (w1..w4), origin (oy, ox), block (by, bx).  The interpolated neighbour is
 * evaluated in the reference's fp64 order without contraction:
 *   N = w1*X[fy][fx]; N += w2*X[fy][cx]; N += w3*X[cy][fx]; N += w4*X[cy][cx]
 * and bit i of the code is (N >= C), C = uint8 centre pixel.
 * codes: uint32 [n][H-by+1][W-bx+1].                                         */
int ofr_elbp_codes(void* stream, const uint8_t* imgs, int64_t n, int H, int W, int P,
                   const int32_t* offs_host, const double* w_host, int oy, int ox, int by, int bx,
                   uint32_t* codes);
/* counts: [n][gr*gc][2^P] of `count_bytes` (1, 2 or 4) unsigned integers;
 * cell (r,c) covers code rows [r*py,(r+1)*py) x cols [c*px,(c+1)*px),
 * py = floor(dy/gr), px = floor(dx/gc).  The float histogram of the
 * reference is count / (py*px) exactly (np.histogram density=True).  P <= 15.
 * (The geometry form the package binds; SURVEY §8b's context form is
 * ofr_elbp_hist, declared with the other context entry points below.)      */
int ofr_elbp_hist_geom(void* stream, const uint8_t* imgs, int64_t n, int H, int W, int P,
                       const int32_t* offs_host, const double* w_host, int oy, int ox, int by, int bx,
                       int gr, int gc, void* counts, int count_bytes);

/* Chi-square search ----------------------------------------------------------
 * Replaces ChiSquareDistance distance.py:112-116 inside NearestNeighbor.predict.
 * Q [B][ldq], G [N][ldg] rows of `nbins` values of type dtype (OFR_DT_*); the
 * reference value of an element is x / denom (denom = py*px for the counts
 * of ofr_elbp_hist / ofr_elbp_hist_geom, whose float histogram is count/(py*px); 1.0 for fp32).
 * Rows must be 16-byte aligned.  Coarse fp32 VALU pass + exact fp64
 * re-evaluation of the reference formula on the best candidates; outputs as
 * ofr_knn_f32.  cert (nullable, [B]): 1 iff the result is provably the exact
 * fp64 top-k -- the k-th exact distance lies below every excluded row's
 * coarse score / (1 + gamma), gamma the coarse pass's relative error bound
 * ((ceil(nbins/2) + 4) 2^-24 + 2 ulp per term).  Queries with cert 0 are
 * re-run by ofr_chi2_knn_exact: the same search with fp64 per-term arithmetic
 * (the reference formula in every tile; its cert covers the fp32 tile keys).   */

size_t ofr_chi2_workspace_bytes(int64_t B, int64_t N, int k);
/* uint8 counts (dtype 0, nbins % 64 == 0, 16-byte rows) take a low-rank MFMA coarse pass instead
 * of the VALU one: (a-c)^2/(a+c) = a + c - 4 ac/(a+c) and ac/(a+c) ~= sum_{r<8} U[a][r] U[c][r]
 * (an fp16 table, v_mfma_f32_16x16x32_f16), |S - S~| <= bound * (Tq + Tg) in count units with
 * Tq, Tg the rows' total counts; ofr_chi2_mfma_bound(nbins) returns that factor.
 * OFR_CHI2_ENGINE=valu keeps the VALU pass.                                    */
double ofr_chi2_mfma_bound(int64_t nbins);
/* the fp16 table U [256][8] (bits) of that pass, host memory (tests re-derive the bound from it) */
void ofr_chi2_table(uint16_t* out);
int ofr_chi2_knn(void* stream, int dtype, const void* Q, int64_t B, int64_t ldq, const void* G, int64_t N,
                 int64_t ldg, int64_t nbins, double denom, int k, int64_t index_base, double* out_d,
                 int64_t* out_i, void* workspace, size_t workspace_bytes, int* cert);
int ofr_chi2_knn_exact(void* stream, int dtype, const void* Q, int64_t B, int64_t ldq, const void* G, int64_t N,
                       int64_t ldg, int64_t nbins, double denom, int k, int64_t index_base, double* out_d,
                       int64_t* out_i, void* workspace, size_t workspace_bytes, int* cert);

/* Training (PCA Gram / LDA scatter) ----------------------------------------
 * C[M][N] = alpha * op(A) op(B) + beta * C in fp64 on the fp64 MFMA
 * (v_mfma_f64_16x16x4_f64); op(X) = X or X^T (row-major storage).  Replaces
 * the fp64 products of PCA.compute feature.py:91-94 (Gram / covariance of the
 * centred data for the eigensolve that replaces np.linalg.svd), LDA.compute
 * feature.py:162-168 (Sw = Fc^T Fc, Sb = Mc^T diag(n) Mc), Fisherfaces.compute
 * feature.py:229 (W = P.L) and the training projections.                    */
int ofr_gemm_f64(void* stream, int transA, int transB, int64_t M, int64_t N, int64_t K,
                 double alpha, const double* A, int64_t lda, const double* B, int64_t ldb,
                 double beta, double* C, int64_t ldc);
/* mean[j] = (1/N) sum_n X[n][j] for uint8 X (exact integer sums; equals
 * numpy's XC.mean(axis=1) of the uint8 column matrix, feature.py:91).        */
int ofr_col_mean_u8(void* stream, const uint8_t* X, int64_t N, int64_t D, int64_t ldx,
                    double* mean);
/* mean[j] = (1/N) sum_n X[n][j] for fp64 X (row chunks summed in fixed order). */
int ofr_col_mean_f64(void* stream, const double* X, int64_t N, int64_t D, int64_t ldx,
                     double* mean);
/* out[n][j] = X[n][j] - mean[j] (uint8 X -> fp64), feature.py:92.            */
int ofr_center_u8_f64(void* stream, const uint8_t* X, int64_t N, int64_t D, int64_t ldx,
                      const double* mean, double* out, int64_t ldo);
/* out[n][j] = X[n][j] - mean[j] (fp64).                                      */
int ofr_sub_mean_f64(void* stream, const double* X, int64_t N, int64_t D, int64_t ldx,
                     const double* mean, double* out, int64_t ldo);
/* Scale every column of U [rows][ldu] to unit 2-norm (zero columns stay zero):
 * the left singular vectors from the Gram eigenvectors, U = XC^T V / sigma.   */
int ofr_normalize_cols_f64(void* stream, double* U, int64_t rows, int64_t cols, int64_t ldu);
/* Class means and class-centred rows for LDA (feature.py:164-167):
 * perm [N] = row indices grouped by class, offsets [c+1] (device int64),
 * means [c][D] = mean of each class's rows, Fc [N][D] = F - means[y] and
 * Mc [c][D] = means[i] - total_mean, Mc_n [c][D] = n_i * Mc[i]; total_mean [D] given. */
int ofr_class_center_f64(void* stream, const double* F, int64_t N, int64_t D, int64_t ldf,
                         const int64_t* perm, const int64_t* offsets, int64_t c,
                         const double* total_mean, double* means, double* Fc, double* Mc,
                         double* Mc_n);
/* The same statistics in pieces, for a training set sharded over ranks (round 4; the caller
 * all-reduces the sums and counts in between): ofr_class_sums_f64 sums[c][D] = per-class sums of
 * this rank's rows; ofr_class_between_f64 means = sums / counts (0 for an empty class), Mc, Mc_n
 * as above from the global sums, counts [c] (fp64) and total_mean; ofr_class_sub_f64 Fc = F -
 * means[y] for this rank's rows.                                                             */
int ofr_class_sums_f64(void* stream, const double* F, int64_t D, int64_t ldf, const int64_t* perm,
                       const int64_t* offsets, int64_t c, double* sums);
int ofr_class_between_f64(void* stream, const double* sums, const double* counts, int64_t c, int64_t D,
                          const double* total_mean, double* means, double* Mc, double* Mc_n);
int ofr_class_sub_f64(void* stream, const double* F, int64_t N, int64_t D, int64_t ldf, const int64_t* perm,
                      const int64_t* offsets, int64_t c, const double* means, double* Fc);

/* Exact training products of uint8 face data (Fisherfaces.compute) -------------
 * Replaces the float64 products of PCA.compute feature.py:91-94 (Gram XC XC^T of
 * the centred images, or their covariance XC^T XC) and LDA.compute feature.py:
 * 160-168 (Sw, Sb) when they are taken over pixels.  With x' = x - 128:
 *   ofr_pad_u8         out [rows'][ldo] = X or X^T, pad columns = 128 (x' = 0);
 *   ofr_gram_u8        C[R][R] = X' X'^T over K columns, EXACT (int8 MFMA, int32
 *                      per chunk of < 2^17 columns, chunks summed in fp64), X the
 *                      padded uint8 [R][ld] (ld % 128 == 0), both triangles written;
 *   ofr_class_sums_u8  sums[c][D] = per-class column sums of x - shift (shift 0 or
 *                      128; exact, fp64 storage), means (nullable) = sums / n_class;
 *   ofr_row_dot_u8     r[n] = sum_j (X[n][j] - 128) s[j] (exact int64, fp64 out);
 *   ofr_center_gram_f64   C[a][b] += alpha (u[a] + u[b]) + beta (R < 65536);
 *   ofr_scatter_combine_f64  Sw = G - T (skipped when Sw is NULL), Sb = T - s s^T / N
 *                      (all [D][ld]);
 *   ofr_rank1_f64      C[a][b] += alpha u[a] v[b];
 *   ofr_row_div_f64    out[r][j] = A[r][j] / n[r] (class means from class sums).       */
int ofr_pad_u8(void* stream, const uint8_t* X, int64_t rows, int64_t cols, int64_t ldx, int transpose,
               uint8_t* out, int64_t ldo);
int ofr_gram_u8(void* stream, const uint8_t* X, int64_t R, int64_t K, int64_t ld, double* C, int64_t ldc);
int ofr_class_sums_u8(void* stream, const uint8_t* X, int64_t D, int64_t ldx, const int64_t* perm,
                      const int64_t* offsets, int64_t c, int shift, double* sums, double* means);
int ofr_row_dot_u8(void* stream, const uint8_t* X, int64_t N, int64_t D, int64_t ldx, const double* s,
                   double* r);
int ofr_center_gram_f64(void* stream, double* C, int64_t R, int64_t ldc, const double* u, double alpha,
                        double beta);
int ofr_scatter_combine_f64(void* stream, const double* G, const double* T, const double* s, double invN,
                            int64_t D, int64_t ld, double* Sw, double* Sb);
int ofr_rank1_f64(void* stream, double* C, int64_t rows, int64_t cols, int64_t ldc, const double* u,
                  const double* v, double alpha);
int ofr_row_div_f64(void* stream, const double* A, int64_t rows, int64_t cols, int64_t lda, const double* n,
                    double* out, int64_t ldo);

/* Multi-GPU search in one process ---------------------------
 * ofr_comm_init_all: one RCCL rank per device (ncclCommInitAll over xGMI; RCCL is
 * bound at run time, OFR_E_UNSUPPORTED when librccl.so.1 is absent); devices NULL
 * = 0 .. ndev-1.  ofr_knn_sharded: shard r (on devices[r], its own stream) holds
 * the gallery rows [index_base, index_base + N) of a row-sharded gallery with its
 * fp6 tier (ofr_f6_quantize_rows) and the replicated query batch (centred fp32
 * rows + fp6 tiles, as for ofr_knn_f6).  Every shard runs the certified fp6 tier,
 * ONE ncclAllGather exchanges the (distance, index, bound) lists, every device
 * merges them (ofr_topk_merge_certify) and certifies a query iff the global k-th
 * squared distance is below every rank's bound.  Uncertified queries go down the
 * tier chain of the single-GPU search on every shard, each stage exchanged and
 * certified the same way: the two-slice fp6 tier (f6x2, when every shard gives
 * Gt2 / gscale2 / gmax2 from ofr_f6x2_quantize_rows), the two-slice int8 tier
 * (when every shard gives G8 / ld8 / gscale8 / gmax8 from ofr_q8_quantize_rows,
 * slices 2), then the exact fp32 pass (ofr_knn_f32); a stage with <= 32 open
 * queries goes straight to the exact pass.  Output on EVERY device: out_d / out_i
 * [B][k] = the exact top-k of the whole gallery (classifier.py:104-119), cert [B]
 * = 1 if a quantized tier certified the query (0: the exact pass resolved it);
 * tier_counts (optional, [4]): open queries after the fp6 tier, after f6x2,
 * after int8 x2, and the number the exact pass ran (-1: stage not run).
 * Euclidean, k <= 16.  workspace: ofr_knn_sharded_workspace_bytes per shard.   */
typedef struct ofr_comm ofr_comm;
typedef struct ofr_knn_shard {
  void* stream;
  const float* Q;
  int64_t ldq;
  const void* Qt;
  const float* qscale;
  const double* qstats;
  const float* G;
  int64_t N;
  int64_t ldg;
  const void* Gt;
  const float* gscale;
  const float* aux;
  const double* gmax;
  int64_t index_base;
  void* workspace;
  size_t workspace_bytes;
  double* out_d;
  int64_t* out_i;
  int* cert;
  /* optional finer tiers (null pointers: the stage is skipped) */
  const void* Gt2;          /* f6x2: second-slice tiles of the shard's rows (first slice = Gt) */
  const float* gscale2;     /* f6x2: row scales */
  const double* gmax2;      /* f6x2: gallery maxima */
  const int8_t* G8;         /* int8 x2: slices [N][ld8] */
  int64_t ld8;
  const float* gscale8;
  const double* gmax8;
  int64_t* tier_counts;     /* optional out [4] (read on shard 0) */
  /* optional row sample of the shard's rows for the fp6 sieve thresholds (ofr_f6_sample_rows;
     null St: the panel sample of ofr_knn_f6) -- round 4, appended */
  const void* St;
  int64_t Ns;
  const float* sscale;
  const float* saux;
  const void* St2;          /* optional: the second slices of the sample (ofr_f6x2_sample_rows) for f6x2 */
  /* the shard's column-block scales (ofr_f6_block_scales; null: unit), also those of its query tiles
     Qt -- round 5, appended */
  const uint8_t* bscale;
  /* optional prefix tier f6p first (ofr_knn_f6p_sampled) -- round 6, appended.  pstages > 0
     (the same on every shard: choose it from all-reduced block sums) runs it for the whole batch, with
     its pruned split merge (ofr_knn_f6p_merge_pruned), the exchange and the global certificate; the
     queries it leaves open then take the fp6 tier (Qt, qscale, qstats are not read for the batch) and
     the rest of the chain.  Needs the row sample (St). */
  int pstages;
  const void* Qtp;          /* the batch's prefix tiles (ofr_f6_quantize_rows_prefix) */
  const float* qscalep;
  const double* qstatsp;
  const float* paux;        /* the shard rows' prefix terms |g_m|^2 (ofr_row_aux over min(d, 128 pstages)) */
  const float* spaux;       /* the row sample's prefix terms */
  int64_t* prefix_open;     /* optional out [1] (shard 0): queries the prefix tier left open */
  /* the prefix tier's own gallery tiles of the shard's rows (ofr_f6p_quantize_rows: pstages stages per
     panel, power-of-two row scales), their row scales and maxima -- needed when pstages > 0 (round 6) */
  const void* Gtp;
  const float* gscalep;
  const double* gmaxp;
} ofr_knn_shard;
int ofr_comm_init_all(int ndev, const int* devices, ofr_comm** comm);
int ofr_comm_destroy(ofr_comm* comm);
int ofr_comm_size(const ofr_comm* comm);
size_t ofr_knn_sharded_workspace_bytes(int64_t B, int64_t N, int64_t ldq, int k, int ndev);
int ofr_knn_sharded(ofr_comm* comm, const ofr_knn_shard* shards, int64_t B, int64_t d, int k);
/* lists [P][B][2k+1] fp64: per rank and query k distances, k indices (int64
 * bit patterns), the rank's bound -> the best k per query and the global
 * certificate (bound -inf / NaN never certifies; +inf always does).             */
int ofr_topk_merge_certify(void* stream, const double* lists, int P, int64_t B, int k, double* out_d,
                           int64_t* out_i, int* cert);
/* The pieces of that exchange for callers with their own transport (the package's
 * torch.distributed path, parallel.py):
 * ofr_topk_pack: d [B][k] fp64, i [B][k] int64, bound [B] (NULL: +inf) -> out [B][2k+1]
 * (the layout ofr_topk_merge_certify reads, one rank's block);
 * ofr_kth_bound: all [P][B][k] fp64, each rank's k upper bounds ascending -> ub [B] = the
 * k-th smallest of the P*k (the pruned merge's global bound, classifier.py:113-119 across
 * shards);
 * ofr_open_rows: cert [B] int -> rows[0..count) = the b with cert[b] == 0, ascending, and
 * count[0] (device; the caller reads count to size the next tier).                    */
int ofr_topk_pack(void* stream, const double* d, const int64_t* i, const double* bound, int64_t B, int k, double* out);
int ofr_kth_bound(void* stream, const double* all, int P, int64_t B, int k, double* ub);
int ofr_open_rows(void* stream, const int* cert, int64_t B, int64_t* rows, int* count);

/* Face-tensor ingestion ------------------------------------
 * Replaces cv2.imread(IMREAD_GRAYSCALE) + cv2.resize(im, size) [INTER_LINEAR] of
 * TheTrainer.read_images trainer/thetrainer.py:99-103 and the recognizers'
 * img[y0:y1, x0:x1] -> cv2.cvtColor(BGR2GRAY) -> cv2.resize(size, INTER_CUBIC)
 * (../bin/ocvf_recognizer.py:64-66), for a ragged batch in ONE launch.
 * src: device bytes holding every source image; jobs: device int64 [n][7] =
 * (byte offset of the image, row pitch in bytes, crop x0, y0, width, height,
 * channels 1 = grey | 3 = BGR | 4 = BGRA); crops must lie inside their image.
 * out: uint8 [n][dh][dw].  interp 1 = INTER_LINEAR, 2 = INTER_CUBIC, in
 * OpenCV's 8-bit fixed point (11-bit coefficients; grey = (1868 B + 9617 G +
 * 4899 R + 2^13) >> 14); a crop of the output size is copied (grey only).       */
int ofr_ingest_faces(void* stream, const uint8_t* src, const int64_t* jobs, int64_t n, int dh, int dw,
                     int interp, uint8_t* out);

/* Training eigensolves on the device -------------------------
 * Replace the host LAPACK of PCA (feature.py:94 svd -> eigh of the Gram /
 * covariance, training.py) and LDA (feature.py:170 eig(inv(Sw) Sb) -> the
 * symmetric-definite pencil Sb v = lambda Sw v, feature.lda_eigen): rocSOLVER
 * divide and conquer (dsyevd / dsygvd, bound at run time: OFR_E_UNSUPPORTED
 * without librocsolver.so.0).  A, Sb, Sw: contiguous symmetric [n][n] fp64,
 * OVERWRITTEN.  Out: the m largest eigenvalues, descending, evals[m]; their
 * eigenvectors as the columns of row-major evecs [n][ldv] (ofr_eigh_f64:
 * orthonormal; ofr_sygv_f64: each scaled to unit 2-norm, as lda_eigen).
 * OFR_E_NUMERIC when Sw is not positive definite (the caller falls back to the
 * reference's general eig) or the solver did not converge.  Synchronises the
 * stream (reads the solver's info).                                              */
size_t ofr_eig_workspace_bytes(int64_t n, int64_t m);
int ofr_eigh_f64(void* stream, int64_t n, double* A, int64_t m, double* evals, double* evecs, int64_t ldv,
                 void* workspace, size_t workspace_bytes);
int ofr_sygv_f64(void* stream, int64_t n, double* Sb, double* Sw, int64_t m, double* evals, double* evecs,
                 int64_t ldv, void* workspace, size_t workspace_bytes);

/* Context-based entry points (SURVEY §8b contract) ---------------------------
 * For FFI callers holding the reference's plain row-major numpy layouts; each
 * call lays its operands out for the kernels above in a workspace the context
 * owns (grown on demand; a call may synchronise the stream when it grows).  A
 * context belongs to one device and one thread at a time.
 * ofr_project_u8: Y [B][d] fp32 = W^T (x - mu) for uint8 faces X [B][D] and
 *   W [D][d] fp32 row-major (Fisherfaces.project feature.py:241-242 with mu
 *   NULL; PCA.project :114-116 with mu [D] fp64) on the exact int8-slice engine
 *   (exact products and sums, one rounding; OFR_FP64_ACC is accepted and always
 *   in effect).  OFR_PROJ_REUSE_W: W is unchanged since the context's last
 *   call with the same pointer and shape -> its prepared slices are reused.
 * ofr_gram: G = A^T A [cols][cols] (OFR_GRAM_ATA) or A A^T [rows][rows]
 *   (OFR_GRAM_AAT) of fp32 A [rows][cols] (feature.py:91-94): products exact
 *   in fp64, fp64 accumulation on the fp64 MFMA; G fp32 or fp64 (prec =
 *   OFR_DT_F32 / OFR_DT_F64).
 * ofr_scatter: fp64 Sw, Sb [d][d] and class means [c][d] (nullable) of fp32
 *   features F [N][d] with int32 device labels y in 0..c-1 (feature.py:160-168).
 * ofr_knn: top-k of fp32 queries Q [B][d] against G [N][d] (Euclidean /
 *   Cosine: exact fp64 re-rank of the fp32-MFMA candidates; ChiSquare: the
 *   certified fp32 pass + exact fp64 pass for the rest, values used as given);
 *   g_norms nullable (EUCLIDEAN: ||g||^2, COSINE: 1/||g||, as ofr_row_aux);
 *   out_d fp32 [B][k] (distance.py values), out_i int64 [B][k] (+ index_base).
 * ofr_elbp_hist: ExtendedLBP codes + SpatialHistogram counts (lbp.py:80-130,
 *   feature.py:286-302) of uint8 faces imgs [n][H][W]; host arrays w [P][4] fp64
 *   and off [P][4] int32 = (fy, fx, cy, cx) of each sample point RELATIVE TO THE CENTRE
 *   pixel (floor / ceil of the reference's sample point, lbp.py:84-121); the
 *   block origin and size follow from them as in lbp.py:90-97.  counts uint8
 *   [n][gr*gc][2^P] (cells of at most 255 pixels, else OFR_E_UNSUPPORTED: use
 *   ofr_elbp_hist_geom with wider counts); the reference histogram is
 *   count / (py*px).                                                             */
typedef struct ofr_ctx ofr_ctx;
enum { OFR_FP64_ACC = 1, OFR_PROJ_REUSE_W = 2 };
enum { OFR_GRAM_ATA = 0, OFR_GRAM_AAT = 1 };
int ofr_ctx_create(int device, ofr_ctx** ctx);
int ofr_ctx_destroy(ofr_ctx* ctx);
int ofr_project_u8(ofr_ctx* ctx, void* stream, const uint8_t* X, int64_t B, int64_t D, const float* W, int64_t d,
                   const double* mu_or_null, float* Y, int flags);
int ofr_gram(ofr_ctx* ctx, void* stream, const float* A, int64_t rows, int64_t cols, int side, int prec, void* G);
int ofr_scatter(ofr_ctx* ctx, void* stream, const float* F, const int32_t* y, int64_t N, int64_t d, int32_t c,
                void* Sw, void* Sb, void* means);
int ofr_knn(ofr_ctx* ctx, void* stream, int metric, const float* Q, int64_t B, const float* G,
            const float* g_norms_or_null, int64_t N, int64_t d, int k, int64_t index_base, float* out_d,
            int64_t* out_i);
int ofr_elbp_hist(ofr_ctx* ctx, void* stream, const uint8_t* imgs, int64_t n, int H, int W, const double* w,
                  const int32_t* off, int P, int gr, int gc, uint8_t* counts);

#ifdef __cplusplus
}
#endif
#endif /* OFR_H */

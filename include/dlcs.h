/*
 * libdlcs_hip -- C-ABI of the MI355X-native Swin-unrolled cine reconstruction
 * hot path (gfx950).  Plain pointers and sizes only: no torch types.
 *
 * Conventions (every entry point):
 *   - pointers are DEVICE pointers; complex64 = interleaved float2 (torch layout);
 *   - `dtype` selects the storage type of real activations/weights:
 *       DLCS_F32 (fp32 parity build) or DLCS_BF16 (fast path); accumulation is fp32;
 *   - `stream` is a hipStream_t (torch's current stream when called from Python);
 *   - no allocation, no host synchronisation, no global mutable state: callers
 *     pass workspaces; every call is re-entrant and graph-capturable;
 *   - return 0 on success, a hipError_t value, or a DLCS_ERR_* code; never abort.
 *
 * Each function cites the reference interface it replaces (paths relative to
 * the reference repository tjtiger86/dl-swin-gan):
 *   tr  = dl_cs/mri/transforms.py        urs = dl_cs/models/unrolledswin.py
 *   s3d = dl_cs/models/swin3D.py         vst = dl_cs/models/video_swin_transformer_mri_downsample.py
 */
#ifndef DLCS_H
#define DLCS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLCS_VERSION 1

enum dlcs_dtype { DLCS_F32 = 0, DLCS_BF16 = 1 };

enum dlcs_status {
    DLCS_OK = 0,
    DLCS_ERR_INVALID_ARG = 100001,
    DLCS_ERR_UNSUPPORTED_SIZE = 100002,
    DLCS_ERR_WORKSPACE = 100003
};

typedef void* dlcs_stream_t; /* hipStream_t */

int dlcs_version(void);
const char* dlcs_status_string(int status);
/* Library-internal scratch: a few per-(device, stream) partial buffers of the
 * fp32 split kernels (split-K / tail / slab partials, column sums; ~220 MB per
 * stream at the BASELINE slice), allocated with hipMalloc on first use and
 * kept for the process (outside torch's caching allocator).  bytes = their
 * total; release = synchronise the devices that own them and free them all
 * (they are re-allocated on the next launch that needs one).                */
size_t dlcs_scratch_bytes(void);
int dlcs_release_scratch(void);

/* ---------------------------------------------------------------------------
 * SENSE operator -- tr:49-110 (SenseModel), tr:12-46 (FFT, ortho, uncentered).
 *   x       c64 [B,E,T,Y,X]      maps c64 [B,E,C,1,Y,X]
 *   weights f32 [B,Wc,T,Y,X] (Wc = 1 broadcast over coils, or C) or NULL
 *   y       c64 [B,C,T,Y,X]
 * Y and X must factor into 2,3,5 and be <= 1024.
 * workspace: dlcs_sense_workspace_bytes() bytes (one k-space-sized buffer).
 * ------------------------------------------------------------------------- */
size_t dlcs_sense_workspace_bytes(int64_t B, int64_t C, int64_t T, int64_t Y, int64_t X);

/* y = W * F( sum_e S_e x_e )                       -- tr:92-98 (_forward_op) */
int dlcs_sense_fwd(const void* x, const void* maps, const float* weights, int64_t weights_coils,
                   void* y, int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                   void* workspace, size_t workspace_bytes, dlcs_stream_t stream);

/* x = sum_c conj(S_c) F^-1( W * y_c )               -- tr:84-90 (_adjoint_op)
 * Fused epilogue (urs:109, the PGD data-consistency step):
 *   out = base + step * (x - sub)   when base != NULL   (sub may be NULL = 0)
 *   out = x                          when base == NULL                    */
int dlcs_sense_adj(const void* y, const void* maps, const float* weights, int64_t weights_coils,
                   void* out, const void* base, const void* sub, float step,
                   int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                   void* workspace, size_t workspace_bytes, dlcs_stream_t stream);

/* out = base_scale * x + step * (A^H A x - sub)   (sub may be NULL = 0; out != x)
 *   PGD data-consistency step (urs:109):  base_scale 1, step s, sub = A^H y
 *   HQS normal operator (urs:151):        base_scale lamda, step 1, sub NULL
 * Three launches, one k-space-sized workspace (the column pass runs FFT_Y,
 * weights^2 and IFFT_Y on a tile in LDS).                                    */
int dlcs_sense_normal(const void* x, const void* maps, const float* weights, int64_t weights_coils,
                      void* out, const void* sub, float base_scale, float step,
                      int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                      void* workspace, size_t workspace_bytes, dlcs_stream_t stream);

/* Conjugate gradient (alg:50-73, ConjugateGradient.forward) on the normal
 * equations (A^H A + lamda I) x = b of urs:151-158: num_iter steps from x, in
 * place on x.  All scalars of the recurrence stay on the device (fp64 partial
 * reductions, complex64 alpha/beta as the reference's torch scalars); no host
 * synchronisation.  workspace: dlcs_sense_cg_workspace_bytes() bytes.       */
size_t dlcs_sense_cg_workspace_bytes(int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X);
int dlcs_sense_cg(void* x, const void* b, const void* maps, const float* weights, int64_t weights_coils,
                  float lamda, int num_iter, int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                  void* workspace, size_t workspace_bytes, dlcs_stream_t stream);

/* Row-sparse normal operator for k-t undersampling masks (tr:84-98 composed
 * as in urs:109 / urs:151; the cine masks of subsample.py sample ~15 of 192
 * phase-encode lines per frame).  A line y of frame t whose weights
 * W(t, y, :) are all zero contributes nothing to A^H W^2 A, so the 2D FFT is
 * taken Y first and only the sampled lines are carried through FFT_X / W^2 /
 * IFFT_X (a compressed k-space of B C T jcap X c64) before the zero-filled
 * IFFT_Y, the conj-map coil sum and the DC epilogue.  Same result as
 * dlcs_sense_normal up to fp32 rounding; Y and X in {64,80,96,128,160,192},
 * X % 16 == 0, E <= 2.
 *   table: dlcs_sense_rowtab_bytes() bytes, filled by dlcs_sense_rowtab once
 *          per weights tensor: int32 [0] = jmax (most lines of any frame),
 *          then counts[B Wc T] and line indices [B Wc T][Y];
 *   jcap:  >= jmax (read back by the caller once per mask);
 *   workspace: dlcs_sense_rows_workspace_bytes(B, C, T, jcap, X) bytes.      */
size_t dlcs_sense_rowtab_bytes(int64_t B, int64_t weights_coils, int64_t T, int64_t Y);
int dlcs_sense_rowtab(const float* weights, int64_t weights_coils, int64_t B, int64_t T, int64_t Y, int64_t X,
                      void* table, size_t table_bytes, dlcs_stream_t stream);
size_t dlcs_sense_rows_workspace_bytes(int64_t B, int64_t C, int64_t T, int64_t jcap, int64_t X);
int dlcs_sense_normal_rows(const void* x, const void* maps, const float* weights, int64_t weights_coils,
                           const void* table, int64_t jcap, void* out, const void* sub, float base_scale, float step,
                           int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                           void* workspace, size_t workspace_bytes, dlcs_stream_t stream);
/* Row-sparse adjoint x = base + step (A^H y - sub) (base / sub may be NULL: then
 * x = step A^H y [- sub]) for k-t masks: only the sampled ky lines of y are read
 * (y is zero elsewhere after the mask): per line W y -> IFFT_X (ortho scale),
 * then the zero-filled IFFT_Y, conj-map coil sum and epilogue of
 * dlcs_sense_normal_rows' third stage.  Replaces transforms.py:84-90 (SenseModel.
 * _adjoint_op) for a mask whose row table (dlcs_sense_rowtab) has been built;
 * same workspace as dlcs_sense_normal_rows. */
int dlcs_sense_adj_rows(const void* y, const void* maps, const float* weights, int64_t weights_coils,
                        const void* table, int64_t jcap, void* out, const void* base, const void* sub, float step,
                        int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                        void* workspace, size_t workspace_bytes, dlcs_stream_t stream);
/* dlcs_sense_cg with the row-sparse normal operator (same workspace size). */
int dlcs_sense_cg_rows(void* x, const void* b, const void* maps, const float* weights, int64_t weights_coils,
                       const void* table, int64_t jcap, float lamda, int num_iter,
                       int64_t B, int64_t E, int64_t C, int64_t T, int64_t Y, int64_t X,
                       void* workspace, size_t workspace_bytes, dlcs_stream_t stream);

/* Batched orthonormal 2D FFT over the last two dims of a c64 [nplanes,Y,X]
 * tensor (tr:31-46); in-place allowed.  Exposed for tests and FFT users.   */
int dlcs_fft2(const void* in, void* out, int64_t nplanes, int64_t Y, int64_t X, int inverse,
              void* workspace, size_t workspace_bytes, dlcs_stream_t stream);


/* ---------------------------------------------------------------------------
 * Swin window bookkeeping -- vst:41-67 (window_partition / window_reverse),
 * vst:229 / :243 (cyclic shift), vst:221-248 (pad / crop), vst:342-355
 * (compute_mask region labels).  Grid (D,H,W) of B images, window (wd,wh,ww)
 * already clamped by get_window_size (vst:72-85), shift (sd,sh,sw).
 *   part_src[r]  token read by windowed row r (-1: zero pad row), r < B*nW*N
 *   rev_dst[t]   windowed row that lands on token t (window_reverse + roll back)
 *   labels[r]    compute_mask region label (0..26) of windowed row r
 * Any output pointer may be NULL.  Bit-exact with the reference.
 * ------------------------------------------------------------------------- */
int dlcs_window_index(int64_t B, int64_t D, int64_t H, int64_t W, int64_t wd, int64_t wh, int64_t ww,
                      int64_t sd, int64_t sh, int64_t sw, int32_t* part_src, int32_t* rev_dst,
                      int32_t* labels, dlcs_stream_t stream);

/* dst[r, :C] = idx[r] >= 0 ? src[idx[r], :C] : 0, with dtype conversion
 * (the data movement of window_partition / window_reverse).                */
int dlcs_gather_rows(int src_dtype, int dst_dtype, const void* src, const int32_t* idx, void* dst,
                     int64_t nrows, int64_t C, int64_t ld_src, int64_t ld_dst, dlcs_stream_t stream);

/* nn.LayerNorm(C, eps=1e-5) over rows (vst:205, :211, fp32 statistics); row r
 * reads x[src_map[r]] (NULL = identity; -1 = zero pad row, vst:225).        */
int dlcs_layernorm_fwd(int out_dtype, const float* x, const int32_t* src_map, const float* gamma,
                       const float* beta, float eps, void* out, float* mean, float* rstd,
                       int64_t rows, int64_t C, dlcs_stream_t stream);
/* dx[src_map[r]] += d LN / d x (dy), or, with dx_in (the residual-stream
 * gradient, may alias dx), dx[src_map[r]] = dx_in[src_map[r]] + d LN / d x: then
 * every row of dx must be the target of exactly one r (the window partition
 * map is a bijection onto the tokens).  dgamma / dbeta accumulated (fp32).
 * workspace (>= dlcs_layernorm_bwd_workspace_bytes) holds per-workgroup column
 * partials reduced by a second launch; NULL falls back to fp32 atomics.      */
size_t dlcs_layernorm_bwd_workspace_bytes(int64_t rows, int64_t C);
int dlcs_layernorm_bwd(const float* dy, const float* x, const int32_t* src_map, const float* gamma,
                       const float* mean, const float* rstd, const float* dx_in, float* dx, float* dgamma, float* dbeta,
                       int64_t rows, int64_t C, void* workspace, size_t workspace_bytes,
                       dlcs_stream_t stream);

/* out[c] += sum_r x[r, c]  (bias gradients)                                   */
int dlcs_colsum(int dtype, const void* x, int64_t rows, int64_t C, int64_t ld, float* out, dlcs_stream_t stream);

/* Generic MFMA GEMM (nn.Linear qkv / proj / fc1 / fc2, vst:131, :133, :27-29;
 * k4s4 PatchEmbed3D / PatchUnembed3D, vst:455, :503, on the patch-blocked
 * layout; their weight gradients with split-K):
 *   C[row(m), n] (+)= alpha * act(sum_k A(m,k) B(n,k) + bias[n])
 *                     + res_scale * residual[row(m), n] + res2_scale * residual2[row(m), n]
 *   A(m,k) = a_trans ? A[k*lda+m] : A[m*lda+k];  B(n,k) = b_trans ? B[k*ldb+n] : B[n*ldb+k]
 *   act 0 none, 1 GELU(erf) (pre-activation -> aux_out if given), 2 times gelu'(aux), 3 ReLU,
 *       4 GELU(tanh) (the DiT Mlp, dit:322; pre-activation -> aux_out), 5 times gelu_tanh'(aux),
 *       6 times (aux > 0) (a ReLU backward), 7 ReLU applied AFTER the residuals
 *   row(m) = row_map ? row_map[m] : m  (-1 drops the row; the window_reverse scatter)
 *   splitk > 1 allows split-K: requires c_dtype = DLCS_F32 and accumulate = 1 and no
 *   bias / act / residual (fp32 atomics; the library picks the split factor).  */
int dlcs_gemm(int dtype, int64_t M, int64_t N, int64_t K,
              const void* A, int64_t lda, int a_trans,
              const void* B, int64_t ldb, int b_trans,
              void* C, int64_t ldc, int c_dtype,
              const float* bias, int act, const void* aux, void* aux_out, int64_t ldaux, float alpha,
              const void* residual, int64_t ldr, int r_dtype, float res_scale,
              const void* residual2, int64_t ldr2, int r2_dtype, float res2_scale,
              const int32_t* row_map, int accumulate, int splitk, dlcs_stream_t stream);

/* Grouped weight gradients (bf16 operands, fp32 results) of one backward phase
 * (the 4 nn.Linear weights of a Swin block, vst:27-29, :131, :133, or the k4s4
 * patch embed / unembed, vst:455, :503):
 *   dW_g[m, n] += sum_t A_g[t*lda_g + m] * B_g[t*ldb_g + n]     dW_g row-major [M_g, N_g]
 *   db_g[c]    += sum_t sum_{m = c mod period_g} A_g[t*lda_g + m] (optional, period 0 = M_g)
 * 1 <= ngroups <= 4; M_g, N_g multiples of 160; T a multiple of 64.  The token
 * sum is split into ranges whose fp32 partials go to the workspace
 * (dlcs_gemm_dw_workspace_bytes) and are summed by a second kernel: no atomics. */
size_t dlcs_gemm_dw_workspace_bytes(int ngroups, const int64_t* M, const int64_t* N, int64_t T);
int dlcs_gemm_dw_grouped(int ngroups, const void* const* A, const int64_t* lda, const void* const* B,
                         const int64_t* ldb, const int64_t* M, const int64_t* N, float* const* dW,
                         float* const* db, const int64_t* db_period, int64_t T, void* workspace,
                         size_t workspace_bytes, dlcs_stream_t stream);
/* The same with fp32 operands (the fp32 headline path): identical arguments,
 * tiles, splits and workspace size; runs on the fp16 2-plane split with one
 * power-of-two scale per column and 32-token step (csrc/gemm_dw_h3.inc). */
int dlcs_gemm_dw_grouped_f32(int ngroups, const void* const* A, const int64_t* lda, const void* const* B,
                             const int64_t* ldb, const int64_t* M, const int64_t* N, float* const* dW,
                             float* const* db, const int64_t* db_period, int64_t T, void* workspace,
                             size_t workspace_bytes, dlcs_stream_t stream);

/* Fused window attention core, vst:139-170 between qkv and proj, per (window, head):
 *   S = (scale q) k^T + table[rpi(i,j), head] + mask;  O = softmax(S) v
 * qkv [nwin*N, 3*heads*hd] (T, window-ordered rows), out [nwin*N, heads*hd] (T),
 * lse [nwin, heads, N] fp32 (saved for backward).  rpi uses the constructed
 * window (wd0,wh0,ww0) numbering sliced [:N,:N] (vst:152).  mask: either region
 * labels [nwin*N] (-100 where labels differ, vst:354) or an explicit additive
 * mask [mask_nw, N, N] (the reference API form), or neither.                 */
int dlcs_window_attn_fwd(int dtype, const void* qkv, void* out, float* lse, const float* table,
                         const int32_t* labels, const float* mask, int64_t mask_nw, int64_t nwin,
                         int64_t N, int64_t heads, int64_t head_dim,
                         int64_t wd0, int64_t wh0, int64_t ww0, float scale, dlcs_stream_t stream);
/* Backward: dqkv [nwin*N, 3*heads*hd] fp32, every element written (no zeroing
 * needed), dtable [nrel, heads] accumulated.                                   */
int dlcs_window_attn_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse,
                         const float* table, const int32_t* labels, const float* mask, int64_t mask_nw,
                         float* dqkv, float* dtable,
                         int64_t nwin, int64_t N, int64_t heads, int64_t head_dim,
                         int64_t wd0, int64_t wh0, int64_t ww0, float scale, dlcs_stream_t stream);

/* ---------------------------------------------------------------------------
 * Conv3d(k=3, stride 1, pad 1) -- s3d:120-134 inside ConvBlock s3d:225-270.
 * Activations in the patch-blocked channels-last layout (D, H, W multiples of 4):
 *   row(b,t,y,x) = ((((b*D/4 + t/4)*H/4 + y/4)*W/4 + x/4)*64 + (t%4)*16 + (y%4)*4 + x%4
 * in [rows, cin_ld] (channels >= cin ignored), weights packed by
 * dlcs_conv3d_pack_weights: [27][cout_pad][cin_pad], cin_pad % 32 == 0.
 *   out[row, co] (+)= epi(conv(relu_in ? relu(in) : in) + bias)
 *   epi: times (mask[row, co] > 0) if mask (ReLU backward); + res_scale * residual;
 *        then ReLU if relu_out (the consumer ConvBlock's pre-activation, s3d:256-259)
 * dgrad = the same call on weights packed with mode 1 (transposed, tap-flipped). */
int dlcs_conv3d_k3(int dtype, const void* in, int64_t cin, int64_t cin_ld, const void* wpacked,
                   int64_t cin_pad, const float* bias, void* out, int out_dtype, int64_t cout,
                   int64_t cout_pad, int64_t cout_ld, int64_t B, int64_t D, int64_t H, int64_t W,
                   int relu_in, const void* mask, int64_t mask_ld, const void* residual, int res_dtype,
                   int64_t res_ld, float res_scale, int accumulate, int relu_out, dlcs_stream_t stream);
/* dw_packed[tap][co][ci] += sum_v gout[v, co] * act(in)[v + off(tap), ci];
 * dbias (optional): dbias[co] += sum_v gout[v, co], the conv's bias gradient
 * (s3d:120-134) -- in the bf16 SFE weight gradient (thin input side) from the g
 * tiles it already holds (an all-ones MFMA operand, per-range partials summed in
 * a fixed order), otherwise by a column-sum launch after the weight gradient. */
int dlcs_conv3d_k3_wgrad(int dtype, const void* in, int64_t cin, int64_t cin_ld, int64_t cin_pad, int relu_in,
                         const void* gout, int64_t cout, int64_t g_ld, int64_t cout_pad, float* dw_packed,
                         float* dbias, int64_t B, int64_t D, int64_t H, int64_t W, int64_t vox_per_block,
                         dlcs_stream_t stream);
/* torch Conv3d weight w [cout][cin][3][3][3] fp32 -> packed (mode 0: [27][rows_pad=cout_pad][cols_pad=cin_pad];
 * mode 1 (dgrad): [27][rows_pad=cin_pad][cols_pad=cout_pad], taps flipped);
 * modes 2 / 3 (DIAG build; the product library returns DLCS_ERR_UNSUPPORTED_SIZE):
 * the forward / dgrad packing split into three bf16 planes for the x6 conv below
 * (cout = cin = 160): WA [27][160][320] (per 16-channel chunk of the contracted
 * index: high | mid plane), then WB [27][160][160] (low plane); dtype, rows_pad
 * and cols_pad are ignored.                                                  */
int dlcs_conv3d_pack_weights(int dtype, const float* w, void* packed, int64_t cout, int64_t cin,
                             int64_t rows_pad, int64_t cols_pad, int mode, dlcs_stream_t stream);
#ifdef DLCS_DIAG_BUILD
/* DIAG build only (libdlcs_hip_diag.so, `make DIAG=1`): the superseded bf16
 * 3-plane conv, kept for A/B measurement; the product library's fp32 160 -> 160
 * conv is dlcs_conv3d_k3_f16x3 below.                                         */
/* fp32 Conv3d 160 -> 160 (s3d:120-134) on bf16 matrix cores at fp32 accuracy:
 * every operand split x = xh + xm + xl into bf16 planes (24 significant bits),
 * the six plane products >= 2^-16 accumulated in fp32.  Same layout and
 * epilogue as dlcs_conv3d_k3 (fp32 out / mask / residual), input given as the
 * planes of dlcs_split3_bf16, weights as dlcs_conv3d_pack_weights modes 2 / 3. */
int dlcs_conv3d_k3_x6(const void* xa, const void* xb, const void* wpacked, const float* bias, float* out,
                      int64_t cout_ld, int64_t B, int64_t D, int64_t H, int64_t W, const float* mask, int64_t mask_ld,
                      const float* residual, int64_t res_ld, float res_scale, int accumulate, int relu_out,
                      dlcs_stream_t stream);
/* dw_packed [27][160][160] += the fp32 weight gradient of the 160 -> 160 conv
 * (dlcs_conv3d_k3_wgrad's sum) from the bf16 planes of x and of gout, six plane
 * products (fp32 atomics: zero dw_packed first or accumulate).               */
int dlcs_conv3d_k3_wgrad_x6(const void* xa, const void* xb, const void* ga, const void* gb, float* dw_packed,
                            int64_t B, int64_t D, int64_t H, int64_t W, dlcs_stream_t stream);
/* x [rows][ld] fp32 (160 channels) -> xa [rows][320] bf16 (high | mid plane per
 * 16-channel chunk), xb [rows][160] bf16 (low plane); x = xh + xm + xl exactly
 * up to the low plane's rounding.                                            */
int dlcs_split3_bf16(const float* x, int64_t rows, int64_t ld, void* xa, void* xb, dlcs_stream_t stream);
/* Cycle-counter stamps of the conv kernels' DIAG instrumentation copied to the
 * host buffer `host` (n words): tools/conv_stamps.py, tools/conv_stamps_h3.py. */
int dlcs_debug_conv_stamps(void* host, int64_t n);
int dlcs_debug_h3_stamps(void* host, int64_t n);
#endif  /* DLCS_DIAG_BUILD */

/* fp32 Conv3d 160 -> 160 on fp16 matrix cores (2-plane split, three plane
 * products, one power-of-two scale per tensor; conv3d_f16x3.inc): same contract
 * and epilogues as dlcs_conv3d_k3.
 *   dlcs_split2_f16: x fp32 [rows][ld] -> planes [rows][320] f16 (per 32-channel
 *     chunk: high plane then low plane) + a 256-B trailer holding max|x|;
 *     planes must be dlcs_split2_f16_bytes(rows) bytes; have_max = 1: the
 *     trailer already holds max|x| (written by the producing kernel's out_max,
 *     zeroed before it ran) and the max-abs pass is skipped.
 *     colsum (optional, fp32 [160]): += the column sums of x (a conv bias
 *     gradient, fused so the tensor is read once).
 *   out_max (conv / GEMM below, optional): atomicMax of |output| as float bits
 *     into a caller-zeroed word -- the next split's trailer.
 *   dlcs_conv3d_pack_weights_f16x3: w [160][160][3][3][3] fp32 -> packed
 *     (dlcs_conv3d_pack_weights_f16x3_bytes() bytes); mode 0 forward, 1 dgrad. */
size_t dlcs_split2_f16_bytes(int64_t rows);
int dlcs_split2_f16(const float* x, int64_t rows, int64_t ld, void* planes, int have_max, float* colsum,
                    dlcs_stream_t stream);
size_t dlcs_conv3d_pack_weights_f16x3_bytes(void);
int dlcs_conv3d_pack_weights_f16x3(const float* w, int mode, void* packed, dlcs_stream_t stream);
int dlcs_conv3d_k3_f16x3(const void* xplanes, const void* wpacked, const float* bias, float* out, int64_t cout_ld,
                         int64_t B, int64_t D, int64_t H, int64_t W, const float* mask, int64_t mask_ld,
                         const float* residual, int64_t res_ld, float res_scale, int accumulate, int relu_out,
                         unsigned* out_max, void* out_planes, float* colsum, const void* mask_planes,
                         dlcs_stream_t stream);
/* C[m, n] (+)= alpha * act(sum_k A[m,k] B[n,k] + bias[n]) + res_scale res[m,n] + res2_scale res2[m,n]
 * for K = 160, A [M][160] and B [N][160] given as dlcs_split2_f16 plane pairs;
 * act 0 or 3 (ReLU); N a multiple of 160; C fp32 (the fp32 build's k4s4 patch
 * unembed forward and patch-embed input gradient, vst:455, :503). */
int dlcs_gemm_k160_f16x3(const void* aplanes, int64_t M, const void* bplanes, int64_t N, float* C, int64_t ldc,
                         const float* bias, int act, float alpha, const float* residual, int64_t ldr, float res_scale,
                         const float* residual2, int64_t ldr2, float res2_scale, int accumulate, unsigned* out_max,
                         void* out_planes, float* colsum, const void* res_planes, const void* res2_planes,
                         dlcs_stream_t stream);
/* Producer-side split (no dlcs_split2_f16 pass over the fp32 output):
 *   out_planes (conv above, residual or mask form only, cout_ld = 160; the K = 160
 *     GEMM with ldc = N, viewed as [M N / 160][160]): the epilogue also writes the
 *     output's split2 planes, with the scale of the word already in their trailer --
 *     an upper bound of max|out| (dlcs_planes_bound), since the true max is not
 *     known until the launch ends.  out_max still receives the true max.  Both
 *     take out / C = null with out_planes (planes-only output, no accumulate) and
 *     colsum (fp32 [160], the conv: fused forms only): += the column sums of the
 *     output (the GEMM: of its [M N / 160][160] view) -- a conv bias gradient,
 *     from per-tile partials summed in a fixed order.  mask_planes (the conv's
 *     masked form, in place of mask): the ReLU mask as the planes of a non-negative
 *     tensor written by a producer (hi | lo != 0 <=> x > 0: a producer keeps a
 *     nonzero value's sign in the smallest subnormal).  The GEMM's res_planes /
 *     res2_planes: the residuals as split2 images of the [M N / 160][160] view
 *     ((hi + lo) / s, 2^-22 relative) in place of residual / residual2.
 *   dlcs_planes_bound: trailer of planes [rows] <- B (1 + 2^-10), B = c0 m0 n0 +
 *     c1 m1 n1 + cvec max|vec[0 .. nvec)|; m / n float-bit words (null n = 1, null
 *     m drops the term): input maxima and weight norms, so B >= max|W x + b + c r|.
 *     Also writes the zero row after the trailer.
 *   dlcs_abs_row_sum_max: *out = max over rows r of sum_{o < n_outer, i < inner}
 *     |w[r row_stride + o outer_stride + i]| (float bits): ||W||_inf of a weight
 *     layout (conv forward: rows co, inner ci x 27; the K = 160 GEMM: rows n). */
int dlcs_planes_bound(void* planes, int64_t rows, const unsigned* m0, const unsigned* n0, float c0,
                      const unsigned* m1, const unsigned* n1, float c1, const float* vec, int64_t nvec, float cvec,
                      dlcs_stream_t stream);
int dlcs_abs_row_sum_max(const float* w, int64_t rows, int64_t row_stride, int64_t n_outer, int64_t outer_stride,
                         int64_t inner, unsigned* out, dlcs_stream_t stream);

/* nn.Linear with in_features = 160 on the f16x3 split (the Swin block's qkv,
 * proj and fc1 forward, and the fc2 / proj input gradients; vst:146, :168,
 * vst:20-38 Mlp): C[row(m), n] (+)= alpha act(x[m] . w[n] + bias[n]) + res[row(m), n]
 * with x and w as dlcs_split2_f16 plane pairs of [M, 160] / [N, 160] (N % 160 == 0).
 * act: 0 none, 1 GELU (erf; the pre-activation is stored to aux_out [M, ldaux]
 * when given), 2 times GELU'(aux [M, ldaux]) (the GELU backward), 3 ReLU.
 * row_map (optional, int32 [M]): output / residual row of m, < 0 = skip (the
 * window_reverse scatter of the proj).  Replaces the fp32 nn.Linear calls of
 * vst:146 / :168 / vst:27-37 on the fp32 path. */
int dlcs_linear_k160_f16x3(const void* xplanes, int64_t M, const void* wplanes, int64_t N, float* C, int64_t ldc,
                           const float* bias, int act, const float* aux, float* aux_out, int64_t ldaux, float alpha,
                           const float* residual, int64_t ldr, const int32_t* row_map, int accumulate,
                           dlcs_stream_t stream);

/* Row-scaled fp16 two-plane split ("h3r") for the fp32 token Linears.
 * dlcs_h3r_pack_multi packs n weight operands (two launches: K-split row maxima,
 * then the split): job i reads B[r][k] = trans[i] ? src[i][k * ld[i] + r] :
 * src[i][r * ld[i] + k] (r < rows[i], k < K[i], K % 32 == 0) into dst[i]
 * (dlcs_h3r_pack_bytes(rows, K) bytes, 16-B aligned): fp16 planes
 * [rows][K / 32][xh 32 | xl 32] with one power-of-two scale per row, then 1 / scale
 * per row (fp32), then the row-max partials (scratch).  dlcs_gemm_h3r:
 *   C[row(m), n] (+)= alpha act(sum_k A[m, k] B[n, k] + bias[n]) + res[row(m), n]
 * with A fp32 [M, K] (row stride lda) split inside the kernel with one scale per
 * row (per row and 192-wide K segment when K is not one of the Swin sizes), B a
 * packed operand: N % 160 == 0 with K % 160 == 0, or N % 64 == 0 with K % 64 == 0
 * (K <= 16384); act 0 none, 1 GELU-erf / 4 GELU-tanh (pre-activation
 * to aux_out [M, ldaux]), 2 / 5 times GELU-erf' / GELU-tanh' of aux; row_map[m] < 0
 * skips a row.  Replaces the fp32 nn.Linear forward / input gradient GEMMs of
 * vst:146, :168, :27-37 (qkv, proj, fc1, fc2) and of the DiT / Latte blocks'
 * timm Attention / Mlp Linears (dit:317-350). */
size_t dlcs_h3r_pack_bytes(int64_t rows, int64_t K);
int dlcs_h3r_pack_multi(int n, const float* const* src, const int64_t* ld, const int* trans, const int64_t* rows,
                        const int64_t* K, void* const* dst, dlcs_stream_t stream);
int dlcs_gemm_h3r(const float* A, int64_t M, int64_t K, int64_t lda, const void* bpacked, int64_t N, float* C,
                  int64_t ldc, const float* bias, int act, const float* aux, float* aux_out, int64_t ldaux, float alpha,
                  const float* residual, int64_t ldr, const int32_t* row_map, int accumulate, dlcs_stream_t stream);

/* fp8 (OCP e4m3) path of the diffusion denoisers' token Linears (BASELINE config 5,
 * inference).  dlcs_f8r_quant: x fp32 [rows, K] (row stride ld, K % 4 == 0) ->
 * q e4m3 [rows][K] with one power-of-two scale per row (max |s x| <= 256), inv[r] =
 * 1 / s.  dlcs_gemm_f8r: C[row(m), n] = alpha act(sum_k A[m, k] B[n, k] ainv[m]
 * binv[n] + bias[n]) + res[row(m), n] on v_mfma_f32_16x16x32_fp8_fp8 (K % 64 == 0,
 * N % 64 == 0); act 0 none, 1 GELU-erf, 4 GELU-tanh (pre-activation to aux_out
 * [M, ldaux]); row_map[m] < 0 skips a row.  Replaces the fp32 nn.Linear calls of the
 * DiT / Latte blocks (dit:317-323, lat:301-309) when the fp8 path is selected. */
int dlcs_f8r_quant(const float* x, int64_t rows, int64_t K, int64_t ld, void* q, float* inv, dlcs_stream_t stream);
int dlcs_gemm_f8r(const void* aq, const float* ainv, int64_t M, int64_t K, const void* bq, const float* binv,
                  int64_t N, float* C, int64_t ldc, const float* bias, int act, float* aux_out, int64_t ldaux,
                  float alpha, const float* residual, int64_t ldr, const int32_t* row_map, dlcs_stream_t stream);

/* C[m, n] += sum_k A[m, k] B[n, k], fp32, A [M, K] / B [N, K] K-contiguous, C [M, N]
 * contiguous (N % 160 == 0): split over K into <= 4 ranges whose raw partials go
 * to `workspace` (dlcs_gemm_f32_splitk_det_workspace_bytes) and are summed in a
 * fixed order -- split-K occupancy, run-to-run deterministic.  The k4s4 patch
 * embed forward (vst:472, 13440 tokens x 10240 -> 160). */
size_t dlcs_gemm_f32_splitk_det_workspace_bytes(int64_t M, int64_t N);
int dlcs_gemm_f32_splitk_det(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int64_t N,
                             int64_t K, float* C, void* workspace, size_t workspace_bytes, dlcs_stream_t stream);
#ifdef DLCS_DIAG_BUILD
/* DIAG build only: the same product (C += A B^T, fp32 in and out) on bf16 matrix
 * cores with the 3-plane split (x = h + m + l, six plane products): B's planes and
 * <= 4 raw K-range partial slabs in `workspace` (dlcs_gemm_nt_x6_workspace_bytes),
 * summed in a fixed order.  N % 160 == 0, K % 32 == 0, lda / ldb % 4 == 0, 16-B
 * aligned pointers, any M.  Superseded by dlcs_gemm_h3r's split-K path (the
 * product's fp32 patch-embed forward, vst:472). */
size_t dlcs_gemm_nt_x6_workspace_bytes(int64_t M, int64_t N, int64_t K);
int dlcs_gemm_nt_x6(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                    float* C, void* workspace, size_t workspace_bytes, dlcs_stream_t stream);
#endif  /* DLCS_DIAG_BUILD */
/* dw_packed [27][160][160] (+)= fp32 weight gradient from the f16 plane pairs of x and g. */
int dlcs_conv3d_k3_wgrad_f16x3(const void* xplanes, const void* gplanes, float* dw_packed, int64_t B, int64_t D,
                               int64_t H, int64_t W, dlcs_stream_t stream);
/* fp32 thin-end Conv3d k3 (the ConvBlocks' 2E <-> 160 ends: SFE s3d:384, final
 * layer s3d:391; replaces their fp32 nn.Conv3d calls, swin3D.py:225-273) on fp16
 * matrix cores (conv3d_thin_f16x3.inc): the fp32 activation is read once and
 * split in registers with a power-of-two scale from its max |x| word.
 *   dlcs_absmax_f32: *out = max(*out, max|x|) as float bits (x 16-B aligned).
 *   dlcs_conv3d_thin_pack_f16x3: wpacked = dlcs_conv3d_pack_weights output fp32
 *     [27][cout_pad][cin_pad] (mode 0 forward or 1 dgrad) -> the kernels' 2-plane
 *     image (dlcs_conv3d_thin_pack_f16x3_bytes(kind) bytes); kind 0 thin input
 *     (cout = cout_pad = 160, cin <= 4), kind 1 thin output (cin = cin_pad = 160, cout <= 4).
 *   dlcs_conv3d_thin_f16x3: out = conv(in) + epilogue as dlcs_conv3d_k3 (thin
 *     input: bias / mask / residual / accumulate / relu_out / out_max; thin output:
 *     bias / accumulate / relu_out, 4 floats written per row, cout_ld >= 4).
 *     in_max: the max |in| word (dlcs_absmax_f32 or a producer's out_max).
 *     Thin input with a mask only: out_planes / colsum as for dlcs_conv3d_k3_f16x3
 *     (out may be null: planes-only output).
 *   dlcs_conv3d_thin_wgrad_f16x3: dw_packed [27][cout_pad][cin_pad] += the fp32
 *     weight gradient (dlcs_conv3d_k3_wgrad's sum) for (cin <= 4, cout = 160) or
 *     (cin = 160, cout <= 4); colsum (optional, first shape only, fp32 [160]):
 *     += sum over voxels of g (the conv bias gradient).  fp32 atomics.        */
int dlcs_absmax_f32(const float* x, int64_t n, unsigned* out, dlcs_stream_t stream);
size_t dlcs_conv3d_thin_pack_f16x3_bytes(int kind);
int dlcs_conv3d_thin_pack_f16x3(const float* wpacked, int64_t cout, int64_t cout_pad, int64_t cin, int64_t cin_pad,
                                int kind, void* out, dlcs_stream_t stream);
int dlcs_conv3d_thin_f16x3(const float* in, int64_t cin, int64_t cin_ld, const unsigned* in_max, const void* wthin,
                           const float* bias, float* out, int64_t cout, int64_t cout_ld, int64_t B, int64_t D,
                           int64_t H, int64_t W, const float* mask, int64_t mask_ld, const float* residual,
                           int64_t res_ld, float res_scale, int accumulate, int relu_out, unsigned* out_max,
                           void* out_planes, float* colsum, const void* mask_planes, dlcs_stream_t stream);
int dlcs_conv3d_thin_wgrad_f16x3(const float* in, int64_t cin, int64_t cin_ld, const unsigned* in_max,
                                 const float* g, int64_t cout, int64_t g_ld, const unsigned* g_max, float* dw_packed,
                                 int64_t cout_pad, int64_t cin_pad, float* colsum, int64_t B, int64_t D, int64_t H,
                                 int64_t W, dlcs_stream_t stream);
/* The same two thin-end products with the 160-channel operand as dlcs_split2_f16
 * planes (one split shared by the forward / input gradient and the weight
 * gradient that read it; conv3d_thin_planes.inc): DMA'd, no in-kernel split,
 * run-to-run deterministic (no float atomics).
 *   dlcs_conv3d_thin_out_planes_f16x3: out [rows][cout_ld] (cout <= 4) = conv(x) +
 *     bias, optional relu_out / accumulate; wthin = dlcs_conv3d_thin_pack_f16x3 kind 1.
 *   dlcs_conv3d_thin_wgrad_planes_f16x3: dw_packed [27][cout_pad][cin_pad] += the
 *     weight gradient between the 160-channel planes and the fp32 thin tensor
 *     ([rows][thin_ld], thin_ch <= 4 used, max word thin_max): big_is_co = 1 for
 *     the SFE conv (planes = g, 160 output channels, thin = its input), 0 for the
 *     final conv (planes = its input, thin = g, 160 input channels).         */
int dlcs_conv3d_thin_out_planes_f16x3(const void* xplanes, const void* wthin, const float* bias, float* out,
                                      int64_t cout, int64_t cout_ld, int64_t B, int64_t D, int64_t H, int64_t W,
                                      int accumulate, int relu_out, dlcs_stream_t stream);
int dlcs_conv3d_thin_wgrad_planes_f16x3(const void* bigplanes, const float* thin, int64_t thin_ch, int64_t thin_ld,
                                        const unsigned* thin_max, int big_is_co, float* dw_packed, int64_t cout_pad,
                                        int64_t cin_pad, int64_t B, int64_t D, int64_t H, int64_t W,
                                        dlcs_stream_t stream);
/* grad [cout][cin][3][3][3] (+)= unpack(dw_packed)                           */
int dlcs_conv3d_unpack_wgrad(const float* dw_packed, float* grad, int64_t cout, int64_t cin, int64_t cout_pad,
                             int64_t cin_pad, int accumulate, dlcs_stream_t stream);

/* ---------------------------------------------------------------------------
 * SwinTransformer3DNet boundary -- s3d:394-418: complex [B,E,T,Y,X] <-> real
 * [2E channels (re | im), circular time pad `pad`] in the patch-blocked layout
 * with row stride ldc (channels >= 2E written as zero).                      */
int dlcs_swin_pre(int dtype, const void* x, void* u, int64_t B, int64_t E, int64_t T, int64_t Y, int64_t X,
                  int64_t pad, int64_t ldc, dlcs_stream_t stream);
int dlcs_swin_pre_bwd(int dtype, const void* gu, void* gx, int64_t B, int64_t E, int64_t T, int64_t Y, int64_t X,
                      int64_t pad, int64_t ldc, dlcs_stream_t stream);
int dlcs_swin_post(int dtype, const void* o, void* out, int64_t B, int64_t E, int64_t T, int64_t Y, int64_t X,
                   int64_t pad, int64_t ldc, dlcs_stream_t stream);
int dlcs_swin_post_bwd(int dtype, const void* gout, void* go, int64_t B, int64_t E, int64_t T, int64_t Y, int64_t X,
                       int64_t pad, int64_t ldc, dlcs_stream_t stream);

/* Elementwise / layout helpers.
 *   axpby:   y = a x + b y  (dtype conversion allowed)
 *   permute: dst (shape dst_shape, contiguous) [i] (+)= src[sum_k i_k * src_strides[k]], ndim <= 6
 *   fill_bias: out[r, c] = bias[c % period] (or 0)
 *   relu_grad: g[i] = (a[i] > 0) ? g[i] : 0, in place (a = stored post-ReLU activation) */
int dlcs_relu_grad(int g_dtype, void* g, int a_dtype, const void* a, int64_t n, dlcs_stream_t stream);
int dlcs_axpby(int x_dtype, int y_dtype, const void* x, void* y, int64_t n, float a, float b, dlcs_stream_t stream);
int dlcs_permute(int src_dtype, int dst_dtype, const void* src, void* dst, int64_t ndim,
                 const int64_t* dst_shape, const int64_t* src_strides, int accumulate, dlcs_stream_t stream);
int dlcs_fill_bias(float* out, const float* bias, int64_t rows, int64_t C, int64_t period, dlcs_stream_t stream);
/* NCDHW [B, C, D, H, W] <-> patch-blocked rows [B * nT * nY * nX * 64, ld] (nT = ceil(D/4), ...)
 * for the standalone module API (s3d ConvBlock, vst PatchEmbed3D / PatchUnembed3D): inverse = 0
 * blocks (grid zero-padded to multiples of 4, channels >= C zero), inverse = 1 unblocks (crops). */
int dlcs_block_layout(int src_dtype, int dst_dtype, const void* src, void* dst, int64_t B, int64_t C, int64_t D,
                      int64_t H, int64_t W, int64_t ld, int inverse, dlcs_stream_t stream);

/* Batched fp32 -> bf16 cast of `count` <= DLCS_CAST_MULTI_MAX tensors in ONE launch
 * (the per-step compute-dtype copies of a network's weights): dst[i][k] = bf16(src[i][k]),
 * k < n[i].  src / dst / n are HOST arrays of device pointers and sizes, read
 * before the call returns.  Replaces one dlcs_axpby launch per weight.        */
#define DLCS_CAST_MULTI_MAX 64
int dlcs_cast_multi_bf16(int64_t count, const float* const* src, void* const* dst, const int64_t* n,
                         dlcs_stream_t stream);

/* ---- Cine preprocessing (prep.hip) ----------------------
 * The per-voxel steps of CinePreprocess.__call__ / _augment (dl_cs/data/preprocess.py:54-180)
 * and of reconstruct.py's DataTransform (scripts/reconstruct.py:114-152); complex64 data.
 *
 * dlcs_kt_window_average replaces time_average / sliding_window (dl_cs/mri/utils.py:29-49,
 * get_mask :69-79) over the T axis of k [P, T, YX]:
 *   full = 1: out [P, 1, YX] = sum_t k / (#{t : |k| > 1e-12} + 1e-6)
 *   full = 0: out [P, T, YX], frame t averages frames (t - window/2 + j) mod T, j < window
 * dlcs_kth_largest_abs: out[0] = k-th largest |x| of n values (torch.topk(|x|, k).values.min(),
 *   preprocess.py:149-153), one workgroup radix select; out is a device float.
 * dlcs_cplx_mask_scale: y[p, r] = x[p, r] * mask[(p % mask_planes), r] (mask optional, float,
 *   mask_planes <= 1 broadcasts plane 0) divided (divide = 1) or multiplied by scale[0], a
 *   DEVICE scalar (preprocess.py:146, :156-157; reconstruct.py:233 rescale); y may alias x.
 * dlcs_crop_flip: out [P, T, ny, nx] = in [P, T, Y, X] cropped at (y0, x0) and flipped along
 *   t / y / x after the crop (preprocess.py:59-120). */
int dlcs_kt_window_average(const void* k, void* out, int64_t P, int64_t T, int64_t YX, int64_t window,
                           int full, dlcs_stream_t stream);
int dlcs_kth_largest_abs(const void* x, int64_t n, int64_t k, float* out, dlcs_stream_t stream);
int dlcs_cplx_mask_scale(const void* x, const float* mask, void* y, int64_t P, int64_t TYX, int64_t mask_planes,
                         const float* scale, int divide, dlcs_stream_t stream);
int dlcs_crop_flip(const void* in, void* out, int64_t P, int64_t T, int64_t Y, int64_t X, int64_t y0, int64_t ny,
                   int64_t x0, int64_t nx, int flip_t, int flip_y, int flip_x, dlcs_stream_t stream);

/* ---- DiT denoiser (BASELINE config 5; dit.hip) -----------------
 * dit = dl_cs/models/DiT.py, udit = dl_cs/models/unrolledDiT.py, timm =
 * timm.models.vision_transformer (not vendored by the reference).
 *
 * dlcs_mhsa_fwd / _bwd: the core of timm's Attention as DiTBlockFactor uses it
 * (dit:336-345) -- per sequence s and head h of qkv [nseq*N, 3*heads*hd] (fp32,
 * columns [3][heads][hd] as timm's reshape(B, N, 3, heads, hd)):
 *   O = softmax(scale q k^T) v -> out [nseq*N, heads*hd] (transpose(1,2).reshape),
 *   lse [nseq, heads, N] (natural log-sum-exp, saved for the backward);
 * bwd writes every element of dqkv [nseq*N, 3*heads*hd] (fp32) from qkv, out, dout
 * and lse (P recomputed); workspace dlcs_mhsa_bwd_workspace_bytes().  hd <= 32, % 4. */
int dlcs_mhsa_fwd(int dtype, const void* qkv, void* out, float* lse, int64_t nseq, int64_t N, int64_t heads,
                  int64_t head_dim, float scale, dlcs_stream_t stream);
size_t dlcs_mhsa_bwd_workspace_bytes(int64_t nseq, int64_t N, int64_t heads);
int dlcs_mhsa_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse, float* dqkv,
                  int64_t nseq, int64_t N, int64_t heads, int64_t head_dim, float scale, void* workspace,
                  size_t workspace_bytes, dlcs_stream_t stream);

/* k3 convolutions with a thin (<= 8 channel) side as GEMMs on the patch-blocked layout
 * (DiTResNet SFE 4 -> F and final F -> 4, dit:1297, :1302; fwd, dgrad and wgrad):
 *   im2col: dst[v][tap*C + c] = src[v + sign*off(tap)][c] (0 outside the grid), columns
 *           [27 C, ld_dst) zeroed;  off(tap) = (kd-1, kh-1, kw-1), tap = 9 kd + 3 kh + kw
 *   col2im: out[v][c] (+)= bias[c] + sum_tap P[v + sign*off(tap)][tap*C + c] for c < C
 *           (columns [C, ld_out) zeroed unless accumulate).                          */
int dlcs_conv3d_thin_im2col(const float* src, int64_t ld_src, int64_t C, float* dst, int64_t ld_dst, int sign,
                            int64_t B, int64_t D, int64_t H, int64_t W, dlcs_stream_t stream);
int dlcs_conv3d_thin_col2im(const float* P, int64_t ld_p, int64_t C, float* out, int64_t ld_out, const float* bias,
                            int sign, int accumulate, int64_t B, int64_t D, int64_t H, int64_t W,
                            dlcs_stream_t stream);

/* adaLN conditioning vectors (dit:184-221, :324-331, :399-406), fp32:
 *   dlcs_dit_vec op 0: y = SiLU(a); 1: y = a * SiLU'(b); 2: y = 1 + a (modulate's
 *     1 + scale, dit:22-23); 3: y = a + b.   (y may alias a or b)
 *   dlcs_timestep_embedding: out [B, dim] = [cos(t f_k), sin(t f_k)],
 *     f_k = exp(-ln(max_period) k / (dim/2)) (dit:198-216); t fp32 [B].
 *   dlcs_scale_rows: Wo[n,:] = gate[n] W[n,:], bo[n] = gate[n] b[n] -- a gated
 *     residual branch g * (x W^T + b) (dit:338, :345, :348) as one Linear.
 *   dlcs_gated_linear_grad: its parameter gradients from G = dy^T x and colsum(dy):
 *     dW[n,:] += g[n] G[n,:], db[n] += g[n] cs[n], dgate[n] += W[n,:].G[n,:] + b[n] cs[n].
 *   dlcs_rows_add: dst[idx[r], :] += src[r, :] (atomic; idx NULL = identity) -- the
 *     embedding_table gradient (dit:250).                                         */
int dlcs_dit_vec(int op, const float* a, const float* b, float* y, int64_t n, dlcs_stream_t stream);
int dlcs_timestep_embedding(const float* t, int64_t B, int64_t dim, float max_period, float* out,
                            dlcs_stream_t stream);
int dlcs_scale_rows(const float* W, const float* b, const float* gate, float* Wo, float* bo, int64_t N, int64_t K,
                    dlcs_stream_t stream);
int dlcs_gated_linear_grad(const float* W, const float* b, const float* G, const float* colsum, const float* gate,
                           float* dW, float* db, float* dgate, int64_t N, int64_t K, dlcs_stream_t stream);
int dlcs_rows_add(float* dst, const int32_t* idx, const float* src, int64_t nrows, int64_t C, dlcs_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DLCS_H */

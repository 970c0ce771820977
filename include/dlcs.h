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

/* Batched orthonormal 2D FFT over the last two dims of a c64 [nplanes,Y,X]
 * tensor (tr:31-46); in-place allowed.  Exposed for tests and FFT users.   */
int dlcs_fft2(const void* in, void* out, int64_t nplanes, int64_t Y, int64_t X, int inverse,
              void* workspace, size_t workspace_bytes, dlcs_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DLCS_H */

/*
 * anr.h — C ABI of libanr_hip.so, the MI355X (gfx950) kernels behind the AtmoNR
 * volumetric-renderer hot path.
 *
 * The reference (nasa/atmospheric-neural-rendering) has no C ABI: its hot path is
 * Python glue (samplers.py, datasets/harp2.py, graphics_utils.py, losses.py) around
 * tiny-cuda-nn's CUDA modules (tinycudann.Encoding / tinycudann.Network, bound through
 * pybind11 at pipelines/instant_ngp.py:4,60-85,163-174,236-237). Each entry point below
 * replaces one of those call sites; the reference line it stands in for is cited on it.
 * The Python host (atmonr_amd/_lib.py) binds these through ctypes; INTEGRATION.md shows
 * the binding.
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer owned by the caller (torch's caching allocator);
 *     the library allocates no device memory of its own;
 *   - work is enqueued on `stream` (a hipStream_t, e.g. torch.cuda.current_stream()
 *     .cuda_stream); nothing synchronises the host;
 *   - return 0 on success, a negative ANR_E* code on error; anr_last_error() returns a
 *     thread-local message for the last failure. Errors never throw across the ABI;
 *   - sizes are int64; row strides are in ELEMENTS of the tensor's dtype;
 *   - dtype codes: ANR_F32 = 0, ANR_F16 = 1, ANR_BF16 = 2 (bf16: field MFMA operands only).
 */
#ifndef ANR_H_
#define ANR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 4 (r06): anr_ingp_hash_field_fwd. ABI 3 (r05): anr_hashgrid_fwd_planes, and the fused
 * field entry points' enc_stride < 0
 * selecting the level-quad-plane layout it writes. */
#define ANR_ABI_VERSION 5

enum anr_dtype { ANR_F32 = 0, ANR_F16 = 1, ANR_BF16 = 2 };

enum anr_status {
  ANR_OK = 0,
  ANR_E_INVALID = -1,     /* bad argument (shape, dtype, unsupported config) */
  ANR_E_LAUNCH = -2,      /* hipLaunchKernel / hipGetLastError reported an error */
  ANR_E_UNSUPPORTED = -3  /* configuration outside the compiled kernel set */
};

typedef void* anr_stream_t; /* hipStream_t */

int anr_abi_version(void);
const char* anr_last_error(void);

/* ------------------------------------------------------------------------------------
 * K1 + K2: stratified ray sampler fused with the HARP2 "horizontal" point preprocessor.
 * ------------------------------------------------------------------------------------
 * anr_prep_params mirrors the closure built by HARP2Dataset.get_point_preprocessor
 * ("horizontal"), datasets/harp2.py:357-388, plus the Instant-NGP remap of
 * pipelines/instant_ngp.py:149,160.
 */
typedef struct {
  int32_t mode;            /* 0: no preprocessing (raw normalized xyz); 1: horizontal */
  int32_t shift_lon;       /* dateline shift, harp2.py:366-370,379-380 */
  int32_t ngp_remap;       /* 1: out = (p+1)/2, out.z /= alt_compress (instant_ngp.py:149,160) */
  int32_t _pad;
  double scale;            /* dataset.scale  (Python float), harp2.py:376 */
  double offset[3];        /* dataset.offset (float64 tensor), harp2.py:376 */
  double lat_min, lat_range, lon_min, lon_range; /* f32 0-dim tensors, harp2.py:361-370 */
  double ray_origin_height;                      /* harp2.py:383 */
  float alt_compress;                            /* config alt_compress_factor */
  float _pad2;
} anr_prep_params;

/* sample_uniform_bins (samplers.py:8-47) [+ preprocess (harp2.py:372-386)].
 *   origin, dir: (B,3) f32; len: (B,) f32; u: (B,N) f32 uniform draws or NULL for bin
 *   midpoints (random=False, samplers.py:37-41); bins: (N+1,) f32 = torch.linspace(0,1,N+1).
 *   Outputs (each nullable): pts (B,N,3) f32 raw sample points (samplers.py:45);
 *   z (B,N) f32 (samplers.py:42); coords (B,N,3) f32 preprocessed (+remapped) points.
 *   z and pts are bit-identical to the reference for identical u (no FMA contraction). */
int anr_sample_uniform_bins(const float* origin, const float* dir, const float* len,
                            const float* u, const float* bins, int64_t B, int32_t N,
                            float* pts, float* z, const anr_prep_params* prep,
                            float* coords, anr_stream_t stream);

/* preprocess_coords applied to arbitrary points (extract path, instant_ngp.py:220-233).
 *   pts (P,3) f32 -> coords (P,3) f32. */
int anr_preprocess_points(const float* pts, int64_t P, const anr_prep_params* prep,
                          float* coords, anr_stream_t stream);

/* Same for f64 points (scripts/extract.py:203-209 passes (xyz - offset) / scale in f64;
 * the whole preprocessor, clip and NGP remap run in f64, the result is rounded to f32
 * once, where tcnn casts the encoder input). */
int anr_preprocess_points_f64(const double* pts, int64_t P, const anr_prep_params* prep,
                              float* coords, anr_stream_t stream);

/* Backward of the preprocessor (the NeRF pipeline back-propagates into the sample points,
 * harp2.py:372-386): d_pts (P,3) f32 WRITTEN = J^T d_coords, J from fp64 forward-mode
 * derivatives of the same formula; clip passes the gradient where -1 <= value <= 1. */
int anr_preprocess_points_bwd(const float* pts, int64_t P, const anr_prep_params* prep,
                              const float* d_coords, float* d_pts, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Ray-batch glue in front of K1 (csrc/gather.hip).
 * ------------------------------------------------------------------------------------
 * anr_gather_rows: dst_k[r] = src_k[idx[r]] for every column k in one launch (the
 * per-field indexing of HARP2Dataset.__getitem__ / __getbatch__, harp2.py:392-420).
 * idx (B,) int64; a column is a row-major array of row_bytes-byte rows (multiple of 4,
 * <= 4096); at most ANR_GATHER_MAX_COLS columns. */
#define ANR_GATHER_MAX_COLS 8
typedef struct {
  const void* src;
  void* dst;
  int64_t row_bytes;
} anr_gather_col;
int anr_gather_rows(const int64_t* idx, int64_t B, int32_t n_cols, const anr_gather_col* cols,
                    anr_stream_t stream);
/* Instant-NGP surface-network input (instant_ngp.py:143,150,173): out (B,5) f32 =
 * [((o + d*len) + 1) / 2 for x, y | d], with torch's f32 rounding of each op.
 * origin, dir (B,3) f32, len (B,) f32. */
int anr_ingp_surface_input(const float* origin, const float* dir, const float* len,
                           int64_t B, float* out, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * K3 / K4: multi-resolution hash-grid encoding (tinycudann.Encoding otype "HashGrid",
 * instant_ngp.py:60-63,163; surface 2-D grid :78-80,173).
 * ------------------------------------------------------------------------------------ */
#define ANR_MAX_LEVELS 32
typedef struct {
  int32_t n_dims;           /* 2 or 3 */
  int32_t n_levels;         /* <= ANR_MAX_LEVELS */
  int32_t n_features;       /* features per level: 1, 2, 4 or 8 */
  int32_t base_resolution;
  float per_level_scale;
  int32_t log2_hashmap_size;
  int64_t n_params;         /* total table entries * n_features (filled by _init) */
  uint32_t offsets[ANR_MAX_LEVELS + 1]; /* first table entry of each level */
  uint32_t resolutions[ANR_MAX_LEVELS];
  float scales[ANR_MAX_LEVELS];
} anr_hashgrid_desc;

/* Fill offsets/resolutions/scales/n_params from the config (tcnn GridEncoding rules). */
int anr_hashgrid_init(anr_hashgrid_desc* d, int32_t n_dims, int32_t n_levels,
                      int32_t n_features, int32_t base_resolution, float per_level_scale,
                      int32_t log2_hashmap_size);

/* Forward: x (M, n_dims) f32 in [0,1] with row stride x_stride; table (n_params) in
 * table_dtype; out (M, n_levels*n_features) written at row stride out_stride
 * (level-major: column l*F+f), out_dtype. Interpolation accumulates in f32. */
int anr_hashgrid_fwd(const anr_hashgrid_desc* d, const float* x, int64_t x_stride,
                     int64_t M, const void* table, int32_t table_dtype, void* out,
                     int32_t out_dtype, int64_t out_stride, anr_stream_t stream);
/* The same, for points that come in runs of run_length spatial neighbours (the altitudes
 * of one extract column, scripts/extract.py:180-211; a ray's samples): the walker's
 * chunks follow the runs (run_length <= 256; 0 = no hint, as anr_hashgrid_fwd). Outputs
 * do not depend on it. */
int anr_hashgrid_fwd_runs(const anr_hashgrid_desc* d, const float* x, int64_t x_stride,
                          int64_t M, int64_t run_length, const void* table,
                          int32_t table_dtype, void* out, int32_t out_dtype,
                          int64_t out_stride, anr_stream_t stream);

/* Kernel generation (test / A-B hook; process-wide; returns the previous mode, or
 * ANR_E_INVALID for an unknown mode; also ANR_HASHGRID_MODE): 0 = default (forward v6
 * branch-free walker -- v1 above 16 levels or past 32-bit buffer offsets -- backward v2
 * four-lanes-per-level), 1 = v1 both, 6 = forward v1 + backward v2 (the r01 default),
 * 7 = mode 0 with the backward's run-time-stride instantiation. */
int anr_hashgrid_force_v1(int32_t mode);
/* Samples per wavefront chunk the v2 backward uses for M points (host-side query: the
 * request counter of tools/hash_requests.py replays the kernel's chunking with it). */
int64_t anr_hashgrid_bwd_chunk(int64_t M);
/* Request-count instrument of the v2 backward: the same launch geometry and walk over
 * the same inputs as anr_hashgrid_bwd (dtable: the gradient buffer that launch would add
 * to -- its addresses decide the 64-B segments; NOT written), adding to *count (one u64,
 * device) the memory-side requests the real launch makes: per flush instruction, the
 * distinct 64-B segments of its active lanes (zero-sum corners skipped as there).
 * bench.py's hash-backward roofline counts its benched step this way. 3-D, 2 features,
 * <= 16 levels; ANR_E_UNSUPPORTED otherwise. */
int anr_hashgrid_bwd_count_requests(const anr_hashgrid_desc* d, const float* x,
                                    int64_t x_stride, int64_t M, const void* dout,
                                    int32_t dout_dtype, int64_t dout_stride,
                                    const float* dtable, unsigned long long* count,
                                    anr_stream_t stream);

/* Backward: dout (M, L*F) (dout_dtype, row stride dout_stride) -> dtable (n_params)
 * f32, ACCUMULATED (caller zeroes). Duplicate corner updates inside a wavefront are
 * pre-summed before the f32 atomics (samples along one ray share cells). */
/* anr_hashgrid_bwd with the field backward's per-tile flags (r05): tile_nz[t] = 0 marks
 * rows [32 t, 32 t + 32) whose dL/dy is zero in every row (anr_ingp_field_bwd_ref16_tiles
 * writes them); the v2 walker neither loads nor walks those rows (their contributions
 * are zero). Same result as anr_hashgrid_bwd for such inputs; shapes outside the tiled
 * walker (not 3-D / 2 features / <= 16 levels, strides other than (3, 32), chunks not a
 * multiple of 32 rows) run anr_hashgrid_bwd and ignore the flags. */
int anr_hashgrid_bwd_tiles(const anr_hashgrid_desc* d, const float* x, int64_t x_stride,
                           int64_t M, const void* dout, int32_t dout_dtype, int64_t dout_stride,
                           float* dtable, const uint8_t* tile_nz, anr_stream_t stream);

/* anr_hashgrid_bwd with per-row bits (ABI 5): bit (m % 32) of row_nz[m / 32] set marks a
 * row m of dout with a nonzero value (anr_ingp_field_bwd_ref16_rows writes them); the v2
 * walker loads and walks only those rows. A row whose bit is clear is taken as zero and
 * need not have been written (anr_ingp_field_bwd_ref16_rows does not write it). Same
 * result as anr_hashgrid_bwd on dout with the clear rows zeroed; shapes other than 3-D /
 * 2 features / 16 levels / strides (3, 32) zero the clear rows IN PLACE (dout is written)
 * and run anr_hashgrid_bwd. Replaces the same call site as anr_hashgrid_bwd (tcnn HashGrid
 * backward, instant_ngp.py:163). */
int anr_hashgrid_bwd_rows(const anr_hashgrid_desc* d, const float* x, int64_t x_stride,
                          int64_t M, void* dout, int32_t dout_dtype, int64_t dout_stride,
                          float* dtable, const uint32_t* row_nz, anr_stream_t stream);

/* Level-quad-plane forward (r05; hashgrid.hip forward v9, one lane per sample): the same
 * features as anr_hashgrid_fwd with f16 output, laid out as planes of four levels: level
 * l, feature f of row m at out[(l / 4) * plane_stride + 8 m + 2 (l % 4) + f]
 * (plane_stride >= 8 M f16 elements, multiple of 8; out 16-byte aligned; a partial last
 * quad is zero-filled). 2 features, <= 16 levels. The fused field kernels read this
 * layout when given enc_stride = -plane_stride. Replaces the same call site as
 * anr_hashgrid_fwd (instant_ngp.py:163, the tcnn Encoding forward). */
int anr_hashgrid_fwd_planes(const anr_hashgrid_desc* d, const float* x, int64_t x_stride,
                            int64_t M, const void* table, int32_t table_dtype, void* out,
                            int64_t plane_stride, anr_stream_t stream);

int anr_hashgrid_bwd(const anr_hashgrid_desc* d, const float* x, int64_t x_stride,
                     int64_t M, const void* dout, int32_t dout_dtype, int64_t dout_stride,
                     float* dtable, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * K5: SphericalHarmonics / Identity encodings (tinycudann Composite members,
 * instant_ngp.py:69-72,165-169; surface :78-80).
 * ------------------------------------------------------------------------------------ */
/* SH of degree `degree` (1..4 -> degree^2 outputs) of x in [0,1]^3 remapped to 2x-1. */
int anr_sh_fwd(int32_t degree, const float* x, int64_t x_stride, int64_t M, void* out,
               int32_t out_dtype, int64_t out_stride, anr_stream_t stream);
/* d(SH)/dx: dout (M, degree^2) -> dx (M,3) f32, ACCUMULATED into dx. */
int anr_sh_bwd(int32_t degree, const float* x, int64_t x_stride, int64_t M,
               const void* dout, int32_t dout_dtype, int64_t dout_stride, float* dx,
               int64_t dx_stride, anr_stream_t stream);
/* Identity: out[:, :n] = x[:, :n] (dtype conversion). x may be f32 or f16. */
int anr_identity(const void* x, int32_t x_dtype, int64_t x_stride, int64_t M, int32_t n,
                 void* out, int32_t out_dtype, int64_t out_stride, anr_stream_t stream);
/* Fill out[:, :n] with a constant (tcnn pads encodings with 1.0). */
int anr_fill_cols(void* out, int32_t out_dtype, int64_t out_stride, int64_t M, int32_t n,
                  float value, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * K6 / K7: fully-fused MLP (tinycudann.Network otype "FullyFusedMLP",
 * instant_ngp.py:64-68,73-77,81-85). Bias-free; ReLU hidden activation; output
 * activation None or ReLU. Weight layout: layer k is a row-major (out_k, in_k) matrix,
 * layers concatenated; in_0 = n_input_padded, out_last = n_output_padded.
 * Input columns [n_input, n_input_padded) are read as 1.0 (tcnn encoding padding).
 * ------------------------------------------------------------------------------------ */
enum anr_activation { ANR_ACT_NONE = 0, ANR_ACT_RELU = 1 };
typedef struct {
  int32_t n_input, n_input_padded;   /* padded to a multiple of 16 */
  int32_t n_output, n_output_padded; /* padded to a multiple of 16 */
  int32_t width;                     /* 16, 32, 64 or 128 */
  int32_t n_hidden_layers;           /* >= 1 */
  int32_t activation;                /* ANR_ACT_RELU */
  int32_t output_activation;         /* ANR_ACT_NONE or ANR_ACT_RELU */
} anr_mlp_desc;

int64_t anr_mlp_n_params(const anr_mlp_desc* d);
/* Force the generic (shape-agnostic) MLP kernels instead of the compile-time specialised
 * ones (on != 0). Test hook; process-wide. Returns the previous setting. */
int anr_mlp_force_generic(int32_t on);
/* Forward. precision = ANR_F16 (f16 MFMA, f32 accumulate; params_f16 used) or ANR_F32
 * (f32 MFMA, exact f32; params_f32 used). in: (M, n_input) in_dtype; out: (M, n_output)
 * out_dtype. */
int anr_mlp_fwd(const anr_mlp_desc* d, int32_t precision, const void* params,
                const void* in, int32_t in_dtype, int64_t in_stride, int64_t M, void* out,
                int32_t out_dtype, int64_t out_stride, anr_stream_t stream);
/* Backward (recomputes the forward activations on chip). dout: (M, n_output);
 * din (nullable): (M, n_input) written (not accumulated); dparams: f32, ACCUMULATED. */
int anr_mlp_bwd(const anr_mlp_desc* d, int32_t precision, const void* params,
                const void* in, int32_t in_dtype, int64_t in_stride, int64_t M,
                const void* dout, int32_t dout_dtype, int64_t dout_stride, void* din,
                int32_t din_dtype, int64_t din_stride, float* dparams,
                anr_stream_t stream);
/* Scratch bytes anr_mlp_bwd_ws can use for M rows (0: it would not use any). With it the
 * specialised backward stores one dW row per wavefront and sums them in a fixed order
 * instead of adding with float atomics (small batches, e.g. the per-ray surface
 * network: deterministic and without the atomics' contention). */
int64_t anr_mlp_bwd_workspace_bytes(const anr_mlp_desc* d, int64_t M);
/* anr_mlp_bwd with a device workspace (f32-aligned, workspace_bytes long; may be null or
 * smaller than anr_mlp_bwd_workspace_bytes, then the atomics path runs). */
int anr_mlp_bwd_ws(const anr_mlp_desc* d, int32_t precision, const void* params,
                   const void* in, int32_t in_dtype, int64_t in_stride, int64_t M,
                   const void* dout, int32_t dout_dtype, int64_t dout_stride, void* din,
                   int32_t din_dtype, int64_t din_stride, float* dparams, void* workspace,
                   int64_t workspace_bytes, anr_stream_t stream);

/* Instant-NGP dir MLP with the dir encoding fused into its input
 * (instant_ngp.py:165-171): row r of the network input is
 * [SH degree 2 of dirs[r / n_per_ray] | pos_out[r, 1:16] | 1.0 padding] (n_input = 19,
 * padded 32), so the encoded tensor is never materialised.
 *   pos_out (M, >=16) f32 (pos_mlp output, row stride pos_stride); dirs (M/n_per_ray, 3)
 *   f32; color (M, n_output) out_dtype. Widths 32/64, 1-2 hidden layers. */
int anr_ingp_dir_mlp_fwd(const anr_mlp_desc* d, int32_t precision, const void* params,
                         const float* pos_out, int64_t pos_stride, const float* dirs,
                         int64_t n_per_ray, int64_t M, void* color, int32_t out_dtype,
                         int64_t out_stride, anr_stream_t stream);
/* Backward: d_color (M, n_output) f32, d_sigma (M,) f32 (nullable) -> d_pos_out (M, 16)
 * f32 WRITTEN: column 0 = d_sigma * [pos_out[:,0] > 0] (density ReLU, instant_ngp.py:184),
 * columns 1..15 = dL/d(pos_out[:, 1:16]); dparams f32 ACCUMULATED. */
int anr_ingp_dir_mlp_bwd(const anr_mlp_desc* d, int32_t precision, const void* params,
                         const float* pos_out, int64_t pos_stride, const float* dirs,
                         int64_t n_per_ray, int64_t M, const float* d_color,
                         int64_t d_color_stride, const float* d_sigma, float* d_pos_out,
                         int64_t d_pos_stride, float* dparams, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * K6 + K7 fused: the Instant-NGP radiance field after the hash encoding, one kernel each
 * way (replaces pos_mlp -> dir_encoder -> dir_mlp -> relu at instant_ngp.py:163-184).
 * ------------------------------------------------------------------------------------
 * Supported pairs: pos 32 -> W -> 16 (1 hidden layer, no output activation), dir 19 -> W
 * (1 or 2 hidden layers) -> n_output <= 16, W in {32, 64}.
 * mma_dtype: ANR_F16 (the reference's tcnn precision: f16 operands, f32 accumulation) or
 * ANR_BF16 (BASELINE configs[4], beyond the reference: bf16 operands over the same f16
 * hash features, f32 accumulation; no gradient scaling). Pack, forward and backward of one
 * network must use the same mma_dtype.
 * Weights: anr_ingp_field_pack converts the f32 master parameters of both networks
 * (tcnn layout) into one 16-bit buffer of anr_ingp_field_packed_size elements (MFMA
 * fragment order); run it after every optimizer step.
 * enc (every entry point below): f16 hash features, enc_stride >= 32 (multiple of 8) for
 *   the row layout (M, enc_stride) with 16-byte aligned rows, or enc_stride = -P for the
 *   level-quad planes of anr_hashgrid_fwd_planes (P >= 8 M, multiple of 8).
 * Forward: enc, dirs (M/n_per_ray, 3) f32 ->
 *   sigma (M,) f32 = relu(pos_out[:,0]), color (M, n_output) f32 = relu(dir_mlp(...)).
 * Backward: d_sigma (M,) f32 (nullable), d_color (M, n_output) f32 -> d_enc (M, 32) f32
 *   WRITTEN; g_pos / g_dir f32 parameter gradients ACCUMULATED. `workspace` is caller-
 *   owned device memory of at least anr_ingp_field_bwd_workspace_bytes(pos, dir,
 *   mma_dtype, M) bytes (per-wavefront f16 gradient maxima; 0 bytes for bf16, then it may
 *   be NULL); it must not be shared with a concurrent backward launch. */
int anr_ingp_field_supported(const anr_mlp_desc* pos, const anr_mlp_desc* dir);
int64_t anr_ingp_field_packed_size(const anr_mlp_desc* pos, const anr_mlp_desc* dir);
/* f16 gradient scale target of the backward (max |dL/dout| per wavefront -> 2^v);
 * returns the previous value. Test hook; process-wide. */
int anr_ingp_field_set_grad_scale(int32_t log2_target);
/* Forward kernel form: 1 = the uniform-tile form wherever the shapes allow it (default:
 * dense rows, samples_per_ray a multiple of 16, 4 colour outputs, 16-byte aligned colour
 * rows; one scalar direction load per 16-row tile, branch-free output stores), 0 = always
 * the general form. Same math and bit-identical results. Test / A-B hook; process-wide;
 * other values keep the current mode. Returns the previous mode. */
int anr_ingp_field_force_fwd(int32_t mode);
int64_t anr_ingp_field_bwd_workspace_bytes(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                           int32_t mma_dtype, int64_t M);
int anr_ingp_field_pack(const anr_mlp_desc* pos, const anr_mlp_desc* dir, int32_t mma_dtype,
                        const float* pos_params, const float* dir_params, void* packed,
                        anr_stream_t stream);
int anr_ingp_field_fwd(const anr_mlp_desc* pos, const anr_mlp_desc* dir, int32_t mma_dtype,
                       const void* packed, const void* enc, int64_t enc_stride,
                       const float* dirs, int64_t n_per_ray, int64_t M, float* sigma,
                       float* color, int64_t color_stride, anr_stream_t stream);
/* Hash-grid forward + field forward in one kernel (ABI 4, r06): the level-quad planes of
 * anr_hashgrid_fwd_planes (written for the backward: planes, plane_stride >= 8 M f16
 * elements) and sigma / color of anr_ingp_field_fwd, bit-identical to those two calls, with
 * the planes never re-read. Replaces the same call sites (instant_ngp.py:163-171: the tcnn
 * Encoding forward, pos_mlp, dir_encoder, dir_mlp). Shapes: 3-D f16 hash grid of 16 levels
 * x 2 features (x: (M, 3) f32 rows), a supported field pair with 4 colour outputs, samples
 * per ray a multiple of 64, 16-byte aligned planes / packed / colour rows;
 * ANR_E_UNSUPPORTED otherwise (the two calls then serve). */
int anr_ingp_hash_field_fwd(const anr_hashgrid_desc* grid, const float* x, int64_t M,
                            const void* table, int32_t table_dtype, void* planes,
                            int64_t plane_stride, const anr_mlp_desc* pos,
                            const anr_mlp_desc* dir, int32_t mma_dtype, const void* packed,
                            const float* dirs, int64_t n_per_ray, float* sigma, float* color,
                            int64_t color_stride, anr_stream_t stream);
/* Density only: sigma[r] = relu(pos_mlp(enc[r])[0]) (f32), bit-identical to
 * anr_ingp_field_fwd's sigma, without the dir MLP -- the extract loop
 * (scripts/extract.py:203-209 -> instant_ngp.py:208-247 reads only the extinction) and the
 * occupancy grid. Same descriptors and packed weights as anr_ingp_field_fwd. */
int anr_ingp_field_density(const anr_mlp_desc* pos, const anr_mlp_desc* dir, int32_t mma_dtype,
                           const void* packed, const void* enc, int64_t enc_stride, int64_t M,
                           float* sigma, anr_stream_t stream);
int anr_ingp_field_bwd(const anr_mlp_desc* pos, const anr_mlp_desc* dir, int32_t mma_dtype,
                       const void* packed, const void* enc, int64_t enc_stride,
                       const float* dirs, int64_t n_per_ray, int64_t M, const float* d_sigma,
                       const float* d_color, int64_t d_color_stride, float* d_enc,
                       int64_t d_enc_stride, float* g_pos, float* g_dir, void* workspace,
                       int64_t workspace_bytes, anr_stream_t stream);

/* The same kernels over occupancy-compacted samples (anr_occupancy_compact): row r of
 * enc / d_enc is dense sample rows[r] (int32, ray-major index < n_rays * n_per_ray) of
 * sigma, color, d_sigma, d_color, whose ray is rows[r] / n_per_ray. The forward writes
 * only the listed dense rows (the caller zero-fills the rest: culled samples have
 * sigma = 0), the backward reads dL/d(sigma, color) at those rows. */
int anr_ingp_field_fwd_rows(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                            int32_t mma_dtype, const void* packed, const void* enc,
                            int64_t enc_stride, const float* dirs, int64_t n_per_ray,
                            int64_t M, const int32_t* rows, float* sigma, float* color,
                            int64_t color_stride, anr_stream_t stream);
int anr_ingp_field_bwd_rows(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                            int32_t mma_dtype, const void* packed, const void* enc,
                            int64_t enc_stride, const float* dirs, int64_t n_per_ray,
                            int64_t M, const int32_t* rows, const float* d_sigma,
                            const float* d_color, int64_t d_color_stride, float* d_enc,
                            int64_t d_enc_stride, float* g_pos, float* g_dir, void* workspace,
                            int64_t workspace_bytes, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Occupancy-grid sample culling (beyond the reference: BASELINE configs[4], SURVEY §8
 * f3; csrc/occupancy.hip). occ: gx*gy*gz bytes (x fastest), nonzero = occupied, over the
 * hash-grid domain [0,1] x [0,1] x [0, 1/zmul]. coords (M,3) f32 ray-major.
 * anr_occupancy_count writes counts[anr_occupancy_n_blocks(M)] (int32, kept samples per
 * block of 1024); the caller forms offsets = exclusive scan (int64) and the total K;
 * anr_occupancy_compact writes rows (K,) int32 (kept sample indices, ascending) and
 * coords_out (K,3). ------------------------------------------------------------------ */
int64_t anr_occupancy_n_blocks(int64_t M);
int anr_occupancy_count(const float* coords, int64_t M, const uint8_t* occ, int32_t gx,
                        int32_t gy, int32_t gz, float zmul, int32_t* counts,
                        anr_stream_t stream);
int anr_occupancy_compact(const float* coords, int64_t M, const uint8_t* occ, int32_t gx,
                          int32_t gy, int32_t gz, float zmul, const int64_t* offsets,
                          int32_t* rows, float* coords_out, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * NeRF path (configs/nerf.json): positional encoding (encoders.py:4-28) and the
 * hierarchical pdf sampler (samplers.py:50-103), forward and backward.
 * ------------------------------------------------------------------------------------ */
#define ANR_POSENC_MAX_DIMS 8
typedef struct {
  int32_t n_dims;       /* input coordinates per row */
  int32_t interleaved;  /* 1: int L (per coordinate [sin f0, cos f0, sin f1, ...]),
                           0: list L (per coordinate [sin f0..f(L-1), cos f0..f(L-1)]) */
  int32_t L[ANR_POSENC_MAX_DIMS]; /* frequencies per coordinate (interleaved: L[0] for all) */
} anr_posenc_desc;
/* Output width (2 * sum of L), or -1 for a bad descriptor. */
int32_t anr_posenc_width(const anr_posenc_desc* d);
/* out (P, >= width) f32 row r = encoding of x row r / rows_per_x (x (P/rows_per_x, n_dims)
 * f32); frequencies (2^l * pi) in f32 times x in f32, sinf/cosf. */
int anr_posenc_fwd(const anr_posenc_desc* d, const float* x, int64_t rows_per_x, int64_t P,
                   float* out, int64_t out_stride, anr_stream_t stream);
/* dx (P, n_dims) f32 WRITTEN from dL/dout (P, >= width). */
int anr_posenc_bwd(const anr_posenc_desc* d, const float* x, int64_t P, const float* dout,
                   int64_t dout_stride, float* dx, anr_stream_t stream);
/* AtmoNeRF Linear+ReLU backward (models/nerf.py:48-93; replaces autograd's
 * threshold_backward + bias-gradient reduction): g_out = g where y > 0 else 0, for
 * contiguous (M, C) f32 g, y, g_out (C a multiple of 4, <= 1024, 16-byte aligned); and
 * partial (n_parts, C) f32 WRITTEN with the column sums of g_out over n_parts row blocks
 * (fixed order; the bias gradient is their sum; M = 0 writes zeros, g/y/g_out may be
 * NULL then). */
int anr_relu_bwd_colsum(const float* g, const float* y, int64_t M, int32_t C, float* g_out,
                        float* partial, int32_t n_parts, anr_stream_t stream);
/* AtmoNeRF dense layers on the f32 matrix cores (csrc/nerf_mlp.hip). They replace the
 * nn.Linear / torch.cat / F.relu calls of src/atmonr/models/nerf.py:48-93 and their
 * autograd backward. Operands are row-major f32 with 16-byte-aligned rows: every leading
 * dimension and segment width is a multiple of 4.
 *
 * Forward: y (M x n, row stride ldy >= round_up(n, 4)) = [a1 | a2] W^T + bias, then ReLU
 * if relu != 0. Columns n .. round_up(n, 4) come out zero.
 *   a1 is M x q1 and a2 is M x q2 (q2 = 0: none; q1 % 16 == 0 when q2 > 0). They are the
 *   fc6 skip and fc10 direction concats, read in place.
 *   W is n x (q1+q2), as nn.Linear.weight. bias is nullable.
 *   relu_bits is nullable. If given, it receives M x ceil(n/64) 64-bit words, one bit
 *   per element: y[m][64w + 16j + 4g + r] > 0 is bit 16g + 4j + r of word w of row m.
 *   That is the ReLU mask for the layer's backward, 32x smaller than the activations. */
int anr_nerf_linear_fwd(const float* a1, int64_t lda1, int32_t q1, const float* a2,
                        int64_t lda2, int32_t q2, int64_t M, const float* w, int32_t n,
                        const float* bias, int32_t relu, float* y, int64_t ldy,
                        uint64_t* relu_bits, anr_stream_t stream);
/* Input gradient: [dx1 | dx2] (M x (p1+p2)) = g (M x n) W, with wt = W^T
 * ((p1+p2) x n, row stride ldwt).
 *   p1 % 4 == 0 and p2 % 4 == 0.
 *   If n % 4 != 0, g's and wt's columns n .. round_up(n, 4) must exist and be zero.
 *   dx1 (first p1 columns) is zeroed where the bit in mask_bits is clear. mask_bits is
 *   the relu_bits of the forward that produced the input, M x ceil(p1/64) words, or
 *   NULL for no mask. This is the ReLU backward of the layer below.
 *   dx2 (last p2 columns) is written, or added to if acc2 != 0. */
int anr_nerf_linear_dx(const float* g, int64_t ldg, int64_t M, int32_t n, const float* wt,
                       int64_t ldwt, int32_t p1, int32_t p2, const uint64_t* mask_bits,
                       float* dx1, int64_t ldx1, float* dx2, int64_t ldx2, int32_t acc2,
                       anr_stream_t stream);
/* Parameter gradients, ACCUMULATED: dw (n x (q1+q2), contiguous) += g^T [a1 | a2], and
 * db (n, nullable) += the column sums of g.
 *   g's columns n .. round_up(n, 4) must be zero.
 *   M is split over blocks into f32 partials in ws (anr_nerf_linear_dw_workspace bytes,
 *   16-byte aligned), summed in a fixed order: the result is deterministic. */
int64_t anr_nerf_linear_dw_workspace(int64_t M, int32_t n, int32_t k);
int anr_nerf_linear_dw(const float* g, int64_t ldg, int64_t M, int32_t n, const float* a1,
                       int64_t lda1, int32_t q1, const float* a2, int64_t lda2, int32_t q2,
                       float* dw, float* db, void* ws, int64_t ws_bytes, anr_stream_t stream);
/* sample_pdf forward, one wavefront per ray (3 <= Nc <= 64, 1 <= Nf <= 256).
 *   weights: coarse render weights, element (b, j) at b*w_ray_stride + j*w_sample_stride
 *   (channel 0 of (B, Nc, S)); z_coarse (B,Nc) f32 ascending; u (B,Nf) f32 draws.
 *   Outputs: z (B, Nc+Nf) sorted, pts (B, Nc+Nf, 3) = o + d*z (nullable), src (B, Nc+Nf)
 *   int32 (source of each sorted value: < Nc coarse, else Nc + sample), inds (B,Nf) int32
 *   = searchsorted(cdf, u, right=True), cdf (B, Nc-1) f32 (saved for the backward). */
int anr_sample_pdf_fwd(const float* weights, int64_t w_ray_stride, int32_t w_sample_stride,
                       const float* z_coarse, const float* u, const float* origin,
                       const float* dir, int64_t B, int32_t Nc, int32_t Nf, float* z,
                       float* pts, int32_t* src, int32_t* inds, float* cdf,
                       anr_stream_t stream);
/* Backward into the weights through t_in_bin (bin width detached): d_z (B, Nc+Nf) and/or
 * d_pts (B, Nc+Nf, 3) (each nullable) -> d_weights channel 0 WRITTEN (rest untouched). */
int anr_sample_pdf_bwd(const float* weights, int64_t w_ray_stride, int32_t w_sample_stride,
                       const float* z_coarse, const float* u, const float* dir,
                       const int32_t* src, const int32_t* inds, const float* cdf, int64_t B,
                       int32_t Nc, int32_t Nf, const float* d_z, const float* d_pts,
                       float* d_weights, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * K8: transmittance / alpha-composite integrator, render + render_with_surface
 * (graphics_utils.py:6-77), one wavefront per ray with shuffle prefix scans.
 * ------------------------------------------------------------------------------------
 * z (B,N) f32 multiplied by z_scale in f32 (instant_ngp.py:188 z_vals*(scale/1000));
 * color (B,N,C) and sigma (B,N,S) (S = 1 or C) in io_dtype; color_surf (B,C) or NULL
 * (plain render). Outputs (nullable unless noted): color_map (B,C) [required],
 * color_map_atmo, color_map_surf (B,C), weights (B,N,S), alpha (B,N,S); io_dtype.
 * Arithmetic is f32 internally. */
int anr_composite_fwd(const float* z, float z_scale, const void* color, const void* sigma,
                      const void* color_surf, int32_t io_dtype, int64_t B, int32_t N,
                      int32_t C, int32_t S, void* color_map, void* color_map_atmo,
                      void* color_map_surf, void* weights, void* alpha,
                      anr_stream_t stream);
/* Use the generic kernels instead of the register-blocked ones (C = 4, S in {1,4},
 * N/64 in {1,2,3,4,8,16}). Test hook; process-wide. Returns the previous setting. */
int anr_composite_force_generic(int32_t on);
/* Backward. Gradients in (nullable; io_dtype): d_color_map, d_atmo, d_surf (B,C),
 * d_weights (B,N,S), d_alpha (B,N,S). Outputs (nullable): d_color (B,N,C),
 * d_sigma (B,N,S), d_color_surf (B,C) (io_dtype), d_z (B,N) f32 (dL/dz before scaling
 * by z_scale is applied, i.e. w.r.t. the unscaled z input). */
int anr_composite_bwd(const float* z, float z_scale, const void* color, const void* sigma,
                      const void* color_surf, int32_t io_dtype, int64_t B, int32_t N,
                      int32_t C, int32_t S, const void* d_color_map, const void* d_atmo,
                      const void* d_surf, const void* d_weights, const void* d_alpha,
                      void* d_color, void* d_sigma, void* d_color_surf, float* d_z,
                      anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * K9: losses (losses.py:5-33) on pred = take_along_dim(color_map, irgb_idx)
 * (instant_ngp.py:259-263). Writes the scalar loss (f32) and dL/dcolor_map (B,C).
 * ------------------------------------------------------------------------------------ */
enum anr_loss { ANR_LOSS_DARK = 0, ANR_LOSS_HDR = 1, ANR_LOSS_L1 = 2,
                ANR_LOSS_L1_PLUS_HDR = 3, ANR_LOSS_MSE = 4, ANR_LOSS_MSE_PLUS_HDR = 5 };
/* color_map (B,C) pred_dtype, irgb_idx (B,) int64, gt (B,) f32. loss_out: 1 f32.
 * grad_out (nullable): (B,C) pred_dtype, dL/dcolor_map scaled by grad_scale.
 * workspace: >= anr_loss_workspace_bytes(B) bytes (f32 partial sums). */
int64_t anr_loss_workspace_bytes(int64_t B);
int anr_loss_fwd_bwd(int32_t loss_type, const void* color_map, int32_t pred_dtype,
                     int32_t C, const int64_t* irgb_idx, const float* gt, int64_t B,
                     float max_i, float grad_scale, float* loss_out, void* grad_out,
                     void* workspace, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Reference numerics (csrc/ref16.hip; opt-in, InstantNGPPipeline(numerics="reference")).
 * The reference's Instant-NGP composite and loss run as chains of torch f16 ops on f16
 * tinycudann outputs (graphics_utils.py:28-76, instant_ngp.py:259-263, losses.py:5-33),
 * and tcnn's backward is loss-scaled f16 (tinycudann/modules.py, loss scale 128). These
 * entry points reproduce those roundings op by op (oracle/ref_f16.py is the restatement;
 * torch's CUDA accumulation: f16 accumulator in cumprod / cumsum, f32 in sum / prod).
 * R rays per wavefront (2, or 1 below 8,192 rays): lane-parallel per-sample ops, the order-sensitive
 * accumulations as serial scans, lane r for ray r.
 * ------------------------------------------------------------------------------------
 * Forward: z (B,N) f32 times z_scale in f32 then rounded to f16; color (B,N,C), sigma
 * (B,N,1), color_surf (B,C) (nullable) in in_dtype, rounded to f16 on load. Outputs f16:
 * color_map (B,C) [required], color_map_atmo, color_map_surf (B,C), weights, alpha
 * (B,N,1) (nullable); color16 (B,N,C), sigma16 (B,N,1) (nullable): the f16-rounded
 * inputs, i.e. tcnn's f16 outputs the reference's forward returns (instant_ngp.py:194-206).
 * Replaces render_with_surface (graphics_utils.py:52-77) at instant_ngp.py:187-192 in that
 * mode. */
/* Rays per wavefront of the two composite kernels: 1, 2, 4 or 8, or 0 for the default
 * (2 from 8,192 rays up, else 1; or ANR_REF16_R); halved while R * C > 64. Outputs do
 * not depend on it. */
int anr_composite_ref16_set_rays(int32_t rays_per_wave);
int anr_composite_ref16_fwd(const float* z, float z_scale, const void* color,
                            const void* sigma, const void* color_surf, int32_t in_dtype,
                            int64_t B, int32_t N, int32_t C, void* color_map,
                            void* color_map_atmo, void* color_map_surf, void* weights,
                            void* alpha, void* color16, void* sigma16, anr_stream_t stream);
/* Backward from dL/dcolor_map (B,C) f16 (torch's f16 autograd of the forward).
 * d_color (B,N,C), d_sigma (B,N,1) [required; also scratch for the cumprod outputs] and
 * d_color_surf (B,C) (nullable) in out_dtype, holding f16 values. zero_rays: one int32
 * (device), incremented per ray in which alpha rounded to exactly 1 (torch's zero-input
 * backward branches, not reproduced: that ray's gradients are 0). */
int anr_composite_ref16_bwd(const float* z, float z_scale, const void* color,
                            const void* sigma, const void* color_surf, int32_t in_dtype,
                            int64_t B, int32_t N, int32_t C, const void* d_color_map,
                            void* d_color, void* d_sigma, void* d_color_surf,
                            int32_t out_dtype, int32_t* zero_rays, anr_stream_t stream);
/* Loss in f16 ops: color_map (B,C) f16, gt (B,) f32 (cast to f16 as instant_ngp.py:262),
 * loss_out: 1 f32 holding the f16 loss value, grad_out (B,C) f16 (nullable),
 * workspace >= anr_loss_workspace_bytes(B). */
int anr_loss_ref16_fwd_bwd(int32_t loss_type, const void* color_map, int32_t C,
                           const int64_t* irgb_idx, const float* gt, int64_t B, float max_i,
                           float* loss_out, void* grad_out, void* workspace,
                           anr_stream_t stream);
/* tcnn's parameter gradient of an f16 module at loss scale s: g <- f16(f16(g*s)/s), in
 * place over n f32 values (the value tinycudann/modules.py hands to torch). */
int anr_grad_quantize_f16(float* grad, int64_t n, float loss_scale, anr_stream_t stream);
/* The fused field backward (anr_ingp_field_bwd) with tcnn's backward semantics: fixed
 * f16 gradient scale loss_scale (128), ReLU masks on the f16 outputs, and the
 * module-boundary gradients of the reference (dir_mlp -> dir_encoder -> pos_out, pos_mlp
 * -> pos_encoder) rounded as f16(f16(g_scaled)/loss_scale). f16 networks, dense rows; no
 * workspace. */
int anr_ingp_field_bwd_ref16(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                             const void* packed, const void* enc, int64_t enc_stride,
                             const float* dirs, int64_t n_per_ray, int64_t M,
                             const float* d_sigma, const float* d_color,
                             int64_t d_color_stride, float* d_enc, int64_t d_enc_stride,
                             float* g_pos, float* g_dir, float loss_scale,
                             anr_stream_t stream);
/* anr_ingp_field_bwd_ref16 that also writes, per 32-row tile t of the M rows, tile_nz[t]
 * = 1 if any row of the tile had a nonzero dL/dcolor or dL/dsigma (the tile was walked)
 * and 0 otherwise (skipped: its dL/denc rows are written as 0). tile_nz: ceil(M / 32)
 * bytes of device memory, for anr_hashgrid_bwd_tiles. */
int anr_ingp_field_bwd_ref16_tiles(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                   const void* packed, const void* enc, int64_t enc_stride,
                                   const float* dirs, int64_t n_per_ray, int64_t M,
                                   const float* d_sigma, const float* d_color,
                                   int64_t d_color_stride, float* d_enc, int64_t d_enc_stride,
                                   float* g_pos, float* g_dir, float loss_scale,
                                   uint8_t* tile_nz, anr_stream_t stream);
/* anr_ingp_field_bwd_ref16 writing dL/denc as f16 rows (d_enc_h: (M, >= 32) halves, row
 * stride d_enc_stride, 8-byte aligned; the reference numerics' dL/denc values are f16
 * numbers, tinycudann/modules.py casts them to the f16 input's dtype, so the rows hold them
 * exactly) and one bit per row in row_nz (ceil(M / 32) words): bit (m % 32) of word m / 32
 * set iff row m has a nonzero value; every row is written (skipping the clear ones made
 * partial 128-B line writes: slower, profiles/r06_field_bwd_skip_clear_rows_ab.log). For
 * anr_hashgrid_bwd_rows (ABI 5).
 * workspace (nullable, 256-byte aligned, anr_ingp_field_bwd_ref16_rows_workspace_bytes(M)
 * bytes): with it the backward runs as a pos pass over the tiles whose dL/dcolor is zero in
 * every row (the dir network adds exactly 0 there) and a full pass over the others, listed
 * in the workspace by the first; the same results. Without it, one kernel does both. */
int64_t anr_ingp_field_bwd_ref16_rows_workspace_bytes(int64_t M);
int anr_ingp_field_bwd_ref16_rows(const anr_mlp_desc* pos, const anr_mlp_desc* dir,
                                  const void* packed, const void* enc, int64_t enc_stride,
                                  const float* dirs, int64_t n_per_ray, int64_t M,
                                  const float* d_sigma, const float* d_color,
                                  int64_t d_color_stride, void* d_enc_h, int64_t d_enc_stride,
                                  float* g_pos, float* g_dir, float loss_scale,
                                  uint32_t* row_nz, void* workspace, int64_t workspace_bytes,
                                  anr_stream_t stream);
/* anr_mlp_bwd_ws in f16 with tcnn's fixed loss scale: dL/dinput written as
 * f16(f16(g_scaled)/loss_scale). Specialised (fused) MLP shapes only. */
int anr_mlp_bwd_ref16(const anr_mlp_desc* d, const void* params, const void* in,
                      int32_t in_dtype, int64_t in_stride, int64_t M, const void* dout,
                      int32_t dout_dtype, int64_t dout_stride, void* din, int32_t din_dtype,
                      int64_t din_stride, float* dparams, void* workspace,
                      int64_t workspace_bytes, float loss_scale, anr_stream_t stream);

/* ------------------------------------------------------------------------------------
 * K10: fused AdamW (torch.optim.AdamW, instant_ngp.py:120-126; Adam nerf.py:70 is
 * weight_decay = 0, decoupled = 0) over one flat f32 parameter buffer.
 * ------------------------------------------------------------------------------------
 * step is the 1-based step count after increment. params_f16 (nullable) receives an
 * f16 shadow copy of the updated params (the tcnn forward precision). If zero_grad,
 * grad is zeroed after use (fused optimizer.zero_grad). decoupled = 1: AdamW
 * (p *= 1 - lr*wd); decoupled = 0: Adam with L2 (g += wd*p). */
int anr_adam_step(float* params, float* grad, float* exp_avg, float* exp_avg_sq,
                  void* params_f16, int64_t n, float lr, float beta1, float beta2,
                  float eps, float weight_decay, int32_t decoupled, int64_t step,
                  int32_t zero_grad, anr_stream_t stream);

/* Every tensor of one optimizer step (torch.optim.AdamW.step over all param groups,
 * instant_ngp.py:120-126 / trainer.py:105) in one launch: per tensor its own lr,
 * weight_decay and step count; beta1/2, eps, decoupled and zero_grad shared. Tensors
 * travel in the kernel arguments, ANR_ADAM_MAX_TENSORS per launch (more: several
 * launches, same stream). Same arithmetic as anr_adam_step. */
#define ANR_ADAM_MAX_TENSORS 16
typedef struct anr_adam_tensor {
  float* params;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  void* params_f16; /* nullable f16 shadow */
  int64_t n;
  float lr;
  float weight_decay;
  int64_t step;
  /* > 0: the gradient is first rounded as tinycudann's f16 parameter gradient at this
   * loss scale, g <- f16(f16(g * s) / s) (anr_grad_quantize_f16, fused into the update's
   * read of g; reference numerics with a deferred quantisation). 0: g as it is. */
  float grad_quant;
} anr_adam_tensor;
int anr_adam_step_multi(const anr_adam_tensor* tensors, int32_t n_tensors, float beta1,
                        float beta2, float eps, int32_t decoupled, int32_t zero_grad,
                        anr_stream_t stream);

/* anr_adam_step_multi with the step count and the learning rates in DEVICE memory, so
 * that one captured launch serves every replay of a hipGraph of the train step
 * (torch.optim.AdamW(capturable=True) keeps its step on the device for the same reason;
 * trainer.py:105 is the call site). Per call: *d_step += 1 on the device, then every
 * tensor t is updated with step = *d_step and lr = d_lr[t] (the descriptors' lr and
 * step fields are ignored; weight_decay and the pointers are taken from them at the
 * call). d_scratch: 3 * ANR_ADAM_DEV_MAX_TENSORS floats of caller-owned device memory
 * (the per-tensor bias-corrected scalars). At most ANR_ADAM_DEV_MAX_TENSORS tensors.
 * Same arithmetic as anr_adam_step_multi (bias corrections in double). */
#define ANR_ADAM_DEV_MAX_TENSORS 64
int anr_adam_step_multi_dev(const anr_adam_tensor* tensors, int32_t n_tensors, float beta1,
                            float beta2, float eps, int32_t decoupled, int32_t zero_grad,
                            int64_t* d_step, const float* d_lr, float* d_scratch,
                            anr_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* ANR_H_ */
